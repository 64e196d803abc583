# Round 6: side-pass grid cap -- bit identity (cap tests, pipelined submit vs align_batch), the side-cost A/B with
# capped real side passes, then the bench line (default cap 512).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06l
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_split_gpu.py tests/test_pipeline_gpu.py -x -q --timeout 300 --timeout-method thread -k "grid_cap or submit_matches or held_for_next" > $O/tests.log 2>&1 || { echo "TESTS FAIL"; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 500 python scripts/side_cost.py --mode ab --replay profiles/r06/side_replay.json --steps 20 --rounds 3 > $O/side_ab.json 2> $O/side_ab.txt || { echo "SIDE AB FAIL"; tail -20 $O/side_ab.txt; exit 1; }
grep -v amdgpu.ids $O/side_ab.txt
timeout -k 10 500 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { echo "BENCH FAIL"; tail -20 $O/bench.err; exit 1; }
python -c "import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]); print(round(d['value']), round(d['ms_per_step'],3), d['step_breakdown']['side_stream_cost_ms'], d['sustained']['last_window_ms_per_step'], d['config4']['value'], d['config5']['value'])"
echo ALLOK
