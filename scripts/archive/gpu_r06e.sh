# Round 6: the stream-order word (tests + bench A/B against the event wait, host CPU per thread) and the side-stream
# decomposition with the fixed occupancy replay.  Outputs under gpurun_out/r06e.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06e
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_pipeline_gpu.py tests/test_rccl_gpu.py tests/test_api_gpu.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo "TESTS FAIL"; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for r in 1 2; do
  for m in event word; do
    timeout -k 10 300 python bench.py --steps 40 --warmup 5 --no-cpu-baseline --no-extra-configs --sustained-s 0 --stream-sync $m > $O/bench_${m}_$r.json 2> $O/bench_${m}_$r.err || { echo "BENCH $m FAIL"; tail -20 $O/bench_${m}_$r.err; exit 1; }
    python -c "import json; d=json.loads(open('$O/bench_${m}_$r.json').read().strip().splitlines()[-1]); print('$m', round(d['ms_per_step'],3), d['host_cpu']['process_cpu_ms_per_step'], d['host_cpu']['threads_cpu_ms_per_step'], d['step_breakdown']['side_stream_cost_ms'])"
  done
done
timeout -k 10 120 python scripts/side_cost.py --mode calib > $O/calib.txt 2>&1 || { echo "CALIB FAIL"; tail -20 $O/calib.txt; exit 1; }
grep -v amdgpu.ids $O/calib.txt
timeout -k 10 400 python scripts/side_cost.py --mode ab --replay profiles/r06/side_replay.json --steps 20 --rounds 3 > $O/side_ab.json 2> $O/side_ab.txt || { echo "SIDE AB FAIL"; tail -20 $O/side_ab.txt; exit 1; }
grep -v amdgpu.ids $O/side_ab.txt
echo ALLOK
