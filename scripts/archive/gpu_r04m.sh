# Round 4: sanity of the shipped build after the attention experiments were reverted: the attention / split GEMM /
# varlen / pipeline tests, smoke and a short bench line.  OUT=gpurun_out/r04m.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04m
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_split_gpu.py tests/test_varlen_gpu.py tests/test_pipeline_gpu.py tests/test_reference10s_gpu.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo "TESTS FAIL"; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "SMOKE FAIL"; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { echo "BENCH FAIL"; tail -20 $O/bench.err; exit 1; }
python -c "import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]); r=d['roofline']; print(d['value'], d['ms_per_step'], r['frac'], r['mfma_busy'], r['clock_ghz'], r['traffic'], d['host_cpu']['threads_cpu_ms_per_step'], d['step_breakdown']['side_stream_cost_ms'])"
echo ALLOK
