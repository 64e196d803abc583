# Quick GPU loop: selected test files (TESTS), then one bench line.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest ${TESTS:-tests/test_split_gpu.py} -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/quick_tests.log 2>&1 || { echo "TESTS FAIL"; tail -40 gpurun_out/quick_tests.log; exit 1; }
tail -2 gpurun_out/quick_tests.log
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/quick_bench.json 2> gpurun_out/quick_bench.err || { echo "BENCH FAIL"; tail -20 gpurun_out/quick_bench.err; exit 1; }
python - <<'PY'
import json
d = json.loads(open('gpurun_out/quick_bench.json').read().strip().splitlines()[-1])
r = d['roofline']
print('value', round(d['value'], 1), 'ms/step', round(d['ms_per_step'], 3), 'frac', round(r['frac'], 4), r['kernel'], round(r['avg_launch_ms'], 4))
print([(s['kernel'][:16], round(s['avg_launch_ms'], 4)) for s in d['secondary']])
PY
