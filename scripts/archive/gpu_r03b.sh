# Round-3 (second session): conv0 packed f16-MFMA apply + cheaper GELU -- parity tests, conv0 microbench, bench.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest ${TESTS:-tests/test_split_gpu.py tests/test_kernels_gpu.py tests/test_reference10s_gpu.py tests/test_pipeline_gpu.py} -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03b_tests.log 2>&1 || { echo "TESTS FAIL"; tail -40 gpurun_out/r03b_tests.log; exit 1; }
tail -2 gpurun_out/r03b_tests.log
timeout -k 10 300 python scripts/conv0_bench.py --reps 20 > gpurun_out/r03b_conv0.txt 2>&1 || { echo "CONV0 BENCH FAIL"; tail -20 gpurun_out/r03b_conv0.txt; exit 1; }
cat gpurun_out/r03b_conv0.txt
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r03b_bench.json 2> gpurun_out/r03b_bench.err || { echo "BENCH FAIL"; tail -20 gpurun_out/r03b_bench.err; exit 1; }
python - <<'PY'
import json
d = json.loads(open('gpurun_out/r03b_bench.json').read().strip().splitlines()[-1])
r = d['roofline']
print('value', round(d['value'], 1), 'ms/step', round(d['ms_per_step'], 3), 'frac', round(r['frac'], 4), r['kernel'], round(r['avg_launch_ms'], 4))
print([(s['kernel'][:16], round(s['avg_launch_ms'], 4), round(s.get('frac', 0), 3)) for s in d['secondary']])
print(d.get('step_breakdown'))
PY
