# Fused UNet kernel: its tests, then the microbenchmark and a bench line with the step breakdown.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_unet_fused_gpu.py tests/test_encoder_gpu.py -k "unet or fused" -v -s --timeout 120 --timeout-method thread > gpurun_out/fused_tests.log 2>&1; rc=$?
grep -E "PASSED|FAILED|ERROR|diff|err" gpurun_out/fused_tests.log | tail -30
[ $rc -eq 0 ] || { tail -60 gpurun_out/fused_tests.log; exit 1; }
timeout -k 10 200 python scripts/unet_bench.py --reps 20 > gpurun_out/unet_bench.txt 2>&1 || { cat gpurun_out/unet_bench.txt; exit 1; }
cat gpurun_out/unet_bench.txt
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bench_fused.json 2> gpurun_out/bench_fused.err || { tail -20 gpurun_out/bench_fused.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/bench_fused.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['step_breakdown'])"
