# Tiled UNet: parity tests, the UNet alone (chip-wide vs tiled), then the step A/B (HFA_UNET_TILED 0/1, interleaved).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_unet_fused_gpu.py -k tiled > gpurun_out/tiled_tests.log 2>&1 || { echo "TESTS FAIL"; tail -40 gpurun_out/tiled_tests.log; exit 1; }
grep -E "PASSED|FAILED|diff|err" gpurun_out/tiled_tests.log | tail -20
timeout -k 10 200 python scripts/unet_tiled_bench.py 2>&1 | grep -v amdgpu.ids || exit 1
for r in 1 2 3; do for f in 0 1; do
HFA_UNET_TILED=$f timeout -k 10 300 python bench.py --steps 30 --warmup 3 --no-cpu-baseline > gpurun_out/bench_ab.json 2> gpurun_out/bench_ab.err || { tail -20 gpurun_out/bench_ab.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/bench_ab.json').read().strip().splitlines()[-1]); print('tiled=$f', round(d['value']), round(d['ms_per_step'],3), {k: round(v,3) for k,v in d['step_breakdown'].items() if k != 'note'})"
done; done
