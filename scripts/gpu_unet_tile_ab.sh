# Interleaved step A/B on one box: the UNet backbone's split-GEMM tiles -- automatic (0) vs a forced tile
# (HFA_UNET_TILE = gemm.hip SCFG index: 23 = 256x192, 17 = 256x256, 18 = 128x128, 19 = 128x64).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python scripts/unet_bench.py > gpurun_out/unet_tile_micro.txt 2>&1 || true
for r in 1 2 3; do for t in 0 ${TILES:-23 19}; do
HFA_UNET_TILE=$t timeout -k 10 300 python bench.py --steps 30 --warmup 3 --no-cpu-baseline > gpurun_out/bench_ab.json 2> gpurun_out/bench_ab.err || { tail -20 gpurun_out/bench_ab.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/bench_ab.json').read().strip().splitlines()[-1]); print('tile=$t', round(d['value']), round(d['ms_per_step'],3), {k: round(v,3) for k,v in d['step_breakdown'].items() if k != 'note'})"
done; done
