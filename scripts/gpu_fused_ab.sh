# Interleaved step A/B on one box (box noise is +-2 %): chip-wide UNet (0) vs the fused UNet kernel (1).
set -o pipefail
mkdir -p gpurun_out
for r in 1 2 3 4 5; do for f in 0 1; do
HFA_UNET_FUSED=$f timeout -k 10 300 python bench.py --steps 30 --warmup 3 --no-cpu-baseline > gpurun_out/bench_ab.json 2> gpurun_out/bench_ab.err || { tail -20 gpurun_out/bench_ab.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/bench_ab.json').read().strip().splitlines()[-1]); print('fused=$f', round(d['value']), round(d['ms_per_step'],3), {k: round(v,3) for k,v in d['step_breakdown'].items() if k != 'note'})"
done; done
