# Step breakdown with the fused UNet on and off (A/B on one box).
set -o pipefail
mkdir -p gpurun_out
for f in 1 0; do
HFA_UNET_FUSED=$f timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bench_f$f.json 2> gpurun_out/bench_f$f.err || { tail -20 gpurun_out/bench_f$f.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/bench_f$f.json').read().strip().splitlines()[-1]); print('fused=$f', round(d['value']), round(d['ms_per_step'],3), {k: round(v,3) for k,v in d['step_breakdown'].items() if k != 'note'})"
done
