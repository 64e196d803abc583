# Step A/B on one box: chip-wide UNet on the side stream (current), UNet on the main stream (only the DP beside
# the next encoder), the fused UNet kernel on the side stream.
set -o pipefail
mkdir -p gpurun_out
for cfg in "0 0" "0 1" "1 0" "0 0" "0 1"; do set -- $cfg
HFA_UNET_FUSED=$1 HFA_HEAD_ON_MAIN=$2 timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/bench_ab.json 2> gpurun_out/bench_ab.err || { tail -20 gpurun_out/bench_ab.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/bench_ab.json').read().strip().splitlines()[-1]); print('fused=$1 head_on_main=$2', round(d['value']), round(d['ms_per_step'],3), {k: round(v,3) for k,v in d['step_breakdown'].items() if k != 'note'})"
done
