# Interleaved step A/B on one box: the side stream (head + lattice + DP) on n CUs of its own, the encoder on the rest
# (HFA_CU_SPLIT = n, CU-masked HIP streams), with the chip-wide UNet or the one-kernel UNet (HFA_UNET_FUSED = 1).
set -o pipefail
mkdir -p gpurun_out
for r in 1 2; do for cfg in "0 0" "16 0" "32 0" "16 1" "32 1"; do
set -- $cfg
HFA_CU_SPLIT=$1 HFA_UNET_FUSED=$2 timeout -k 10 300 python bench.py --steps 30 --warmup 3 --no-cpu-baseline > gpurun_out/bench_ab.json 2> gpurun_out/bench_ab.err || { tail -20 gpurun_out/bench_ab.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/bench_ab.json').read().strip().splitlines()[-1]); print('cu_split=$1 fused=$2', round(d['value']), round(d['ms_per_step'],3), {k: round(v,3) for k,v in d['step_breakdown'].items() if k != 'note'})"
done; done
