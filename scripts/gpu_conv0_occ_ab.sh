# Interleaved step A/B on one box: conv0's packed apply pass at its natural 3 workgroups per CU (mode 0) vs held to
# 2 (mode 10: room for a side-stream GEMM workgroup beside it).
set -o pipefail
mkdir -p gpurun_out
for r in 1 2 3; do for m in 0 10; do
HFA_CONV0_TUNING=$m timeout -k 10 300 python bench.py --steps 30 --warmup 3 --no-cpu-baseline > gpurun_out/bench_ab.json 2> gpurun_out/bench_ab.err || { tail -20 gpurun_out/bench_ab.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/bench_ab.json').read().strip().splitlines()[-1]); print('conv0 mode=$m', round(d['value']), round(d['ms_per_step'],3), {k: round(v,3) for k,v in d['step_breakdown'].items() if k != 'note'})"
done; done
