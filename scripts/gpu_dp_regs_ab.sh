# Interleaved step A/B on one box: the one-wave DP with its default emission ring (177 VGPRs: a GEMM workgroup,
# 2 x 208 VGPRs per SIMD, cannot share the CU) vs short rings (hfa_viterbi_tuning 1: 69 VGPRs, 5: 109).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_viterbi_gpu.py -m gpu -x -q --timeout 120 > gpurun_out/dp_t.log 2>&1 || { tail -20 gpurun_out/dp_t.log; exit 1; }
tail -1 gpurun_out/dp_t.log
for r in 1 2 3; do for k in 0 1 5; do
HFA_VITERBI_TUNING=$k timeout -k 10 300 python bench.py --steps 30 --warmup 3 --no-cpu-baseline > gpurun_out/bench_ab.json 2> gpurun_out/bench_ab.err || { tail -20 gpurun_out/bench_ab.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/bench_ab.json').read().strip().splitlines()[-1]); s=d['secondary'][0]; print('k=$k', round(d['value']), round(d['ms_per_step'],3), 'dp', round(s['avg_launch_ms'],4), round(s['in_pipeline_avg_launch_ms'],4), {k: round(v,3) for k,v in d['step_breakdown'].items() if k != 'note'})"
done; done
