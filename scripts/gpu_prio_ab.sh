# Step A/B on one box: side-stream priority relative to the encoder (same / high / low).
set -o pipefail
mkdir -p gpurun_out
for p in same low high same low high; do
HFA_SIDE_PRIO=$p timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/bench_ab.json 2> gpurun_out/bench_ab.err || { tail -20 gpurun_out/bench_ab.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/bench_ab.json').read().strip().splitlines()[-1]); print('prio=$p', round(d['value']), round(d['ms_per_step'],3), {k: round(v,3) for k,v in d['step_breakdown'].items() if k != 'note'})"
done
