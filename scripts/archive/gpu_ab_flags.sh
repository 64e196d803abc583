# Interleaved A/B of bench.py flag sets on one box: FLAGS_A vs FLAGS_B (default: --serial vs two-stream).
set -o pipefail
mkdir -p gpurun_out
A=${FLAGS_A:---serial}; B=${FLAGS_B:-}
for rep in 1 2; do
  for tag in A B; do
    f=$A; [ $tag = B ] && f=$B
    timeout -k 10 300 python bench.py --steps ${STEPS:-10} --warmup 3 --no-cpu-baseline $f > gpurun_out/abf_$tag.json 2> gpurun_out/abf_$tag.err || { echo "BENCH FAIL $tag"; tail -5 gpurun_out/abf_$tag.err; exit 1; }
    python -c "import json; d=json.loads(open('gpurun_out/abf_$tag.json').read().strip().splitlines()[-1]); print('$tag [$f]', round(d['value'],1), round(d['ms_per_step'],3), round(d['roofline']['avg_launch_ms'],4))"
  done
done
echo ALLOK
