# Interleaved A/B of bench.py between the working tree (cur) and an older Python tree under _ab/old (same libhfa),
# on one box: the effect of a host-side change (device-to-device clock differences make cross-box comparisons
# unreliable).
set -o pipefail
mkdir -p gpurun_out
for rep in 1 2 3; do
  for n in cur old; do
    dir=$PWD; [ $n = old ] && dir=$PWD/_ab/old
    (cd $dir && timeout -k 10 300 python bench.py --steps ${STEPS:-10} --warmup 3 --no-cpu-baseline) > gpurun_out/abt_$n.json 2> gpurun_out/abt_$n.err || { echo "BENCH FAIL $n"; tail -5 gpurun_out/abt_$n.err; exit 1; }
    python -c "import json; d=json.loads(open('gpurun_out/abt_$n.json').read().strip().splitlines()[-1]); print('$n', round(d['value'],1), round(d['ms_per_step'],3))"
  done
done
echo ALLOK
