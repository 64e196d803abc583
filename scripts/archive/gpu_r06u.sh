# Round 6: interleaved bench A/B of the two-kernel chain edge pass (working tree) against the previous commit's tree
# (_ab/old: its Python and its libhfa), one box.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06u
mkdir -p $O
for rep in 1 2 3; do
  for n in cur old; do
    dir=$PWD; [ $n = old ] && dir=$PWD/_ab/old
    (cd $dir && timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extra-configs --sustained-s 5) > $O/bench_${n}_$rep.json 2> $O/bench_${n}_$rep.err || { echo "BENCH FAIL $n"; tail -5 $O/bench_${n}_$rep.err; exit 1; }
    python -c "import json; d=json.loads(open('$O/bench_${n}_$rep.json').read().strip().splitlines()[-1]); print('$n', $rep, round(d['ms_per_step'],3), round(d['sustained']['ms_per_step'],3))"
  done
done
echo ALLOK
