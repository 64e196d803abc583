# Round 6: split GEMM MFMA issue order A/B (HFA_AB_GROUPED_ORDER: per A fragment, the NJ products of each of the
# three split terms back to back, every accumulator's own sequence unchanged) -- output digests of both builds, the
# layer microbenchmark and the config-2 bench, interleaved.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06s
mkdir -p $O
ALT=$PWD/hubertfa_amd/_build_ab/libhfa.so
for n in cur alt; do
  if [ $n = alt ]; then export HFA_LIB=$ALT; else unset HFA_LIB; fi
  timeout -k 10 200 python scripts/layer_gemm_bench.py --reps 50 --dump $O/digest_$n.json > $O/micro_$n.txt 2>&1 || { echo "MICRO FAIL $n"; tail -5 $O/micro_$n.txt; exit 1; }
  echo "== micro $n"; grep -v amdgpu.ids $O/micro_$n.txt
done
unset HFA_LIB
python -c "import json; a=json.load(open('$O/digest_cur.json')); b=json.load(open('$O/digest_alt.json')); print('bit-identical' if a==b else 'DIFFER', a==b)"
for rep in 1 2 3; do
  for n in cur alt; do
    if [ $n = alt ]; then export HFA_LIB=$ALT; else unset HFA_LIB; fi
    timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extra-configs --sustained-s 5 > $O/bench_${n}_$rep.json 2> $O/bench_${n}_$rep.err || { echo "BENCH FAIL $n"; tail -5 $O/bench_${n}_$rep.err; exit 1; }
    python -c "import json; d=json.loads(open('$O/bench_${n}_$rep.json').read().strip().splitlines()[-1]); print('$n', $rep, round(d['ms_per_step'],3), round(d['sustained']['ms_per_step'],3), round(d['roofline']['avg_launch_ms']*1e3,1))"
  done
done
unset HFA_LIB
echo ALLOK
