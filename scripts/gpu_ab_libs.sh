# Interleaved A/B on one box of the working libhfa (cur) and hubertfa_amd/_build_ab/libhfa.so (alt): the layer
# GEMM/attention microbenchmark and the bench step, REPS rounds.  OUT=gpurun_out/<tag>.
set -o pipefail
export TMPDIR=/tmp
O=${OUT:-gpurun_out/ab}
mkdir -p $O
ALT=$PWD/hubertfa_amd/_build_ab/libhfa.so
for rep in $(seq 1 ${REPS:-3}); do
  for n in cur alt; do
    if [ $n = alt ]; then export HFA_LIB=$ALT; else unset HFA_LIB; fi
    timeout -k 10 120 ${MICRO:-python scripts/layer_gemm_bench.py} > $O/micro_${n}_$rep.txt 2>&1 || { echo "MICRO FAIL $n"; tail -5 $O/micro_${n}_$rep.txt; exit 1; }
    echo "== micro $n $rep"; grep -v amdgpu.ids $O/micro_${n}_$rep.txt || true
    timeout -k 10 300 python bench.py --steps ${STEPS:-20} --warmup 5 --no-cpu-baseline > $O/bench_${n}_$rep.json 2> $O/bench_${n}_$rep.err || { echo "BENCH FAIL $n"; tail -5 $O/bench_${n}_$rep.err; exit 1; }
    python -c "import json; d=json.loads(open('$O/bench_${n}_$rep.json').read().strip().splitlines()[-1]); print('$n', round(d['value'],1), round(d['ms_per_step'],3), 'side', round(d['step_breakdown']['side_stream_cost_ms'],3), 'enc', round(d['step_breakdown']['encoder_only_ms'],3))"
  done
done
unset HFA_LIB
echo ALLOK
