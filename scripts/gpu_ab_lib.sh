# Interleaved A/B of a kernel change on one box: the working libhfa (cur) against an alternative build (alt,
# HFA_LIB=hubertfa_amd/_build_ab/libhfa.so, e.g. `make -C hubertfa_amd/csrc OUT=../_build_ab EXTRA=-D...`).
# MICRO="python scripts/attn_bench.py" adds a microbenchmark pass per side.
set -o pipefail
mkdir -p gpurun_out
ALT=$PWD/hubertfa_amd/_build_ab/libhfa.so
for rep in 1 2 3; do
  for n in cur alt; do
    if [ $n = alt ]; then export HFA_LIB=$ALT; else unset HFA_LIB; fi
    if [ -n "$MICRO" ] && [ $rep = 1 ]; then
      timeout -k 10 120 $MICRO > gpurun_out/abl_micro_$n.txt 2>&1 || { echo "MICRO FAIL $n"; tail -5 gpurun_out/abl_micro_$n.txt; exit 1; }
      echo "== micro $n"; grep -v amdgpu.ids gpurun_out/abl_micro_$n.txt
    fi
    timeout -k 10 300 python bench.py --steps ${STEPS:-10} --warmup 3 --no-cpu-baseline > gpurun_out/abl_$n.json 2> gpurun_out/abl_$n.err || { echo "BENCH FAIL $n"; tail -5 gpurun_out/abl_$n.err; exit 1; }
    python -c "import json; d=json.loads(open('gpurun_out/abl_$n.json').read().strip().splitlines()[-1]); print('$n', round(d['value'],1), round(d['ms_per_step'],3))"
  done
done
unset HFA_LIB
echo ALLOK
