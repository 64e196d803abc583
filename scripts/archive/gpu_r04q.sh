# Round 4: split attention with V two tiles ahead in a 3-stage LDS ring (candidate library in hubertfa_amd/_build_ab)
# against the shipped 2-stage ring: the attention parity tests on the candidate, then the layer microbenchmark and the
# bench step interleaved (scripts/gpu_ab_libs.sh) and the length sweep on both.  OUT=gpurun_out/r04q.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04q
mkdir -p $O
ALT=$PWD/hubertfa_amd/_build_ab/libhfa.so
HFA_LIB=$ALT timeout -k 10 400 python -u -m pytest tests/test_split_gpu.py tests/test_varlen_gpu.py tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "attention or varlen" > $O/tests.log 2>&1 || { echo "TESTS FAIL"; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
OUT=$O/libs REPS=3 bash scripts/gpu_ab_libs.sh
for n in cur alt; do
  if [ $n = alt ]; then export HFA_LIB=$ALT; else unset HFA_LIB; fi
  timeout -k 10 200 python scripts/attn_len_sweep.py > $O/sweep_$n.txt 2>&1 || { echo "SWEEP FAIL"; tail -5 $O/sweep_$n.txt; exit 1; }
  echo "== sweep $n"; grep -v amdgpu.ids $O/sweep_$n.txt
done
unset HFA_LIB
echo ALLOK
