# Viterbi forward A/B on one box: DP parity tests on the working libhfa, then scripts/dp_bench.py on the old
# build (HFA_LIB=hubertfa_amd/_build_ab/dpold/libhfa.so) and the new one, interleaved.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_viterbi_gpu.py > gpurun_out/dp_tests.log 2>&1 || { echo "DP TESTS FAIL"; tail -30 gpurun_out/dp_tests.log; exit 1; }
tail -n 2 gpurun_out/dp_tests.log
for rep in 1 2; do for n in old new; do
  if [ $n = old ]; then export HFA_LIB=$PWD/hubertfa_amd/_build_ab/dpold/libhfa.so; else unset HFA_LIB; fi
  echo "== $n"; timeout -k 10 200 python scripts/dp_bench.py 2>&1 | grep -v amdgpu.ids || { echo "BENCH FAIL"; exit 1; }
done; done
