# DP: the skip's allow mask folded into its compare (one select fewer per state): Viterbi parity tests, DP alone vs
# the previous build (_build_ab), twice
set -o pipefail
O=gpurun_out/dpmask; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_viterbi_gpu.py tests/test_longform_gpu.py > $O/tests.txt 2>&1 || { echo "TESTS FAIL"; tail -40 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
A=hubertfa_amd/_build_ab/libhfa.so; B=hubertfa_amd/_build/libhfa.so
for i in 1 2; do
echo "== dp prev $i"; HFA_LIB=$A timeout -k 10 200 python scripts/dp_bench.py 2>&1 | grep "K=auto" || exit 1
echo "== dp new $i"; HFA_LIB=$B timeout -k 10 200 python scripts/dp_bench.py 2>&1 | grep "K=auto" || exit 1
done
echo ALLOK
