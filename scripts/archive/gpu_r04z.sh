# Round 4, end: the whole GPU test suite and smoke on the final tree (the shipped libhfa.so).  OUT=gpurun_out/r04z.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04z
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gputests.log 2>&1 || { echo "GPU TESTS FAIL"; tail -40 $O/gputests.log; exit 1; }
tail -2 $O/gputests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "SMOKE FAIL"; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
echo ALLOK
