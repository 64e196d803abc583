# Round-2 GPU validation: the whole -m gpu suite (per-test timeout), then smoke.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1500 python -u -m pytest tests -m gpu -v -rf --timeout 420 --timeout-method thread ${PYTEST_ARGS:-} > gpurun_out/gputests.log 2>&1
rc=$?
tail -30 gpurun_out/gputests.log
[ $rc -eq 0 ] || { echo "GPU TESTS rc=$rc"; exit 1; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "SMOKE FAIL"; tail -20 gpurun_out/smoke.log; exit 1; }
tail -2 gpurun_out/smoke.log
echo ALLOK
