set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -m gpu -q -x -s > gpurun_out/gputests.log 2>&1 || { echo "GPU TESTS FAIL"; tail -40 gpurun_out/gputests.log; exit 1; }
echo ALLOK
