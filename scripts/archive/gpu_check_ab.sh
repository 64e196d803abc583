# Kernel + pipeline parity tests, then an interleaved A/B bench against hubertfa_amd/_build_abl/* builds.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/gputests.log 2>&1 || { echo "GPU TESTS FAIL"; tail -40 gpurun_out/gputests.log; exit 1; }
tail -1 gpurun_out/gputests.log
bash scripts/gpu_ab_bench.sh
