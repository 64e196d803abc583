# Parity tests of the working build, then the interleaved A/B of scripts/gpu_ab_lib.sh.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_split_gpu.py tests/test_reference10s_gpu.py tests/test_pipeline_gpu.py} -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/ab_tests.log 2>&1 || { echo "TESTS FAIL"; tail -30 gpurun_out/ab_tests.log; exit 1; }
tail -1 gpurun_out/ab_tests.log
bash scripts/gpu_ab_lib.sh
