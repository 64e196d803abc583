# Round 4, first box: the GPU tests the retirements touch, then the per-shape roofline profile of the build.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04a
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_split_gpu.py tests/test_viterbi_gpu.py tests/test_encoder_gpu.py tests/test_kernels_gpu.py tests/test_pipeline_gpu.py tests/test_api_gpu.py tests/test_reference10s_gpu.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo "TESTS FAIL"; tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
OUT=$O bash scripts/gpu_shapes.sh
