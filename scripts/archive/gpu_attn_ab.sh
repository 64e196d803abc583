# Split attention: round-3 P split / unrolled loop vs the round-2 body -- parity, then the microbenchmark.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_split_gpu.py tests/test_kernels_gpu.py -m gpu -x -q -k "attention or attn" --timeout 120 --timeout-method thread > gpurun_out/attn_tests.log 2>&1 || { echo "TESTS FAIL"; tail -40 gpurun_out/attn_tests.log; exit 1; }
tail -2 gpurun_out/attn_tests.log
timeout -k 10 300 python scripts/attn_bench.py --reps 400 > gpurun_out/attn_ab.txt 2>&1 || { echo "BENCH FAIL"; tail -20 gpurun_out/attn_ab.txt; exit 1; }
cat gpurun_out/attn_ab.txt
