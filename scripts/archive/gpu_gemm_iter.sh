# GEMM iteration loop: DMA probe, kernel parity tests, microbench over pipelines/tiles, PMC summary.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 60 ./scripts/probes/dma_oob || { echo "PROBE FAIL"; exit 1; }
timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -x -q > gpurun_out/ktest.log 2>&1 || { echo "KTEST FAIL"; tail -30 gpurun_out/ktest.log; exit 1; }
tail -2 gpurun_out/ktest.log
timeout -k 10 300 python scripts/gemm_bench.py --variants ${V:-16:1,16:4,102:1,102:4,103:1,103:4,103:2} --reps 10 > gpurun_out/gemm_iter.log 2>&1 || { echo "GEMM BENCH FAIL"; tail -20 gpurun_out/gemm_iter.log; exit 1; }
cat gpurun_out/gemm_iter.log
echo ALLOK
