set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -x -q > gpurun_out/k1.log 2>&1 || { echo "KTEST FAIL"; tail -30 gpurun_out/k1.log; exit 1; }
timeout -k 10 500 python scripts/gemm_bench.py > gpurun_out/gemm1.log 2>&1 || { echo "GEMMBENCH FAIL"; exit 1; }
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bench2.json 2> gpurun_out/bench2.err || { echo "BENCH FAIL"; exit 1; }
echo ALLOK
