set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -x -q -k "variants or gemm or erf" > gpurun_out/k3.log 2>&1 || { echo "KTEST FAIL"; tail -30 gpurun_out/k3.log; exit 1; }
timeout -k 10 500 python scripts/gemm_bench.py --variants 16:1,16:4 > gpurun_out/gemm2.log 2>&1 || { echo "GEMMBENCH FAIL"; exit 1; }
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bench4.json 2> gpurun_out/bench4.err || { echo "BENCH FAIL"; tail gpurun_out/bench4.err; exit 1; }
echo ALLOK
