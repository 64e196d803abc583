# Round-1 measurement: bench line, rocprof kernel stats, PMC traffic of the dominant kernel.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
K='gemm_f32_kernel<1, true, 16, 128, 256, 2, 4>'
timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -x -q > gpurun_out/k2.log 2>&1 || { echo "KTEST FAIL"; tail -30 gpurun_out/k2.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof2 -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/prof2.log 2>&1 || { echo "PROF FAIL"; exit 1; }
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/pmc1.log 2>&1 || { echo "PMC1 FAIL"; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/pmc2.log 2>&1 || { echo "PMC2 FAIL"; exit 1; }
python scripts/pmc_traffic.py --fetch gpurun_out/pmc_fetch --write gpurun_out/pmc_write --kernel "$K" --out gpurun_out/traffic_r01.json > gpurun_out/traffic.log 2>&1 || echo "TRAFFIC PARSE FAIL"
cp gpurun_out/traffic_r01.json profiles/ 2>/dev/null
timeout -k 10 400 python bench.py --steps 10 --warmup 3 > gpurun_out/bench3.json 2> gpurun_out/bench3.err || { echo "BENCH FAIL"; exit 1; }
echo ALLOK
