set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -m pytest tests/test_pipeline_gpu.py -x -q -s > gpurun_out/t4.log 2>&1 || { echo "PYTEST FAIL $?" >> gpurun_out/t4.log; exit 1; }
timeout -k 10 300 python bench.py --steps 5 --warmup 2 > gpurun_out/bench1.json 2> gpurun_out/bench1.err || { echo "BENCH FAIL $?"; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof1 -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/prof1.log 2>&1 || { echo "PROF FAIL $?"; exit 1; }
echo ALLOK
