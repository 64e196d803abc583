set -o pipefail
timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -x -q > gpurun_out/kt.log 2>&1 || { echo KFAIL; tail -30 gpurun_out/kt.log; exit 1; }
tail -1 gpurun_out/kt.log
timeout -k 10 120 python scripts/gemm_bench.py --variants 0:0,103:2 --shapes posconv --reps 10 2>&1 | grep -v amdgpu.ids
echo ALLOK
