set -o pipefail
timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -x -q -k "variants or gemm" > gpurun_out/kt.log 2>&1 || { echo KFAIL; tail -20 gpurun_out/kt.log; exit 1; }
tail -1 gpurun_out/kt.log
timeout -k 10 300 python scripts/gemm_bench.py --variants 102:1,102:5,102:6,103:5,103:6 --shapes conv1,conv3,conv5,qkv,outproj,ffn1,ffn2 --reps 10 2>&1 | grep -v amdgpu.ids
echo ALLOK
