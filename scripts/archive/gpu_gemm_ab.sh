# GEMM kernel tests, microbench current vs hubertfa_amd/_build_abl/* builds, then the interleaved pipeline A/B.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -x -q > gpurun_out/kt.log 2>&1 || { echo KFAIL; tail -30 gpurun_out/kt.log; exit 1; }
tail -1 gpurun_out/kt.log
for n in cur $(ls hubertfa_amd/_build_abl 2>/dev/null); do
  lib=$PWD/hubertfa_amd/_build_abl/$n/libhfa.so; [ $n = cur ] && lib=$PWD/hubertfa_amd/_build/libhfa.so
  echo "== $n"
  HFA_LIB=$lib timeout -k 10 120 python scripts/gemm_bench.py --variants ${V:-0:0} --shapes ${SH:-conv1,conv3,qkv,outproj,ffn1,ffn2,posconv,unet_k3} --reps 10 2>&1 | grep -v amdgpu.ids || exit 1
done
bash scripts/gpu_ab_bench.sh
