# A/B timing of alternative GEMM builds (hubertfa_amd/_build_abl/<name>/libhfa.so) against the default build.
set -o pipefail
mkdir -p gpurun_out
for n in base $(ls hubertfa_amd/_build_abl); do
  lib=hubertfa_amd/_build_abl/$n/libhfa.so; [ $n = base ] && lib=hubertfa_amd/_build/libhfa.so
  echo "== $n"
  HFA_LIB=$PWD/$lib timeout -k 10 200 python scripts/gemm_bench.py --variants ${V:-102:1,102:2,103:2} --shapes ${SH:-conv1,conv3,conv5,qkv,outproj,ffn1,ffn2,posconv,unet_k3} --reps 10 2>&1 | grep -v amdgpu.ids || { echo "FAIL $n"; exit 1; }
done
echo ALLOK
