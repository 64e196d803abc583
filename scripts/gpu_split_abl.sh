# Timing-only ablations of the split-f16 GEMM (hubertfa_amd/_build_abl/<name>/libhfa.so built with
# HFA_SABL_* macros) against the default build, on the workload's shapes.
set -o pipefail
mkdir -p gpurun_out
for n in base $(ls hubertfa_amd/_build_abl); do
  lib=hubertfa_amd/_build_abl/$n/libhfa.so; [ $n = base ] && lib=hubertfa_amd/_build/libhfa.so
  echo "== $n"
  HFA_LIB=$PWD/$lib timeout -k 10 200 python scripts/split_gemm_bench.py --cfgs ${CFGS:-1,3} --reps 10 2>&1 | grep -v amdgpu.ids || { echo "FAIL $n"; exit 1; }
done
echo ALLOK
