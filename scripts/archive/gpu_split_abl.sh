# Split GEMM microbench, current build vs hubertfa_amd/_build_abl/<name> builds, interleaved on one box.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for rep in 1 2; do
  for n in cur $(ls hubertfa_amd/_build_abl 2>/dev/null); do
    lib=$PWD/hubertfa_amd/_build_abl/$n/libhfa.so; [ $n = cur ] && lib=$PWD/hubertfa_amd/_build/libhfa.so
    echo "== $n"
    HFA_LIB=$lib timeout -k 10 200 python scripts/split_gemm_bench.py --reps ${REPS:-20} --cfgs ${CFGS:-17} --shapes ${SHAPES:-conv1,ffn1,ffn2,qkv} 2>&1 | grep -v amdgpu.ids || exit 1
  done
done | tee gpurun_out/split_abl.txt
