# Epilogue cost split: GELU on/off (--epi) and, for hubertfa_amd/_build_abl/* builds (e.g. stores disabled), the same.
set -o pipefail
for n in cur $(ls hubertfa_amd/_build_abl 2>/dev/null); do
  lib=$PWD/hubertfa_amd/_build_abl/$n/libhfa.so; [ $n = cur ] && lib=$PWD/hubertfa_amd/_build/libhfa.so
  for e in 0 1; do
    echo "== $n epi=$e"
    HFA_LIB=$lib timeout -k 10 120 python scripts/gemm_bench.py --variants ${V:-102:1} --shapes ${SH:-conv1,qkv,ffn1,ffn2} --epi $e --reps 10 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
echo ALLOK
