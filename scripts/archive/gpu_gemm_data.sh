# Split-GEMM speed against operand data (power: the chip runs the GEMMs power-limited): randn vs zeros vs
# f16-exact operands on the current build, and the no-DMA ablation build beside them.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/gemm_data
mkdir -p $O
for rep in 1 2; do
  for d in randn zeros hionly; do
    timeout -k 10 200 python scripts/gemm_abl.py --data $d > $O/cur_$d.$rep.txt 2>&1 || { echo FAIL; tail -5 $O/cur_$d.$rep.txt; exit 1; }
    grep -v amdgpu.ids $O/cur_$d.$rep.txt
  done
  HFA_LIB=$PWD/hubertfa_amd/_abl_nodma/libhfa.so timeout -k 10 200 python scripts/gemm_abl.py --data randn > $O/nodma.$rep.txt 2>&1 || { echo FAIL; exit 1; }
  grep -v amdgpu.ids $O/nodma.$rep.txt
done
echo ALLOK
