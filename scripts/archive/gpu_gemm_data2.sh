# Split-GEMM speed against operand data patterns (the power limit): randn, zeros, every W row equal (consecutive
# MFMAs of a wave see the same B fragments), every A row equal (the same A fragments).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/gemm_data2
mkdir -p $O
for rep in 1 2; do
  for d in randn wrows arows zeros; do
    timeout -k 10 200 python scripts/gemm_abl.py --data $d > $O/cur_$d.$rep.txt 2>&1 || { echo FAIL; tail -5 $O/cur_$d.$rep.txt; exit 1; }
    grep -v amdgpu.ids $O/cur_$d.$rep.txt
  done
done
echo ALLOK
