set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
rocprofv3 -L > gpurun_out/counters.txt 2>&1 || true
for C in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CYCLES" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS"; do
  tag=$(echo $C | cut -d' ' -f1)
  timeout -k 10 200 rocprofv3 --pmc $C --output-format csv -d gpurun_out/pmc_gemm_$tag -o run -- python3 scripts/gemm_bench.py --variants 16:1,16:4 --reps 3 > gpurun_out/pmc_gemm_$tag.log 2>&1 || echo "PMC $tag FAIL"
done
echo ALLOK
