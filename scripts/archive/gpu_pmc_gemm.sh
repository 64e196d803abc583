# PMC passes over the GEMM microbenchmark: wave-state breakdown, MFMA-pipe busy + effective clock, LDS.
# Each counter group in its own rocprofv3 pass (with --kernel-trace for durations); parsed by pmc_gemm.py.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
V=${V:-16:1}
SH=${SH:-conv1,qkv,outproj,ffn1,ffn2}
for C in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CYCLES" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS"; do
  tag=$(echo $C | cut -d' ' -f1)
  rm -rf gpurun_out/pmc_gemm_$tag
  timeout -k 10 200 rocprofv3 --kernel-trace --pmc $C --output-format csv -d gpurun_out/pmc_gemm_$tag -o run -- python3 scripts/gemm_bench.py --variants $V --shapes $SH --reps 3 > gpurun_out/pmc_gemm_$tag.log 2>&1 || { echo "PMC $tag FAIL"; exit 1; }
done
python scripts/pmc_gemm.py gpurun_out > gpurun_out/pmc_gemm_summary.txt 2>&1; cat gpurun_out/pmc_gemm_summary.txt
echo ALLOK
