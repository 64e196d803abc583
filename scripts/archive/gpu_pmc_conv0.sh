# PMC passes over the conv0 microbenchmark: HBM traffic of the packed apply pass (FETCH_SIZE, WRITE_SIZE in separate
# passes) and its issue profile (wave cycles / waits / VALU and MFMA busy).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/pmc_c0_fetch gpurun_out/pmc_c0_write
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_c0_fetch -o run -- python3 scripts/conv0_bench.py --reps 3 > gpurun_out/pmc_c0_fetch.log 2>&1 || { echo "PMC FETCH FAIL"; tail -5 gpurun_out/pmc_c0_fetch.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_c0_write -o run -- python3 scripts/conv0_bench.py --reps 3 > gpurun_out/pmc_c0_write.log 2>&1 || { echo "PMC WRITE FAIL"; tail -5 gpurun_out/pmc_c0_write.log; exit 1; }
python scripts/pmc_traffic.py --fetch gpurun_out/pmc_c0_fetch --write gpurun_out/pmc_c0_write --kernel "conv0_packed_kernelILi0ELi1ELi0ELb1E" --out gpurun_out/traffic_conv0_r03.json && cat gpurun_out/traffic_conv0_r03.json
for C in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU"; do
  tag=$(echo $C | cut -d' ' -f1)
  rm -rf gpurun_out/pmc_gemm_$tag
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $C --output-format csv -d gpurun_out/pmc_gemm_$tag -o run -- python3 scripts/conv0_bench.py --reps 3 > gpurun_out/pmc_gemm_$tag.log 2>&1 || { echo "PMC $tag FAIL"; exit 1; }
done
KFILTER=conv0_ python scripts/pmc_gemm.py gpurun_out > gpurun_out/pmc_conv0_summary.txt 2>&1; cat gpurun_out/pmc_conv0_summary.txt
echo ALLOK
