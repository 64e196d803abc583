# PMC passes (MFMA busy, clock, wait states, LDS) of the split GEMM microbench for several builds / tile cfgs.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for spec in ${SPECS:-cur:7 cur:17 p2:17}; do
  n=${spec%%:*}; cf=${spec##*:}
  lib=$PWD/hubertfa_amd/_build_abl/$n/libhfa.so; [ $n = cur ] && lib=$PWD/hubertfa_amd/_build/libhfa.so
  echo "== $n cfg $cf"
  d=gpurun_out/pmc_$n_$cf; rm -rf $d; mkdir -p $d
  for C in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CYCLES" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS"; do
    tag=$(echo $C | cut -d' ' -f1)
    HFA_LIB=$lib timeout -k 10 200 rocprofv3 --kernel-trace --pmc $C --output-format csv -d $d/pmc_gemm_$tag -o run -- python3 scripts/split_gemm_bench.py --cfgs $cf --shapes ${SH:-conv1,ffn1} --reps 3 > $d/$tag.log 2>&1 || { echo "PMC $tag FAIL"; tail -5 $d/$tag.log; exit 1; }
  done
  KFILTER=gemm_split_kernel python scripts/pmc_gemm.py $d | awk 'NR==1 || NR%4==0'
  rm -rf $d
done
echo ALLOK
