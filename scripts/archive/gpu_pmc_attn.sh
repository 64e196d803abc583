# PMC view of the flash-attention kernel on the workload shape (MFMA-pipe busy, clock, wave states, LDS).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for C in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CYCLES" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_MFMA"; do
  tag=$(echo $C | cut -d' ' -f1)
  rm -rf gpurun_out/pmc_attn_$tag
  timeout -k 10 200 rocprofv3 --kernel-trace --pmc $C --output-format csv -d gpurun_out/pmc_attn_$tag -o run -- python3 scripts/attn_bench.py --reps 3 > gpurun_out/pmc_attn_$tag.log 2>&1 || { echo "PMC $tag FAIL"; tail -5 gpurun_out/pmc_attn_$tag.log; exit 1; }
done
python - <<'PY'
import csv, glob, collections
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for d in glob.glob("gpurun_out/pmc_attn_*"):
    for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "attn_fwd" not in r["Kernel_Name"]: continue
            k = (int(r["Grid_Size"]),)
            e = agg[k]
            e[r["Counter_Name"]] += float(r["Counter_Value"])
            e["ns_" + r["Counter_Name"]] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
for k, e in agg.items():
    cyc = e["GRBM_GUI_ACTIVE"] / 8
    wc = e["SQ_WAVE_CYCLES"] or 1
    print(f"grid {k[0]}: clk {cyc / e['ns_GRBM_GUI_ACTIVE']:.2f} GHz  mfma busy {100 * e['SQ_VALU_MFMA_BUSY_CYCLES'] / (cyc * 1024):.1f} %"
          f"  wait {100 * e['SQ_WAIT_ANY'] / wc:.1f} %  instw {100 * e['SQ_WAIT_INST_ANY'] / wc:.1f} %  act {100 * e['SQ_ACTIVE_INST_ANY'] / wc:.1f} %"
          f"  ldsconf {100 * e['SQ_LDS_BANK_CONFLICT'] / max(1, e['SQ_LDS_IDX_ACTIVE']):.1f} %  valu/mfma {e['SQ_INSTS_VALU'] / max(1, e['SQ_INSTS_MFMA']):.2f}")
PY
echo ALLOK
