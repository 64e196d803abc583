# Round 4: PMC passes over the config-2 split attention alone (scripts/attn_pmc_driver.py), each in its own run:
# the SQ issue / wait split, MFMA / VALU co-execution and LDS bank conflicts; then per-instruction-class activity.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04p
rm -rf $O; mkdir -p $O
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_VALU_MFMA_COEXEC_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT --output-format csv -d $O/p1 -o run -- python3 scripts/attn_pmc_driver.py > $O/p1.log 2>&1 || { echo "P1 FAIL"; tail -5 $O/p1.log; exit 1; }
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE --output-format csv -d $O/p2 -o run -- python3 scripts/attn_pmc_driver.py > $O/p2.log 2>&1 || { echo "P2 FAIL"; tail -5 $O/p2.log; exit 1; }
python3 - <<'PY'
import csv, glob, collections
for p in ("p1", "p2"):
    agg = collections.defaultdict(float); n = collections.Counter()
    for fn in glob.glob(f"gpurun_out/r04p/{p}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(fn)):
            if "attn_fwd_split" in r["Kernel_Name"]:
                agg[r["Counter_Name"]] += float(r["Counter_Value"]); n[r["Counter_Name"]] += 1
    print(p, {k: round(v / max(n[k], 1), 1) for k, v in sorted(agg.items())})
PY
echo ALLOK
