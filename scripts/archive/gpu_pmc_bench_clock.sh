# In-pipeline effective clock and MFMA-pipe utilisation of every GEMM dispatch of bench.py (one PMC pass).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/pmc_gemm_SQ_VALU_MFMA_BUSY_CYCLES
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CYCLES --output-format csv -d gpurun_out/pmc_gemm_SQ_VALU_MFMA_BUSY_CYCLES -o run -- python3 bench.py --steps 4 --warmup 2 --no-cpu-baseline > gpurun_out/pmcclk.log 2>&1 || { echo PMCFAIL; tail gpurun_out/pmcclk.log; exit 1; }
python - <<'PY'
import csv, glob, collections
rows = []
for fn in glob.glob("gpurun_out/pmc_gemm_SQ_VALU_MFMA_BUSY_CYCLES/**/*counter_collection.csv", recursive=True):
    rows += list(csv.DictReader(open(fn)))
d = collections.defaultdict(dict)
for r in rows:
    if "gemm_dma_kernel" not in r["Kernel_Name"] and "attn_fwd" not in r["Kernel_Name"]:
        continue
    e = d[int(r["Dispatch_Id"])]
    e["name"] = r["Kernel_Name"].split("::")[1][:48]
    e["grid"] = int(r["Grid_Size"])
    e["ns"] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    e[r["Counter_Name"]] = e.get(r["Counter_Name"], 0) + float(r["Counter_Value"])
agg = collections.defaultdict(lambda: [0, 0.0, 0.0, 0.0])
for e in d.values():
    cyc = e["GRBM_GUI_ACTIVE"] / 8
    k = (e["name"], e["grid"])
    a = agg[k]; a[0] += 1; a[1] += e["ns"]; a[2] += cyc; a[3] += e["SQ_VALU_MFMA_BUSY_CYCLES"]
for (n, g), (c, ns, cyc, mb) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
    print(f"{n:48s} grid {g:9d} n {c:3d} avg {ns / c / 1e3:8.1f} us  clk {cyc / ns:5.2f} GHz  mfma {100 * mb / (cyc * 1024):5.1f} %")
PY
echo ALLOK
