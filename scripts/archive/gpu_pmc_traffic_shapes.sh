set -o pipefail
export TMPDIR=/tmp
rm -rf gpurun_out/pmcf gpurun_out/pmcw
timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmcf -o run -- python3 scripts/gemm_bench.py --variants 102:1 --shapes conv1,conv3,qkv,ffn1 --reps 2 > /dev/null 2>&1 || exit 1
timeout -k 10 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmcw -o run -- python3 scripts/gemm_bench.py --variants 102:1 --shapes conv1,conv3,qkv,ffn1 --reps 2 > /dev/null 2>&1 || exit 1
python - <<'PY'
import csv, glob, collections
def load(d, cn):
    out = collections.OrderedDict()
    for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "gemm_dma" not in r["Kernel_Name"] or r["Counter_Name"] != cn: continue
            out[int(r["Dispatch_Id"])] = out.get(int(r["Dispatch_Id"]), 0) + float(r["Counter_Value"])
    return list(out.values())
f = load("gpurun_out/pmcf", "FETCH_SIZE"); w = load("gpurun_out/pmcw", "WRITE_SIZE")
for i, (a, b) in enumerate(zip(f, w)):
    print(i, f"fetch {2 * a / 1e6:.1f} GB-corrected ({a / 1e6:.2f} GB raw KiB-units)  write {b / 1e6:.2f}")
PY
echo ALLOK
