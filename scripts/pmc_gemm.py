"""Summarise the PMC passes of scripts/archive/gpu_pmc_gemm.sh per GEMM dispatch shape.

MFMA-pipe utilisation = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE/8 x 1024 SIMDs) (BUSY counts 64 cycles per
32x32x2 f32 MFMA summed over SIMDs; GRBM_GUI_ACTIVE is summed over the 8 XCDs); effective clock =
GRBM_GUI_ACTIVE/8 / kernel wall time (MI355X_MICROARCH.md 'DVFS give-back'); SQ_* wave-state counters are
quad-cycles per wave, reported as fractions of SQ_WAVE_CYCLES.

python scripts/pmc_gemm.py gpurun_out
"""
import csv
import glob
import os
import sys
from collections import defaultdict

KERNELS = tuple(os.environ.get("KFILTER", "gemm_f32_kernel,gemm_dma_kernel,gemm_split_kernel").split(","))


def load(d):
    out = defaultdict(dict)
    for fn in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(fn)):
            if not any(t in r["Kernel_Name"] for t in KERNELS):
                continue
            k = int(r["Dispatch_Id"])
            e = out[k]
            e["name"] = r["Kernel_Name"].split("(anonymous namespace)::")[-1].split("(")[0][:60]
            e["grid"] = int(r["Grid_Size"])
            e["ns"] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
            e[r["Counter_Name"]] = e.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    return [out[k] for k in sorted(out)]


def main():
    root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out"
    groups = {tag: load(os.path.join(root, f"pmc_gemm_{tag}"))
              for tag in ("SQ_WAVE_CYCLES", "SQ_VALU_MFMA_BUSY_CYCLES", "SQ_LDS_BANK_CONFLICT")}
    n = min(len(v) for v in groups.values())
    print(f"{'kernel':44s} {'grid':>8s} {'us':>8s} {'GHz':>5s} {'mfma%':>6s} {'wait%':>6s} {'instw%':>6s} "
          f"{'act%':>6s} {'ldsconf%':>8s}")
    for i in range(n):
        w, m, l = groups["SQ_WAVE_CYCLES"][i], groups["SQ_VALU_MFMA_BUSY_CYCLES"][i], groups["SQ_LDS_BANK_CONFLICT"][i]
        cyc = m.get("GRBM_GUI_ACTIVE", 0) / 8
        ghz = cyc / m["ns"] if m["ns"] else 0
        util = m.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / (cyc * 1024) if cyc else 0
        wc = w.get("SQ_WAVE_CYCLES", 0) or 1
        lds = l.get("SQ_LDS_IDX_ACTIVE", 0) or 1
        print(f"{m['name'][:44]:44s} {m['grid']:8d} {m['ns'] / 1e3:8.1f} {ghz:5.2f} {100 * util:6.1f} "
              f"{100 * w.get('SQ_WAIT_ANY', 0) / wc:6.1f} {100 * w.get('SQ_WAIT_INST_ANY', 0) / wc:6.1f} "
              f"{100 * w.get('SQ_ACTIVE_INST_ANY', 0) / wc:6.1f} {100 * l.get('SQ_LDS_BANK_CONFLICT', 0) / lds:8.1f}")


if __name__ == "__main__":
    main()
