"""Per-kernel MFMA utilisation and clock from rocprofv3 PMC passes (CPU): for every kernel instantiation, over all
of its dispatches in the pass, MFMA pipe busy = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x GRBM_GUI_ACTIVE / 8) and the
effective clock = GRBM_GUI_ACTIVE / 8 / dispatch time (MI355X_MICROARCH.md 'DVFS give-back'), plus the SQ wait
split (SQ_WAIT_ANY, SQ_WAIT_INST_ANY, SQ_ACTIVE_INST_ANY over SQ_WAVE_CYCLES) when a second pass carries it.

    python scripts/pmc_kernels.py --mfma DIR [--wait DIR] --out profiles/r04/pmc_r04.json

bench.py reads the file (--pmc-file) and reports the probed kernel's mfma_busy / clock_ghz in its roofline block.
The profiler serialises dispatches under --pmc, so these are per-kernel-alone figures."""
import argparse
import csv
import glob
import json
import os
from collections import defaultdict


def norm_name(n: str) -> str:
    n = n[5:] if n.startswith("void ") else n
    n = n.replace("(anonymous namespace)::", "")
    depth, out = 0, []
    for ch in n:
        if ch == "<":
            depth += 1
        elif ch == ">":
            depth -= 1
        elif ch == "(" and depth == 0:
            break
        out.append(ch)
    return "".join(out).strip()


def load(d):
    disp = {}
    for fn in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(fn)):
            e = disp.setdefault(int(r["Dispatch_Id"]), {"name": norm_name(r["Kernel_Name"]),
                                                        "ns": int(r["End_Timestamp"]) - int(r["Start_Timestamp"])})
            e[r["Counter_Name"]] = e.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    agg = defaultdict(lambda: defaultdict(float))
    for e in disp.values():
        a = agg[e["name"]]
        a["dispatches"] += 1
        for k, v in e.items():
            if k != "name":
                a[k] += v
    return agg


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mfma", required=True)
    ap.add_argument("--wait")
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    res = {}
    for name, v in load(a.mfma).items():
        if not v.get("GRBM_GUI_ACTIVE") or not v.get("ns"):
            continue
        cyc = v["GRBM_GUI_ACTIVE"] / 8.0
        res[name] = {"dispatches": int(v["dispatches"]), "avg_us_profiled": v["ns"] / v["dispatches"] / 1e3,
                     "clock_ghz": cyc / v["ns"], "mfma_busy": v.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) / (cyc * 1024.0)}
    if a.wait:
        for name, v in load(a.wait).items():
            if name in res and v.get("SQ_WAVE_CYCLES"):
                for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
                    res[name][k.lower()[3:] + "_frac"] = v.get(k, 0.0) / v["SQ_WAVE_CYCLES"]
    out = {"method": "rocprofv3 --kernel-trace --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CYCLES (and a "
                     "separate SQ_WAVE_CYCLES / SQ_WAIT_* pass) over scripts/shape_trace.py (the pipelined config-2 "
                     "step); per kernel over all its dispatches: mfma_busy = MFMA_BUSY / (1024 x GRBM_GUI_ACTIVE/8), "
                     "clock = GRBM_GUI_ACTIVE/8 / dispatch time; dispatches serialised by the profiler",
           "kernels": res}
    os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(out, f, indent=1)
    for n, v in sorted(res.items(), key=lambda kv: -kv[1]["avg_us_profiled"] * kv[1]["dispatches"])[:15]:
        print(f"{n[:80]:80s} n {v['dispatches']:4d} busy {v['mfma_busy']:.3f} clk {v['clock_ghz']:.2f}")


if __name__ == "__main__":
    main()
