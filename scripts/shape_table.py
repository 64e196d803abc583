"""Per-shape in-pipeline roofline table from a rocprofv3 kernel trace (+ optional PMC passes) of
scripts/shape_trace.py (CPU; see that script for the recipe).

Each launch the ops layer logged (host order) is paired with the next trace dispatch of the same kernel (dispatch
ids follow host enqueue order; one host thread enqueues both streams), which separates roles that share one
instantiation and grid (the out-projection and FFN2).  Dispatches the log does not list (the resamplers' GEMMs
launch inside libhfa) stay unlabelled and are reported under their kernel name.

    python scripts/shape_table.py --trace DIR --log LOG.json [--pmc DIR --pmc-log LOG.json ...] [--csv OUT.csv]

Columns: role, shape (M x N x K x Z as launched), launches per step, average µs, ms per step, f32-equivalent
TF/s (2·M·N·K·Z per launch; attention 4·B·H·L²·d), fraction of the split-f16 ceiling (2516.6 / 3 TF/s) and, with
PMC passes: MFMA pipe busy (SQ_VALU_MFMA_BUSY_CYCLES over 1024 SIMDs x GRBM_GUI_ACTIVE/8 cycles), effective clock
(GRBM_GUI_ACTIVE / 8 / dispatch time) and SQ wait fractions.  The PMC dispatches are serialised by the profiler,
so their busy/clock figures are per kernel alone; the timing columns come from the unserialised trace.
"""
import argparse
import csv
import glob
import json
import os
from collections import defaultdict

SPLIT_PEAK = 2516.6 / 3
HIDDEN = {"cnhubert": (768, 3072), "cnhubert-large": (1024, 4096)}


def norm_name(n: str) -> str:
    n = n[5:] if n.startswith("void ") else n
    n = n.replace("(anonymous namespace)::", "")
    depth, out = 0, []
    for ch in n:                        # drop the argument list: the first top-level "("
        if ch == "<":
            depth += 1
        elif ch == ">":
            depth -= 1
        elif ch == "(" and depth == 0:
            break
        out.append(ch)
    return "".join(out).strip()


def matches(log_name: str, trace_name: str) -> bool:
    if "<" in log_name:
        return trace_name == log_name
    return trace_name.split("<")[0] == log_name


def role(entry, enc) -> str:
    name, shape = entry["name"], entry["shape"]
    if entry.get("label"):
        return entry["label"]
    if shape is None:
        return name
    if name.startswith("attn_fwd"):
        B, H, L, d = shape
        return f"attention (L={L}, {H} heads x {d})"
    M, N, K, Z = shape
    H, F = HIDDEN.get(enc, (768, 3072))
    if Z > 1 and N == 512:
        return f"extractor conv k{K // 512} ({M} frames)"
    if Z > 1 and N in (48, 64):
        return "positional conv (grouped)"
    if Z == 1:
        if N == H and K == 512:
            return "feature projection"
        if N == 3 * H and K == H:
            return "QKV projection"
        if N == H and K == H:
            return "attention out-projection (+res)"
        if N == F and K == H:
            return "FFN1 (GELU)"
        if N == H and K == F:
            return "FFN2 (+res)"
        if N < 128 and K == 192:
            return "head"
    return f"UNet GEMM N={N} K={K}" + (f" ({M} frames)" if Z > 1 else "")


def load_trace(d):
    fs = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
    if not fs:
        raise SystemExit(f"no kernel_trace.csv under {d}")
    disp = []
    for fn in fs:
        for r in csv.DictReader(open(fn)):
            disp.append({"id": int(r["Dispatch_Id"]), "name": norm_name(r["Kernel_Name"]),
                         "ns": int(r["End_Timestamp"]) - int(r["Start_Timestamp"])})
    disp.sort(key=lambda r: r["id"])
    return disp


def load_pmc(d):
    fs = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    disp = {}
    for fn in fs:
        for r in csv.DictReader(open(fn)):
            i = int(r["Dispatch_Id"])
            e = disp.setdefault(i, {"id": i, "name": norm_name(r["Kernel_Name"]),
                                    "ns": int(r["End_Timestamp"]) - int(r["Start_Timestamp"])})
            e[r["Counter_Name"]] = e.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    return sorted(disp.values(), key=lambda r: r["id"])


def pair(log_entries, disp):
    """Greedy in-order pairing of logged launches with dispatches of the same kernel family.  The log covers the
    last steps of the run, so the pairing starts near the tail of the dispatch list; a start that cannot pair the
    whole log is retried one candidate later.  Returns (pairs, unlogged dispatches of those families in between)."""
    fam = {e["name"].split("<")[0] for e in log_entries}
    cand = [r for r in disp if r["name"].split("<")[0] in fam]
    start = max(0, len(cand) - int(len(log_entries) * 1.5) - 64)
    for s in range(start, len(cand)):
        if not matches(log_entries[0]["name"], cand[s]["name"]):
            continue
        out, j, ok = [], s, True
        for e in log_entries:
            while j < len(cand) and not matches(e["name"], cand[j]["name"]):
                j += 1
            if j == len(cand):
                ok = False
                break
            out.append((e, cand[j]))
            j += 1
        if ok:
            used = {id(d) for _, d in out}
            lo, hi = out[0][1]["id"], out[-1][1]["id"]
            return out, [d for d in cand if lo <= d["id"] <= hi and id(d) not in used]
    raise SystemExit("could not pair the launch log with the dispatches")


def build(trace_dir, log_path, pmc_dirs=(), pmc_logs=()):
    lg = json.load(open(log_path))
    steps, enc = lg["steps"], lg["encoder"]
    entries = [e for e in lg["launches"] if e["shape"] is not None]
    pairs, extra = pair(entries, load_trace(trace_dir))
    agg = defaultdict(lambda: {"n": 0, "ns": 0, "work": 0.0, "kernels": set(), "shape": None, "pmc": {}})
    for e, d in pairs:
        g = agg[role(e, enc)]
        g["n"] += 1
        g["ns"] += d["ns"]
        g["work"] += e["work"]
        g["kernels"].add(d["name"])
        g["shape"] = e["shape"]
    for d in extra:
        g = agg["(unlogged) " + d["name"][:60]]
        g["n"] += 1
        g["ns"] += d["ns"]
        g["kernels"].add(d["name"])
    for pdir, plog in zip(pmc_dirs, pmc_logs):
        pl = json.load(open(plog))
        pe = [e for e in pl["launches"] if e["shape"] is not None]
        pp, _ = pair(pe, load_pmc(pdir))
        for e, d in pp:
            g = agg[role(e, enc)]["pmc"].setdefault(pdir, defaultdict(float))
            g["n"] += 1
            g["ns"] += d["ns"]
            for k, v in d.items():
                if k.startswith("SQ_") or k.startswith("GRBM_"):
                    g[k] += v
    rows = []
    for r, g in agg.items():
        per = g["n"] / steps
        avg_us = g["ns"] / max(g["n"], 1) / 1e3
        tf = g["work"] / (g["ns"] * 1e-9) / 1e12 if g["work"] else None
        row = {"role": r, "shape": "x".join(map(str, g["shape"])) if g["shape"] else "",
               "kernel": " | ".join(sorted(g["kernels"]))[:200], "launches_per_step": round(per, 2),
               "avg_us": round(avg_us, 1), "ms_per_step": round(per * avg_us / 1e3, 3),
               "tflops_f32eq": round(tf, 1) if tf else None,
               "frac_split_ceiling": round(tf / SPLIT_PEAK, 3) if tf else None}
        for p in g["pmc"].values():     # one PMC pass each; clock and busy from the pass that carried them
            if p.get("GRBM_GUI_ACTIVE"):
                cyc = p["GRBM_GUI_ACTIVE"] / 8.0
                row["clock_ghz"] = round(cyc / p["ns"], 3)
                if p.get("SQ_VALU_MFMA_BUSY_CYCLES"):
                    row["mfma_busy"] = round(p["SQ_VALU_MFMA_BUSY_CYCLES"] / (cyc * 1024.0), 3)
            if p.get("SQ_WAVE_CYCLES"):
                for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
                    if p.get(k):
                        row[k.lower().replace("sq_", "") + "_frac"] = round(p[k] / p["SQ_WAVE_CYCLES"], 3)
        rows.append(row)
    rows.sort(key=lambda r: -r["ms_per_step"])
    return {"steps": steps, "encoder": enc, "rows": rows}


COLS = ["role", "shape", "launches_per_step", "avg_us", "ms_per_step", "tflops_f32eq", "frac_split_ceiling",
        "mfma_busy", "clock_ghz", "wait_any_frac", "wait_inst_any_frac", "active_inst_any_frac", "kernel"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--trace", required=True)
    ap.add_argument("--log", required=True)
    ap.add_argument("--pmc", action="append", default=[])
    ap.add_argument("--pmc-log", action="append", default=[])
    ap.add_argument("--csv")
    ap.add_argument("--json")
    a = ap.parse_args()
    res = build(a.trace, a.log, a.pmc, a.pmc_log)
    print(" | ".join(COLS[:-1]))
    for r in res["rows"]:
        print(" | ".join(str(r.get(c, "")) for c in COLS[:-1]))
    if a.csv:
        with open(a.csv, "w", newline="") as f:
            w = csv.DictWriter(f, fieldnames=COLS)
            w.writeheader()
            for r in res["rows"]:
                w.writerow({c: r.get(c, "") for c in COLS})
    if a.json:
        with open(a.json, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
