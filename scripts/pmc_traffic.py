"""Turn rocprofv3 PMC CSVs (FETCH_SIZE and WRITE_SIZE, collected in separate passes) into HBM bytes per launch
of one kernel, following MI355X_MICROARCH.md §HBM: FETCH_SIZE reads half the bytes of a wide coalesced
stream on gfx950 (x2 correction); WRITE_SIZE is exact for 16-B/lane stores and uncalibrated otherwise.

python scripts/pmc_traffic.py --fetch DIR --write DIR --kernel 'gemm_f32_kernel<1, true, 16, 128>' --out FILE
"""
import argparse
import csv
import glob
import json
import os


def per_dispatch(dirname, counter, kernel):
    files = glob.glob(os.path.join(dirname, "**", "*counter_collection.csv"), recursive=True)
    vals = {}
    for fn in files:
        for row in csv.DictReader(open(fn)):
            name = row.get("Kernel_Name", "")
            if kernel not in name or row.get("Counter_Name") != counter:
                continue
            key = row.get("Dispatch_Id") or row.get("Correlation_Id") or str(len(vals))
            vals[key] = vals.get(key, 0.0) + float(row["Counter_Value"])
    return list(vals.values())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--fetch", required=True)
    ap.add_argument("--write", required=True)
    ap.add_argument("--kernel", required=True)
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    f = per_dispatch(a.fetch, "FETCH_SIZE", a.kernel)
    w = per_dispatch(a.write, "WRITE_SIZE", a.kernel)
    if not f or not w:
        raise SystemExit(f"no dispatches of {a.kernel!r} found (fetch {len(f)}, write {len(w)})")
    fetch_kb = sum(f) / len(f)
    write_kb = sum(w) / len(w)
    res = {"kernel": a.kernel, "dispatches": [len(f), len(w)], "fetch_kb_raw": fetch_kb, "write_kb": write_kb,
           "bytes_per_launch": (2.0 * fetch_kb + write_kb) * 1024.0,
           "method": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE in separate passes; bytes = (2*FETCH_SIZE + "
                     "WRITE_SIZE) KiB per dispatch (gfx950 FETCH_SIZE half-count correction); WRITE_SIZE of 4-B/lane "
                     "stores is uncalibrated"}
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    with open(a.out, "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
