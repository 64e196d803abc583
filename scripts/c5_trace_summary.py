"""Per-stream kernel time and the largest kernels of a rocprof kernel trace, over the window between the first and
last launch of an anchor kernel (CPU): python scripts/c5_trace_summary.py TRACE_CSV [anchor]"""
import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
anchor = sys.argv[2] if len(sys.argv) > 2 else "conv0_apply"
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if anchor in r["Kernel_Name"]]
t0, t1 = int(rows[idx[-3]]["Start_Timestamp"]), int(rows[idx[-2]]["Start_Timestamp"])
print(f"window between the last anchors but one: {(t1 - t0) / 1e6:.3f} ms")
by = defaultdict(list)
for r in rows:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    if s < t0 or s >= t1:
        continue
    by[(r["Queue_Id"], r.get("Stream_Id", ""))].append((s, e, r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0][:80]))
for k, ks in by.items():
    busy = sum(e - s for s, e, _ in ks)
    span = (max(e for _, e, _ in ks) - min(s for s, _, _ in ks)) / 1e6
    print(f"queue {k}: {len(ks)} kernels, busy {busy / 1e6:.3f} ms over {span:.3f} ms "
          f"(first at +{(ks[0][0] - t0) / 1e6:.3f} ms)")
    agg = defaultdict(float)
    for s, e, n in ks:
        agg[n] += (e - s) / 1e6
    for n, ms in sorted(agg.items(), key=lambda x: -x[1])[:8]:
        print(f"   {ms:8.3f} ms  {n}")
