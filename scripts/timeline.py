"""Per-stream busy time and idle gaps of one pipelined bench step from a rocprofv3 kernel trace (CPU).
python scripts/timeline.py TRACE_CSV [--anchor conv0_apply] -- takes the last complete step between two launches
of the anchor kernel (one per batch on the encoder stream) and reports, per stream, kernel time, gaps and the
largest kernels."""
import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
anchor = sys.argv[sys.argv.index("--anchor") + 1] if "--anchor" in sys.argv else "conv0_apply"
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
starts = [int(r["Start_Timestamp"]) for r in rows if anchor in r["Kernel_Name"]]
if len(starts) < 4:
    sys.exit("not enough anchor launches")
t0, t1 = starts[-4], starts[-3]          # a step well inside the timed region (bench's last steps are isolated)
print(f"step window {(t1 - t0) / 1e6:.3f} ms")
by_stream = defaultdict(list)
for r in rows:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    if e <= t0 or s >= t1:
        continue
    by_stream[(r["Queue_Id"], r["Stream_Id"])].append((max(s, t0), min(e, t1), r["Kernel_Name"]))
for key, ks in sorted(by_stream.items()):
    busy = sum(e - s for s, e, _ in ks)
    gaps, last = [], t0
    for s, e, n in ks:
        if s > last:
            gaps.append(s - last)
        last = max(last, e)
    print(f"queue {key[0]} stream {key[1]}: {len(ks)} kernels, busy {busy / 1e6:.3f} ms, gaps {sum(gaps) / 1e6:.3f} ms "
          f"(largest {max(gaps) / 1e3 if gaps else 0:.1f} us)")
    agg = defaultdict(float)
    for s, e, n in ks:
        n = n.replace("(anonymous namespace)::", "")
        agg[n.split("(")[0][:90]] += (e - s) / 1e3
    for n, us in sorted(agg.items(), key=lambda x: -x[1])[:int(sys.argv[sys.argv.index("--top") + 1]) if "--top" in sys.argv else 8]:
        print(f"    {us:8.1f} us  {n}")
