"""Compare the encoder stream's kernels of one pipelined step between two rocprof kernel traces (CPU):
python scripts/pipe_cmp.py TRACE_A TRACE_B [--anchor conv0_apply].  Takes the second-to-last complete step of
each (anchor = one launch per batch on the encoder stream), matches encoder-stream kernels by order, and prints
the largest per-kernel differences, grouped by kernel name, plus what the other stream ran meanwhile."""
import csv
import sys
from collections import defaultdict


def step(path, anchor):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    starts = [i for i, r in enumerate(rows) if anchor in r["Kernel_Name"]]
    a, b = starts[-3], starts[-2]
    enc_q = (rows[a]["Queue_Id"], rows[a]["Stream_Id"])
    t0, t1 = int(rows[a]["Start_Timestamp"]), int(rows[b]["Start_Timestamp"])
    enc, side = [], []
    for r in rows:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if s < t0 or s >= t1:
            continue
        n = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0][:80]
        (enc if (r["Queue_Id"], r["Stream_Id"]) == enc_q else side).append((s - t0, e - s, n))
    return (t1 - t0), enc, side


anchor = sys.argv[sys.argv.index("--anchor") + 1] if "--anchor" in sys.argv else "conv0_apply"
sa, ea, za = step(sys.argv[1], anchor)
sb, eb, zb = step(sys.argv[2], anchor)
print(f"step A {sa / 1e6:.3f} ms ({len(ea)} encoder kernels, {len(za)} side), "
      f"step B {sb / 1e6:.3f} ms ({len(eb)} encoder kernels, {len(zb)} side)")
print(f"encoder busy A {sum(d for _, d, _ in ea) / 1e6:.3f} ms, B {sum(d for _, d, _ in eb) / 1e6:.3f} ms; "
      f"side busy A {sum(d for _, d, _ in za) / 1e6:.3f} ms, B {sum(d for _, d, _ in zb) / 1e6:.3f} ms")
diff = defaultdict(float)
for (s1, d1, n1), (s2, d2, n2) in zip(ea, eb):
    diff[n1] += (d2 - d1) / 1e3
for n, us in sorted(diff.items(), key=lambda x: -abs(x[1]))[:12]:
    print(f"  {us:+8.1f} us  {n}")
for name, z in (("A", za), ("B", zb)):
    print(f"side stream {name}:")
    for s, d, n in z[:6] + ([] if len(z) <= 6 else [(0, 0, "...")]):
        print(f"  {s / 1e3:8.1f} {d / 1e3:8.1f}  {n}")
    if len(z) > 6:
        s, d, n = z[-1]
        print(f"  {s / 1e3:8.1f} {d / 1e3:8.1f}  {n} (last)")
# encoder kernels overlapped by the side stream in B: per kernel, A vs B durations for the first 40
print("encoder kernels, step order: start_A dur_A | dur_B  name")
for (s1, d1, n1), (s2, d2, n2) in list(zip(ea, eb))[:60]:
    print(f"  {s1 / 1e3:8.1f} {d1 / 1e3:7.1f} | {d2 / 1e3:7.1f}  {n1}")
