"""Per-batch kernel time table from a rocprofv3 --stats kernel_stats.csv: python scripts/kstats.py CSV NBATCH"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
nb = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
tot = sum(float(r["TotalDurationNs"]) for r in rows)
for r in rows[:40]:
    n = r["Name"].replace("(anonymous namespace)::", "")[:100]
    print(f"{float(r['TotalDurationNs']) / nb / 1e3:9.1f} us/batch  calls/b {int(r['Calls']) / nb:6.1f}  "
          f"avg {float(r['AverageNs']) / 1e3:8.1f}  {n}")
print(f"{tot / nb / 1e6:.3f} ms kernel time per batch")
