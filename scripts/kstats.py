"""Summarize a rocprofv3 kernel_stats.csv (top kernels by total time)."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 25
tot = sum(float(r["TotalDurationNs"]) for r in rows)
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:n]:
    print(f"{r['Name'][:80]:80s} calls={r['Calls']:>6} total_ms={float(r['TotalDurationNs'])/1e6:8.2f} "
          f"avg_us={float(r['AverageNs'])/1e3:8.2f} pct={float(r['TotalDurationNs'])/tot*100:6.2f}")
