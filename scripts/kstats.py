"""Summarize a rocprofv3 kernel_stats.csv: python scripts/kstats.py <csv> [n]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 20
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:n]:
    print(f"{r['Name'][:60]:60s} calls={r['Calls']:>5} avg={float(r['AverageNs']) / 1e3:10.1f}us "
          f"total={float(r['TotalDurationNs']) / 1e6:9.2f}ms {float(r['Percentage']):5.1f}%")
