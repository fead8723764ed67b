"""Print a rocprofv3 kernel-stats CSV sorted by total time (name, calls, avg us, total ms)."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
tot = sum(float(r['TotalDurationNs']) for r in rows)
for r in sorted(rows, key=lambda r: -float(r['TotalDurationNs'])):
    print(f"{r['Name'][:72]:72s} {int(r['Calls']):6d} {float(r['AverageNs']) / 1e3:8.1f} {float(r['TotalDurationNs']) / 1e6:8.2f}")
print(f'total {tot / 1e6:.2f} ms')
