"""Print a rocprofv3 kernel_stats.csv as 'avg_us calls share name' lines (top N)."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 25
tot = sum(float(r["TotalDurationNs"]) for r in rows)
for r in rows[:n]:
    print(f"{float(r['AverageNs']) / 1e3:8.1f} us {int(r['Calls']):4d} {float(r['TotalDurationNs']) / tot * 100:5.1f}%  {r['Name'][:110]}")
print(f"total {tot / 1e3:.1f} us")
