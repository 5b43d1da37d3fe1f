"""Print the top kernels of a rocprofv3 kernel_stats.csv (share, calls, avg)."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 16
tot = sum(float(r["TotalDurationNs"]) for r in rows)
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:n]:
    print(f'{float(r["TotalDurationNs"]) / tot * 100:5.1f}% {int(r["Calls"]):5d} '
          f'{float(r["AverageNs"]) / 1000:8.1f}us  {r["Name"][:100]}')
print(f"{tot / 1e6:.2f} ms total")
