"""Average per-dispatch value of each counter for kernels whose name contains a
filter, from rocprofv3 --pmc CSV passes.  usage: pmc_summary.py <filter> <csv>..."""
import collections
import csv
import sys

flt = sys.argv[1]
for path in sys.argv[2:]:
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        if flt in r["Kernel_Name"]:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, v in sorted(agg.items()):
        print(f"{path.split('/')[-2]} {k:28s} n={len(v):3d} avg={sum(v) / len(v):14.1f}")
