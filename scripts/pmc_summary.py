"""Summarise a rocprofv3 --pmc counter_collection.csv per kernel (mean per dispatch)."""
import collections
import csv
import re
import sys


def short(name):
    m = re.search(r"namespace\)::(\w+)(<[^()]*>)?", name)
    if m:
        return m.group(1) + (m.group(2) or "")[:40]
    return name[:60]


rows = list(csv.DictReader(open(sys.argv[1])))
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for r in rows:
    agg[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in agg.items():
    if len(sys.argv) > 2 and sys.argv[2] not in k:
        continue
    print(k)
    for c, v in sorted(d.items()):
        print(f"   {c:28s} {sum(v) / len(v):14.1f}  (n={len(v)})")
