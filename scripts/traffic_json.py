"""Turn a FETCH_SIZE/WRITE_SIZE counter CSV into profiles/pmc_traffic.json:
HBM bytes per launch per kernel (FETCH_SIZE x 2: on gfx950 it reports half
the bytes of wide streaming reads, MI355X_MICROARCH.md §HBM; both in KB).
An existing <out.json> is updated, not replaced: one config's passes must not
drop the other configs' kernels (the bench lines look them up by name).
    python scripts/traffic_json.py <fetch.csv> <write.csv> <out.json>"""
import os
import collections
import csv
import json
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1]))) + list(csv.DictReader(open(sys.argv[2])))
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for r in rows:
    m = re.search(r"namespace\)::(\w+)(<[^()]*>)?", r["Kernel_Name"])
    name = (m.group(1) + (m.group(2) or "")) if m else r["Kernel_Name"][:60]
    acc[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
out = {}
for k, d in acc.items():
    if "FETCH_SIZE" in d and "WRITE_SIZE" in d:
        f = sum(d["FETCH_SIZE"]) / len(d["FETCH_SIZE"]) * 1024 * 2
        w = sum(d["WRITE_SIZE"]) / len(d["WRITE_SIZE"]) * 1024
        out[k] = int(f + w)
        print(f"{k:60s} read {f / 1e6:9.2f} MB  write {w / 1e6:9.2f} MB")
merged = {}
if os.path.exists(sys.argv[3]):
    with open(sys.argv[3]) as f:
        merged = json.load(f)
merged.update(out)
json.dump(merged, open(sys.argv[3], "w"), indent=1, sort_keys=True)
