"""HBM bytes per `mx_gemm` call of the config-5 step (the bench line's
roofline.traffic) from the FETCH_SIZE / WRITE_SIZE passes of
scripts/pmc_traffic.sh --config c5: the MXFP8 GEMM launches of one encoder
layer — QKV (bf16 out), out_proj and FFN2 (fp32 out + residual; FFN2's split
tail is its whole-tile launch, the K-half launch and splitk_epi_kernel), FFN1
(GELU, MXFP8 out) — summed, averaged over the layer's four calls (FETCH_SIZE
x 2 as in scripts/traffic_json.py), and written to pmc_traffic.json as
"mx_gemm".  Prints the per-(kernel, grid) table it used.
    python scripts/mx_gemm_traffic.py <fetch.csv> <write.csv> <pmc_traffic.json>"""
import collections
import csv
import json
import re
import sys


def per_launch(path, scale):
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        m = re.search(r"namespace\)::(\w+)(<[^()]*>)?", r["Kernel_Name"])
        name = (m.group(1) + (m.group(2) or "")) if m else r["Kernel_Name"][:60]
        acc[(name, int(r["Grid_Size"]))].append(float(r["Counter_Value"]) * 1024 * scale)
    return {k: (sum(v) / len(v), len(v)) for k, v in acc.items()}


fetch, write = per_launch(sys.argv[1], 2), per_launch(sys.argv[2], 1)
for k in sorted(fetch, key=lambda k: -fetch[k][0] * fetch[k][1]):
    if k in write:
        print(f"{k[0][:44]:44s} grid {k[1]:>9d} x{fetch[k][1]:5d}  read {fetch[k][0] / 1e6:8.1f} MB  "
              f"write {write[k][0] / 1e6:8.1f} MB")
# one layer's launches, by (kernel, grid in threads) at M = 23,936 rows
layer = {"QKV": [("gemm256_kernel<true, 0, 1>", 577536)],
         "out_proj": [("gemm256_kernel<true, 0, 0>", 192512)],
         "FFN1": [("gemm256_kernel<true, 4, 2>", 770048)],
         "FFN2": [("gemm256_kernel<true, 0, 0>", 131072), ("gemm256_kernel<true, 0, 0>", 122880),
                  ("splitk_epi_kernel<0>", 491520)]}
total = 0.0
for call, ks in layer.items():
    b = sum(fetch[k][0] + write[k][0] for k in ks)
    total += b
    print(f"{call:9s} {b / 1e6:8.1f} MB per call")
avg = total / len(layer)
print(f"mx_gemm: {avg / 1e6:.1f} MB per call (mean of the layer's four)")
with open(sys.argv[3]) as f:
    merged = json.load(f)
merged["mx_gemm"] = int(avg)
json.dump(merged, open(sys.argv[3], "w"), indent=1, sort_keys=True)
