"""Tile sweep for the config-3 step's two plain GEMMs (GPU box, not the
product): the src Linear (12032 x 640 -> 256, bias, fp32 out) and the stacked
linear_pos (751 x 256 -> 3072, bf16 out)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from speechbrain_amd import _enc  # noqa: E402
from scripts.kbench import timeit  # noqa: E402

dev = torch.device("cuda")
bf = torch.bfloat16
for (M, N, K, odt, bias) in ((12032, 256, 640, torch.float32, True), (751, 3072, 256, bf, False)):
    a = torch.randn(M, K, device=dev).to(bf)
    w = torch.randn(N, K, device=dev).to(bf)
    b = torch.randn(N, device=dev) if bias else None
    fl = 2.0 * M * N * K
    ref = _enc.gemm(a, w, bias=b, out_dtype=odt, tile=2).float()
    res = []
    for t in (0, 2, 1, 3, 4, 5, 6, 7, 8, 9, 10, 18, 19, 20, 21, 22):
        try:
            o = _enc.gemm(a, w, bias=b, out_dtype=odt, tile=t)
            err = float((o.float() - ref).abs().max() / ref.abs().max())
            us = timeit(lambda: _enc.gemm(a, w, bias=b, out_dtype=odt, tile=t), reps=50)
            res.append(f"t{t} {us:.2f}us {fl / us / 1e6:.0f}TF/s{'' if err < 1e-2 else ' BAD'}")
        except Exception as e:  # noqa: BLE001
            res.append(f"t{t} err")
    print(f"M={M} N={N} K={K}: " + " | ".join(res), flush=True)
