"""Tile sweep for the training-path GEMM shapes (GPU box, not the product):
dX = dY W (sbk_gemm, every tile variant) and dW = dY^T X (sbk_gemm_tn), with
torch.mm (hipBLASLt) beside them as a reference point."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from speechbrain_amd import _enc  # noqa: E402
from scripts.kbench import timeit  # noqa: E402

dev = torch.device("cuda")
bf = torch.bfloat16
M = 12032
for N, K in ((1024, 256), (256, 1024), (256, 256), (512, 256), (768, 256)):
    a = torch.randn(M, K, device=dev).to(bf)
    w = torch.randn(N, K, device=dev).to(bf)
    fl = 2.0 * M * N * K
    res = [f"lib {fl / timeit(lambda: torch.mm(a, w.t()), reps=20) / 1e6:.0f}"]
    for t in (2, 1, 3, 7, 8, 9, 10, 18, 19, 20, 21, 22):
        try:
            us = timeit(lambda: _enc.gemm(a, w, out_dtype=bf, tile=t), reps=20)
            res.append(f"t{t} {fl / us / 1e6:.0f}")
        except Exception as e:  # noqa: BLE001
            res.append(f"t{t} err")
    print(f"dX M={M} N={N} K={K} TF/s: " + "  ".join(res), flush=True)
from speechbrain_amd._lib import lib, ptr, stream_of  # noqa: E402
for Mw, Nw in ((1024, 256), (256, 1024), (256, 256), (512, 256), (768, 256)):
    dy = torch.randn(M, Mw, device=dev).to(bf)
    x = torch.randn(M, Nw, device=dev).to(bf)
    fl = 2.0 * M * Mw * Nw
    c = torch.zeros(Mw, Nw, device=dev)
    res = []
    for tile in (64, 128):
        for ns in (0, 1, 2, 4, 8, 16, 32):
            f = lambda: lib().sbk_gemm_tn_cfg(ptr(dy), Mw, 0, ptr(x), Nw, 0, Mw, Nw, M, 1, ptr(c), Nw, 0, tile, ns,  # noqa
                                              stream_of(dy))
            us = timeit(f, reps=20)
            res.append(f"t{tile}/s{ns} {us:.1f}")
    ul = timeit(lambda: torch.mm(dy.t(), x), reps=20)
    print(f"dW {Mw}x{Nw} K={M} us: " + "  ".join(res) + f"  lib {ul:.1f}", flush=True)
