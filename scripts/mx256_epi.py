"""Epilogue cost of the 256-tile MXFP8 GEMM on config 5's FFN1 / FFN2 shapes:
device time per call for act (none / GELU) x out (fp32 / bf16 / MXFP8), by
graph replay (GPU box, not the product)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from speechbrain_amd import _w2v  # noqa: E402
from speechbrain_amd._lib import lib  # noqa: E402
from scripts.kbench import timeit  # noqa: E402
from scripts.mx256_bench import call  # noqa: E402

dev = torch.device("cuda")
L = lib()
for (M, N, K, tag) in ((23936, 4096, 1024, "ffn1"), (23936, 1024, 4096, "ffn2"), (23936, 3072, 1024, "in_proj")):
    a = _w2v.mx_quant((torch.rand(M, K, device=dev) * 2 - 1))
    w = _w2v.mx_quant((torch.rand(N, K, device=dev) * 2 - 1))
    bias = torch.randn(N, device=dev)
    fl = 2.0 * M * N * K
    line = f"{tag:8s} M={M} N={N} K={K}:"
    for act in (0, 4):
        for mode in (0, 1, 2):
            us = timeit(lambda: call(L.sbk_mx_gemm256, a, w, M, N, K, mode, bias, act), reps=20)
            line += f" a{act}/o{mode} {us:7.1f}us {fl / us / 1e6:5.0f}TF"
    print(line, flush=True)
