"""Debug MXFP8-output mode of sbk_mx_gemm256 vs sbk_mx_gemm (GPU box)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from speechbrain_amd import _w2v  # noqa: E402
from speechbrain_amd._lib import lib  # noqa: E402
from scripts.mx256_bench import call  # noqa: E402

dev = torch.device("cuda")
L = lib()
M, N, K = int(sys.argv[1]), 256, 256
bias = torch.randn(N, device=dev)
torch.manual_seed(1)
a = _w2v.mx_quant((torch.rand(M, K, device=dev) * 2 - 1))
w = _w2v.mx_quant((torch.rand(N, K, device=dev) * 2 - 1))
ref, _ = call(L.sbk_mx_gemm, a, w, M, N, K, 0, bias, 4)
for fn in (L.sbk_mx_gemm, L.sbk_mx_gemm256):
    o, s = call(fn, a, w, M, N, K, 2, bias, 4)
    d = _w2v.mx_dequant(_w2v.MX(o, s))
    err = (d - ref).abs() / ref.abs().clamp(min=1e-3)
    print("max rel err", float(err.max()), "scales[0,:8]", s[0, :8].tolist(), "q[0,:8]", o[0, :8].tolist(), flush=True)
o0, s0 = call(L.sbk_mx_gemm, a, w, M, N, K, 2, bias, 4)
o1, s1 = call(L.sbk_mx_gemm256, a, w, M, N, K, 2, bias, 4)
print("scale mismatches", int((s0 != s1).sum()), "of", s0.numel(), " byte mismatches", int((o0 != o1).sum()))
idx = (o0 != o1).nonzero()[:10].tolist()
print("first mismatches", idx, [(int(o0[i, j]), int(o1[i, j])) for i, j in idx])
