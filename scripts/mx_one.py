"""One MXFP8 GEMM shape launched N times (for rocprofv3 --pmc passes)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from speechbrain_amd import _w2v  # noqa: E402

M, N, K = (int(v) for v in (sys.argv[1:4] if len(sys.argv) > 3 else (23936, 4096, 1024)))
dev = torch.device("cuda:0")
x = _w2v.mx_quant(torch.randn(M, K, device=dev))
w = _w2v.mx_quant(torch.randn(N, K, device=dev) * 0.03)
for _ in range(10):
    _w2v.mx_gemm(x, w)
torch.cuda.synchronize()
print("done", flush=True)
