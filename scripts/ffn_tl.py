"""FFN s_memtime timeline of every wave of workgroup 128 (probe build with
-DSBK_PROBE_TL; never the product).
usage: SBK_PROBE_LIB=gpurun_probe_TL.so python scripts/ffn_tl.py"""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import speechbrain_amd._lib as _L  # noqa: E402
_L.LIB_PATH = os.path.abspath(os.environ["SBK_PROBE_LIB"])
from speechbrain_amd.nnet.attention import PositionalwiseFeedForward  # noqa: E402
from speechbrain_amd.nnet.activations import Swish  # noqa: E402

dev = torch.device("cuda")
D, H, M = 256, 1024, 12032
ffn = PositionalwiseFeedForward(H, input_size=D, activation=Swish).to(dev).eval()
x = torch.randn(M, D, device=dev)
ln = (torch.ones(D, device=dev), torch.zeros(D, device=dev), 1e-5)
with torch.no_grad():
    for _ in range(5):
        ffn.run_fused(x, ln, 0.5, next_ln=ln)
torch.cuda.synchronize()
buf = (ctypes.c_ulonglong * (16 * 80))()
lib = ctypes.CDLL(_L.LIB_PATH)
assert lib.sbk_probe_ffn_tl(buf) == 0
tl = np.array(buf, dtype=np.int64).reshape(16, 80)
t0 = tl[:, 0].min()
rel = tl - t0
print("per wave: start, loop start (1), step-s barrier exits (2+2s) and step ends (3+2s), loop end (70), end (72)")
for w in range(16):
    r = rel[w]
    steps = [f"{r[2 + 2 * s]:6d}/{r[3 + 2 * s] - r[2 + 2 * s]:5d}" for s in range(16)]
    print(f"w{w:2d} st {r[0]:5d} L {r[1]:6d} " + " ".join(steps) + f" | end loop {r[70]:6d} end {r[72]:6d}")
