"""Conv-module kernel s_memtime phase timeline (probe build -DSBK_PROBE_TL; never the product)."""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import speechbrain_amd._lib as _L  # noqa: E402
_L.LIB_PATH = os.path.abspath(os.environ["SBK_PROBE_LIB"])
from speechbrain_amd.lobes.models.transformer.Conformer import ConvolutionModule  # noqa: E402

dev = torch.device("cuda")
B, T = 32, 376
cm = ConvolutionModule(256, 31).to(dev).eval()
x = torch.randn(B * T, 256, device=dev)
pre = None
if os.environ.get("CM_PRE"):  # the encoder's variant: MHSA out_proj + residual fused in (phase -1)
    pre = ((torch.randn(B * T, 256, device=dev) * 0.5).to(torch.bfloat16),
           (torch.randn(256, 256, device=dev) / 16).to(torch.bfloat16), torch.zeros(256, device=dev))
with torch.no_grad():
    for _ in range(5):
        cm.run_fused(x, B, T, None, pre=pre)
torch.cuda.synchronize()
buf = (ctypes.c_ulonglong * 128)()
assert ctypes.CDLL(_L.LIB_PATH).sbk_probe_cm_tl(buf) == 0
tl = np.array(buf, dtype=np.int64).reshape(16, 8)  # the 16 waves of workgroup 100
base = tl[:, 0].min()
print("per wave, cycles from the workgroup's first mark: start | o staged (6) | x_att (7) | LN0 done (1) | P1 (2) | P2a (3) | P2b (4) | end (5)")
for w, r in enumerate(tl):
    print(f"w{w:2d}: " + " | ".join(f"{int(r[k] - base):6d}" for k in (0, 6, 7, 1, 2, 3, 4, 5)))
