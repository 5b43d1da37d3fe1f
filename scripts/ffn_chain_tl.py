"""s_memtime timeline of the layer-chain FFN kernel (sbk_ffn_chain: FFN2 +
norm2 of layer i, FFN1 + norm1 + in_proj of layer i+1) for every wave of
workgroup 128 (probe build with -DSBK_PROBE_TL; never the product).
usage: scripts/probe_build.sh speechbrain_amd/csrc/ffn.hip TL &&
       SBK_PROBE_LIB=gpurun_probe_TL.so python scripts/ffn_chain_tl.py"""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import speechbrain_amd._lib as _L  # noqa: E402
_L.LIB_PATH = os.path.abspath(os.environ["SBK_PROBE_LIB"])
from speechbrain_amd import _enc  # noqa: E402

dev = torch.device("cuda")
D, H, M = 256, 1024, 12032
g = torch.Generator(device=dev).manual_seed(0)


def blk():
    w1 = _enc.cast_bf16((torch.randn(H, D, device=dev, generator=g) / 16).contiguous())
    w2 = _enc.cast_bf16((torch.randn(D, H, device=dev, generator=g) / 32).contiguous())
    ln = (torch.ones(D, device=dev), torch.zeros(D, device=dev), 1e-5)
    return ln, w1, torch.zeros(H, device=dev), w2, torch.zeros(D, device=dev), 0.5


la = blk() + (((torch.ones(D, device=dev), torch.zeros(D, device=dev), 1e-5)),)
lb = blk() + (None,)
wp = _enc.cast_bf16((torch.randn(3 * D, D, device=dev, generator=g) / 16).contiguous())
nl = (torch.ones(D, device=dev), torch.zeros(D, device=dev), 1e-5)
x = torch.randn(M, D, device=dev)
for _ in range(5):
    _enc.ffn_chain(x, la, lb, "swish", 0.0, nl, wp)
torch.cuda.synchronize()
buf = (ctypes.c_ulonglong * (16 * 256))()
lib = ctypes.CDLL(_L.LIB_PATH)
assert lib.sbk_probe_ffn_tl(buf) == 0
tl = np.array(buf, dtype=np.int64).reshape(16, 256)
t0 = tl[:8, 0].min()
rel = tl[:8] - t0
for w in range(8):
    r = rel[w]
    st = [r[3 + 2 * s] - r[2 + 2 * s] for s in range(76)]
    gaps = [r[2 + 2 * (s + 1)] - r[3 + 2 * s] for s in range(75)]
    print(f"w{w}: start {r[0]} loop {r[1]} | A steps {r[2]}..{r[3 + 2 * 31]} | between {r[197]} z {r[200]} "
          f"postLN {r[201]} LN0b {r[202]} bar {r[203]} ->{r[198]} | B steps {r[2 + 64]}..{r[3 + 2 * 63]} | "
          f"epi {r[194]} z {r[195]} nextLN {r[204]} xa {r[205]} proj-end {r[206]} | end {r[196]}")
    print(f"   step body  mean A {np.mean(st[:32]):.0f} B {np.mean(st[32:64]):.0f}; "
          f"gap mean {np.mean(gaps):.0f}; phase1/2 bodies {np.mean([st[s] for s in range(32) if s % 8 < 4]):.0f}"
          f"/{np.mean([st[s] for s in range(32) if s % 8 >= 4]):.0f}")
