"""s_memtime timeline of the 4 waves of tile 200 of relpos_flash_dma_kernel
(probe build with -DSBK_PROBE_TL; never the product).
usage: SBK_PROBE_LIB=gpurun_probe_TL.so python scripts/att_dma_tl.py"""
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
B, T, H, dh = 32, 376, 4, 64
d = H * dh
qkv = torch.randn(B * T, 3 * d, device=dev).to(torch.bfloat16)
pk = torch.randn(2 * T - 1, d, device=dev).to(torch.bfloat16)
u = torch.randn(H * dh, device=dev)
v = torch.randn(H * dh, device=dev)
for _ in range(5):
    _enc.relpos_attention(qkv, pk, u, v, None, B, T, H, dh, 1 / 16.0)
torch.cuda.synchronize()
s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
s.record()
for _ in range(50):
    _enc.relpos_attention(qkv, pk, u, v, None, B, T, H, dh, 1 / 16.0)
e.record()
torch.cuda.synchronize()
print(f"avg {s.elapsed_time(e) / 50 * 1e3:.2f} us per launch (probe build)")
buf = (ctypes.c_ulonglong * 256)()
assert ctypes.CDLL(_L.LIB_PATH).sbk_probe_att_tl(buf) == 0
tl = np.array(buf, dtype=np.int64).reshape(4, 64)
print("per chunk (memtime ticks): barA-wait->S/G+Gwrite | barB wait | softmax | PV | ->next barA")
for w in range(4):
    r = tl[w]
    parts = []
    for ch in range(6):
        b = 1 + 5 * ch
        nxt = r[b + 5] if ch < 5 else r[62]
        parts.append(f"{r[b+1]-r[b]:5d} {r[b+2]-r[b+1]:5d} {r[b+3]-r[b+2]:5d} {r[b+4]-r[b+3]:5d} {nxt-r[b+4]:5d}")
    print(f"w{w} pre {r[1]-r[0]:5d} | " + " | ".join(parts) + f" | total {r[62]-r[0]}")

# per-workgroup start / end of the last launch: rounds of residency and the clock
wg = (ctypes.c_ulonglong * (4096 * 4))()
assert ctypes.CDLL(_L.LIB_PATH).sbk_probe_att_wg(wg) == 0
a = np.array(wg, dtype=np.int64).reshape(4096, 4)[: B * H * ((T + 63) // 64)]
rt0, rt1, mt0, mt1 = a[:, 0], a[:, 1], a[:, 2], a[:, 3]
t0 = rt0.min()
life_us = (rt1 - rt0) / 100.0  # memrealtime: 100 MHz
print(f"workgroups {len(a)}: launch span {(rt1.max() - t0) / 100.0:.2f} us; life us min/med/max "
      f"{life_us.min():.2f}/{np.median(life_us):.2f}/{life_us.max():.2f}")
print(f"memtime ticks per us (median): {np.median((mt1 - mt0) / np.maximum(life_us, 1e-3)):.0f}")
st = (rt0 - t0) / 100.0
print("start-time histogram (us):", np.histogram(st, bins=10)[0].tolist(), "edges",
      np.round(np.histogram(st, bins=10)[1], 2).tolist())
nwg, nqb = len(a), (T + 63) // 64
orig = np.arange(nwg)
xcd, q8, r8 = orig & 7, nwg >> 3, nwg & 7
tile = np.where(xcd < r8, xcd * (q8 + 1), r8 * (q8 + 1) + (xcd - r8) * q8) + (orig >> 3)
qb = tile % nqb
for k in range(nqb):
    print(f"qb {k}: life median {np.median(life_us[qb == k]):.2f} max {life_us[qb == k].max():.2f}")
for k in range(8):
    print(f"xcd {k}: life median {np.median(life_us[xcd == k]):.2f} max {life_us[xcd == k].max():.2f}")
end = (rt1 - t0) / 100.0
print("end-time histogram (us):", np.histogram(end, bins=10)[0].tolist(), "edges",
      np.round(np.histogram(end, bins=10)[1], 2).tolist())
os.makedirs("gpurun_out", exist_ok=True)
np.save("gpurun_out/att_wg.npy", a)
