"""s_memtime timeline of the Fbank spectrum kernel: per-workgroup phase marks
(wave 0) of every workgroup at config 3's batch (probe build with
-DSBK_PROBE_TL; never the product).
usage: scripts/probe_build.sh speechbrain_amd/csrc/features.hip TL &&
       SBK_PROBE_LIB=gpurun_probe_TL.so python scripts/spec_tl.py"""
import collections
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import speechbrain_amd._lib as _L  # noqa: E402
_L.LIB_PATH = os.path.abspath(os.environ["SBK_PROBE_LIB"])
from speechbrain_amd.lobes.features import Fbank  # noqa: E402

dev = torch.device("cuda")
fb = Fbank(n_mels=80).to(dev)
wav = torch.randn(int(sys.argv[1]) if len(sys.argv) > 1 else 32, 240000, device=dev) * 0.1
for _ in range(5):
    fb(wav)
torch.cuda.synchronize()
buf = (ctypes.c_ulonglong * (8192 * 8))()
assert ctypes.CDLL(_L.LIB_PATH).sbk_probe_spec_tl(buf) == 0
a = np.frombuffer(buf, dtype=np.uint64).reshape(8192, 8).astype(np.int64)
n = int((a[:, 5] > 0).sum())
a = a[:n]
t0 = a[:, 0].min()
st, en = a[:, 0] - t0, a[:, 5] - t0
print(f"workgroups {n}: kernel span {en.max()} cycles (s_memtime)")
dur = en - st
ph = np.diff(a[:, :6], axis=1)
print("per-WG duration mean %.0f p10 %.0f p50 %.0f p90 %.0f" % (dur.mean(), *np.percentile(dur, [10, 50, 90])))
for i, nm in enumerate(["loads+stage0", "stages1..", "split", "mel", "max+end"]):
    print(f"  {nm:14s} mean {ph[:, i].mean():8.0f}  p50 {np.median(ph[:, i]):8.0f}  p90 {np.percentile(ph[:, i], 90):8.0f}")
hw = a[:, 6]
cu = ((hw >> 32) & 0xFF) * 1000 + ((hw >> 13) & 7) * 100 + ((hw >> 12) & 1) * 20 + ((hw >> 8) & 0xF)
per = collections.Counter(cu.tolist())
print("CUs used", len(per), "workgroups per CU min/max", min(per.values()), max(per.values()))
wg = (hw >> 40) & 0xFFFFFF
print("workgroups", len(set(wg.tolist())))
# concurrency: how many WGs of one CU overlap in time
c0 = max(per, key=per.get)
idx = np.where(cu == c0)[0]
ev = sorted([(st[i], 1) for i in idx] + [(en[i], -1) for i in idx])
cur = mx = 0
for _, d in ev:
    cur += d
    mx = max(mx, cur)
print(f"busiest CU {c0}: {len(idx)} WGs, max concurrent {mx}, first start {st[idx].min()} last end {en[idx].max()}")
# start-time histogram over the kernel (10 bins)
h, _ = np.histogram(st, bins=10, range=(0, en.max()))
print("WG starts per tenth of the span:", h.tolist())
