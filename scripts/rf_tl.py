"""s_memtime timeline of the register-FFT spectrum kernel (spec_reg_kernel):
per-wave phase marks of every wave at config 3's batch (probe build with
-DSBK_PROBE_TL; never the product).
usage: scripts/probe_build.sh speechbrain_amd/csrc/features.hip TL &&
       SBK_PROBE_LIB=gpurun_probe_TL.so python scripts/rf_tl.py"""
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
wav = torch.randn(32, 240000, device=dev) * 0.1
for _ in range(5):
    fb(wav)
torch.cuda.synchronize()
buf = (ctypes.c_ulonglong * (16384 * 8))()
assert ctypes.CDLL(_L.LIB_PATH).sbk_probe_rf_tl(buf) == 0
a = np.frombuffer(buf, dtype=np.uint64).reshape(16384, 8).astype(np.int64)
live = a[:, 7] > 0
a = a[live]
t0 = a[:, 0].min()
st, en = a[:, 0] - t0, a[:, 7] - t0
print(f"waves {len(a)}: kernel span {en.max()} cycles (s_memtime)")
dur = en - st
print("per-wave duration mean %.0f p10 %.0f p50 %.0f p90 %.0f" % (dur.mean(), *np.percentile(dur, [10, 50, 90])))
ph = np.diff(a, axis=1)
for i, nm in enumerate(["tables", "loads", "dft25+tw", "pass A", "pass B", "P write", "mel+end"]):
    print(f"  {nm:10s} mean {ph[:, i].mean():8.0f}  p50 {np.median(ph[:, i]):8.0f}  p90 {np.percentile(ph[:, i], 90):8.0f}")
h, _ = np.histogram(st, bins=10, range=(0, en.max()))
print("wave starts per tenth of the span:", h.tolist())
