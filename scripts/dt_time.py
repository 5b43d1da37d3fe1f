"""Per-call time of sbk_deltas_floor at config 2 (32 x 1501 x 80 -> 240,
window 5, deferred top_db floor) for one library build; A/B of probe builds
(never the product).  usage: SBK_PROBE_LIB=... python scripts/dt_time.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import speechbrain_amd._lib as _L  # noqa: E402
if os.environ.get("SBK_PROBE_LIB"):
    _L.LIB_PATH = os.path.abspath(os.environ["SBK_PROBE_LIB"])
from speechbrain_amd import ops  # noqa: E402
from scripts.kbench import timeit  # noqa: E402

dev = torch.device("cuda")
N, T, F = 32, 1501, 80
x = torch.randn(N, T, F, device=dev) * 10 - 40
nslot = (T + 7) // 8
sm = torch.randn(N, nslot, device=dev)
us = timeit(lambda: ops.deltas_floor(x, 5, sm, 80.0), reps=50)
y = ops.deltas_floor(x, 5, sm, 80.0)
print(f"{us:7.2f} us/call  {(N * T * F * 4 * 4) / us / 1e3:7.0f} GB/s algorithmic  checksum {float(y.double().abs().sum()):.6e}")
