"""Host time of the config-2 step (Fbank(deltas) -> SpecAugment, eager): per-call
wall time of each module without device syncs, and a cProfile of 200 steps
(the step is host-paced when these exceed its kernels' ~105 us)."""
import cProfile
import os
import pstats
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from speechbrain_amd.lobes.augment import SpecAugment  # noqa: E402
from speechbrain_amd.lobes.features import Fbank  # noqa: E402

dev = torch.device("cuda")
fb = Fbank(sample_rate=16000, n_fft=400, n_mels=80, deltas=True).to(dev)
sa = SpecAugment(time_warp=True, time_warp_window=5, time_warp_mode="bicubic", freq_mask=True,
                 freq_mask_width=(0, 30), n_freq_mask=2, time_mask=True, time_mask_width=(0, 40), n_time_mask=2,
                 replace_with_zero=False)
wav = 0.1 * torch.randn(32, 240000, device=dev)
it = [0]


def step():
    torch.default_generator.manual_seed(1234 + it[0])
    it[0] += 1
    with torch.no_grad():
        return sa(fb(wav))


for _ in range(20):
    step()
torch.cuda.synchronize()
tf = ts = 0.0
n = 200
for _ in range(n):
    t0 = time.perf_counter()
    with torch.no_grad():
        y = fb(wav)
    t1 = time.perf_counter()
    with torch.no_grad():
        sa(y)
    t2 = time.perf_counter()
    tf += t1 - t0
    ts += t2 - t1
torch.cuda.synchronize()
print(f"host per call: Fbank(deltas) {tf / n * 1e6:.1f} us, SpecAugment {ts / n * 1e6:.1f} us")
t0 = time.perf_counter()
for _ in range(n):
    step()
torch.cuda.synchronize()
print(f"step wall (no sync inside): {(time.perf_counter() - t0) / n * 1e6:.1f} us")
pr = cProfile.Profile()
pr.enable()
for _ in range(n):
    step()
torch.cuda.synchronize()
pr.disable()
pstats.Stats(pr).sort_stats("tottime").print_stats(18)
