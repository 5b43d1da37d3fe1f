"""Spectrum-kernel probe (GPU box, not part of the product): times the
STFT / power / Fbank modes at several batch sizes to separate per-block
latency from throughput."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import speechbrain_amd._lib as _L  # noqa: E402
if os.environ.get("SBK_PROBE_LIB"):
    _L.LIB_PATH = os.path.abspath(os.environ["SBK_PROBE_LIB"])  # probe builds of the kernel (not product)
from speechbrain_amd.lobes.features import Fbank  # noqa: E402
from speechbrain_amd.processing.features import STFT  # noqa: E402
from speechbrain_amd import ops  # noqa: E402
from scripts.kbench import timeit  # noqa: E402

dev = torch.device("cuda")
fb = Fbank(n_mels=80).to(dev)
st = STFT(sample_rate=16000).to(dev)
sizes = [int(sys.argv[1])] if len(sys.argv) > 1 else (1, 4, 32, 128)
for B in sizes:
    wav = torch.randn(B, 240000, device=dev) * 0.1
    t_fb = timeit(lambda: fb(wav), reps=20)
    t_st = timeit(lambda: st(wav), reps=20)
    t_pw = timeit(lambda: st.power_spectrum(wav), reps=20)
    print(f"B={B}: fbank {t_fb:.1f}us  stft {t_st:.1f}us  power {t_pw:.1f}us", flush=True)
