"""Fbank output of one library build on a fixed input, saved for a bitwise
comparison of probe builds (never the product).
usage: SBK_PROBE_LIB=... python scripts/fb_out.py <out.npy>"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import speechbrain_amd._lib as _L  # noqa: E402
if os.environ.get("SBK_PROBE_LIB"):
    _L.LIB_PATH = os.path.abspath(os.environ["SBK_PROBE_LIB"])
from speechbrain_amd.lobes.features import Fbank  # noqa: E402

dev = torch.device("cuda")
g = torch.Generator(device=dev).manual_seed(0)
outs = []
for B, S in ((32, 240000), (5, 170003), (3, 16000)):
    wav = torch.randn(B, S, device=dev, generator=g) * 0.1
    outs.append(Fbank(n_mels=80).to(dev)(wav).float().cpu().numpy().ravel())
np.save(sys.argv[1], np.concatenate(outs))
print("saved", sys.argv[1])
