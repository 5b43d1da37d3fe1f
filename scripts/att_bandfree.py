"""Band vs band-free attention kernel times (GPU box, not the product):
the rel-pos LDS-DMA kernel and its band-free (MultiheadAttention) variant at
the config-3 shape (B=32, T=376, H=4) and the config-5 shape (B=32, T=748,
H=16); dh = 64, bf16, ragged key padding."""
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from speechbrain_amd import _enc  # noqa: E402
from scripts.kbench import timeit  # noqa: E402

dev = torch.device("cuda")
for B, T, H in [(32, 376, 4), (32, 748, 16)]:
    dh = 64
    qkv = (torch.randn(B * T, 3 * H * dh, device=dev) * 0.5).to(torch.bfloat16)
    lens = torch.randint(T // 2, T + 1, (B,))
    lens[0] = T
    kpm = (torch.arange(T)[None] >= lens[:, None]).to(torch.uint8).to(dev)
    pk = (torch.randn(2 * T - 1, H * dh, device=dev) * 0.5).to(torch.bfloat16)
    pb = torch.randn(dh, H, device=dev) * 0.1
    sc = 1.0 / math.sqrt(dh)
    t_band = timeit(lambda: _enc.relpos_attention(qkv, pk, pb, pb, kpm, B, T, H, dh, sc))
    t_free = timeit(lambda: _enc.mha_attention(qkv, kpm, B, T, H, dh, sc))
    fl = 4.0 * B * H * T * T * dh
    print(f"B={B} T={T} H={H}: band {t_band:.1f} us ({1.5 * fl / t_band / 1e6:.0f} TF/s incl. band), "
          f"band-free {t_free:.1f} us ({fl / t_free / 1e6:.0f} TF/s)", flush=True)
