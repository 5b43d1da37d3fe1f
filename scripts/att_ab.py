"""A/B of the encoder's rel-pos attention kernels (sbk_attention_variant 1:
4 waves x 16 queries, 2: 2 waves x 32 queries) at config 3's shape and a
few ragged T: outputs compared bitwise, device time per call interleaved in
one process (GPU box, not the product)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from speechbrain_amd import _enc  # noqa: E402
from speechbrain_amd._lib import lib  # noqa: E402
from scripts.kbench import timeit  # noqa: E402

dev = torch.device("cuda")
bf = torch.bfloat16
L = lib()
torch.manual_seed(0)
for (B, T, band) in ((32, 376, True), (32, 376, False), (3, 37, True), (2, 97, True), (2, 640, True), (1, 2200, True)):
    H, dh = 4, 64
    qkv = torch.randn(B * T, 3 * H * dh, device=dev).to(bf)
    pk = torch.randn(2 * T - 1, H * dh, device=dev).to(bf)
    pbu, pbv = torch.randn(H * dh, device=dev), torch.randn(H * dh, device=dev)
    kpm = (torch.arange(T, device=dev)[None, :] >= torch.randint(T // 2, T + 1, (B,), device=dev)[:, None])
    kpm = kpm.to(torch.uint8).contiguous()
    sc = 1.0 / 16

    def run():
        if band:
            return _enc.relpos_attention(qkv, pk, pbu, pbv, kpm, B, T, H, dh, sc)[0]
        return _enc.mha_attention(qkv, kpm, B, T, H, dh, 0.125)

    outs, times = {}, {1: [], 2: []}
    for v in (1, 2):
        L.sbk_attention_variant(v)
        outs[v] = run().clone()
    for _ in range(3):
        for v in (1, 2):
            L.sbk_attention_variant(v)
            times[v].append(timeit(run, reps=20))
    L.sbk_attention_variant(2)
    eq = torch.equal(outs[1], outs[2])
    d = float((outs[1].float() - outs[2].float()).abs().max())
    print(f"B={B} T={T} band={band}: equal={eq} maxdiff={d:.3e}  v1 {min(times[1]):.2f} us  v2 {min(times[2]):.2f} us "
          f"({' '.join(f'{t:.2f}' for t in times[1])} | {' '.join(f'{t:.2f}' for t in times[2])})", flush=True)
