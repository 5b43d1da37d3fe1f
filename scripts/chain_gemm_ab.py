"""A/B (GPU box, not the product): the C3 layer chain — FFN2 + norm2 of layer
i, FFN1 + norm1 + in_proj of layer i+1 — as the one fused ffn_chain launch
vs the same math as separate GEMM launches on sbk_gemm (LN kernels between,
Swish / residual in the GEMM epilogues, hidden activations in bf16 through
HBM / MALL).  Prints device time per chain and per GEMM (graph replay),
and the largest difference of the two results.
    python scripts/chain_gemm_ab.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from speechbrain_amd import _enc  # noqa: E402
from scripts.kbench import timeit  # noqa: E402

bf = torch.bfloat16
dev = torch.device("cuda")
torch.manual_seed(0)
M, D, H, NP = 12032, 256, 1024, 768


def ln():
    return (1 + 0.1 * torch.randn(D, device=dev), 0.1 * torch.randn(D, device=dev), 1e-5)


def blk():
    return (ln(), (torch.randn(H, D, device=dev) / D ** 0.5).to(bf), 0.1 * torch.randn(H, device=dev),
            (torch.randn(D, H, device=dev) / H ** 0.5).to(bf), 0.1 * torch.randn(D, device=dev), 0.5)


a, b = blk(), blk()
post, nxt = ln(), ln()
a = a + (post,)
b = b + (None,)
wp = (torch.randn(NP, D, device=dev) / D ** 0.5).to(bf)
x = torch.randn(M, D, device=dev)


def fused():
    return _enc.ffn_chain(x, a, b, "swish", 0.0, nxt, wp)


def gemms(tile=0):
    h = _enc.layernorm(x, *a[0], out1_dtype=bf)[0]
    u = _enc.gemm(h, a[1], bias=a[2], act="swish", out_dtype=bf, tile=tile)
    z = _enc.gemm(u, a[3], bias=a[4], res=x, alpha=a[5], tile=tile)
    z2, h2 = _enc.layernorm(z, *post, out1_dtype=torch.float32, w2=b[0][0], b2=b[0][1], eps2=b[0][2])
    u2 = _enc.gemm(h2, b[1], bias=b[2], act="swish", out_dtype=bf, tile=tile)
    out = _enc.gemm(u2, b[3], bias=b[4], res=z2, alpha=b[5], tile=tile)
    hn = _enc.layernorm(out, *nxt, out1_dtype=bf)[0]
    y = _enc.gemm(hn, wp, out_dtype=bf, tile=tile)
    return out, y


if __name__ == "__main__":
    with torch.no_grad():
        o0, y0 = fused()
        o1, y1 = gemms()
        print(f"max |out diff| {float((o0 - o1).abs().max()):.3e}  max |y diff| "
              f"{float((y0.float() - y1.float()).abs().max()):.3e}", flush=True)
        fl = 4 * 2.0 * M * D * H + 2.0 * M * D * NP
        us = timeit(fused, reps=20)
        print(f"fused ffn_chain: {us:7.1f} us  {fl / us / 1e6:5.0f} TF/s", flush=True)
        for tile in (0, 30):
            try:
                us = timeit(lambda: gemms(tile), reps=20)
            except Exception as e:  # gemm256 does not take N=256 x K=1024 on a forced tile
                print(f"gemm chain tile={tile}: {e}", flush=True)
                continue
            print(f"gemm chain tile={tile}: {us:7.1f} us  {fl / us / 1e6:5.0f} TF/s", flush=True)
        h = _enc.layernorm(x, *a[0], out1_dtype=bf)[0]
        u = _enc.gemm(h, a[1], bias=a[2], act="swish", out_dtype=bf)
        parts = (("layernorm", lambda: _enc.layernorm(x, *a[0], out1_dtype=bf)),
                 ("ln+ln", lambda: _enc.layernorm(x, *post, out1_dtype=torch.float32, w2=b[0][0], b2=b[0][1],
                                                  eps2=b[0][2])),
                 ("up 1024x256 swish", lambda: _enc.gemm(h, a[1], bias=a[2], act="swish", out_dtype=bf)),
                 ("down 256x1024 +res", lambda: _enc.gemm(u, a[3], bias=a[4], res=x, alpha=0.5)),
                 ("in_proj 768x256", lambda: _enc.gemm(h, wp, out_dtype=bf)))
        for name, fn in parts:
            us = timeit(fn, reps=50)
            print(f"  {name:20s} {us:7.1f} us", flush=True)
        for tile in (2, 4, 5, 6, 8, 9, 30):
            try:
                us = timeit(lambda: _enc.gemm(u, a[3], bias=a[4], res=x, alpha=0.5, tile=tile), reps=50)
                us2 = timeit(lambda: _enc.gemm(h, a[1], bias=a[2], act="swish", out_dtype=bf, tile=tile), reps=50)
            except Exception as e:
                print(f"  tile {tile}: {e}", flush=True)
                continue
            print(f"  tile {tile:2d}: down {us:6.1f} us ({2.0 * M * D * H / us / 1e6:4.0f} TF/s)  up {us2:6.1f} us "
                  f"({2.0 * M * D * H / us2 / 1e6:4.0f} TF/s)", flush=True)
