"""256x256-tile GEMM (sbk_gemm tile 30, csrc/gemm256.hip): correctness
against torch fp32 matmul of the same bf16 operands, then device time per
call vs the existing tiles on the config-3 / config-5 / square shapes
(GPU box, not the product).  Uniform [-1, 1) operands (rule 25)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from speechbrain_amd import _enc  # noqa: E402
from scripts.kbench import timeit  # noqa: E402

dev = torch.device("cuda")
bf = torch.bfloat16
torch.manual_seed(0)


def rnd(*s):
    return (torch.rand(*s, device=dev) * 2 - 1)


# correctness: tails in M, every epilogue
for (M, N, K) in ((256, 256, 64), (300, 512, 128), (1000, 768, 256), (12032, 1024, 256), (777, 256, 1024)):
    a, w = rnd(M, K).to(bf), rnd(N, K).to(bf)
    b, r = rnd(N), rnd(M, N)
    mask = (torch.rand(M, device=dev) < 0.1).to(torch.uint8)
    ref = a.float() @ w.float().t()
    for act in (None, "swish", "gelu"):
        for odt in (torch.float32, bf):
            o = _enc.gemm(a, w, bias=b, act=act, res=r, alpha=0.5, rowmask=mask, out_dtype=odt, tile=30)
            x = ref + b
            if act == "swish":
                x = x * torch.sigmoid(x)
            elif act == "gelu":
                x = torch.nn.functional.gelu(x)
            x = torch.where(mask.bool()[:, None], torch.zeros_like(x), 0.5 * x) + r
            err = float((o.float() - x).abs().max())
            tol = 2e-3 * float(x.abs().max()) if odt == torch.float32 else 1e-2 * float(x.abs().max())
            print(f"check M={M} N={N} K={K} act={act} out={odt}: max err {err:.3e} {'ok' if err <= tol else 'BAD'}",
                  flush=True)
    o = _enc.gemm(a, w, out_dtype=torch.float32, tile=30)
    print(f"plain M={M} N={N} K={K}: max err {float((o - ref).abs().max()):.3e}", flush=True)

shapes = [(23936, 4096, 1024, bf, "c5 ffn1"), (23936, 1024, 4096, torch.float32, "c5 ffn2"),
          (23936, 3072, 1024, bf, "c5 in_proj"), (23936, 1024, 1024, torch.float32, "c5 out_proj"),
          (12032, 1024, 256, bf, "c3 ffn1"), (12032, 256, 1024, torch.float32, "c3 ffn2"),
          (12032, 768, 256, bf, "c3 in_proj"), (4096, 4096, 4096, bf, "4k^3"), (8192, 8192, 8192, bf, "8k^3")]
for (M, N, K, odt, tag) in shapes:
    a, w = rnd(M, K).to(bf), rnd(N, K).to(bf)
    fl = 2.0 * M * N * K
    res = []
    for t in (30, 0, 7, 2):
        try:
            us = timeit(lambda: _enc.gemm(a, w, out_dtype=odt, tile=t), reps=20 if K < 8192 else 5)
            res.append(f"t{t} {us:8.2f}us {fl / us / 1e6:6.0f}TF/s")
        except Exception as e:  # noqa: BLE001
            res.append(f"t{t} err {e}")
    print(f"{tag:12s} M={M} N={N} K={K}: " + " | ".join(res), flush=True)
