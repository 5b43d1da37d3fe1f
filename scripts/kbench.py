"""Kernel micro-benchmarks on the GPU box (not part of the product):
per-shape GEMM TFLOP/s for each tile config, attention, dwconv, LN, Fbank.
    python scripts/kbench.py [gemm|attn|misc|all]
"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import speechbrain_amd._lib as _L  # noqa: E402
if os.environ.get("SBK_PROBE_LIB"):
    _L.LIB_PATH = os.path.abspath(os.environ["SBK_PROBE_LIB"])  # probe builds of a kernel (not product)
from speechbrain_amd import _enc  # noqa: E402
from speechbrain_amd._lib import lib, ptr, stream_of  # noqa: E402


def timeit(fn, reps=50, warm=5):
    """Device time per call: `reps` calls captured in one HIP graph and
    replayed, so host dispatch cost is excluded (kernels run back to back)."""
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps):
            fn()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(3):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / (3 * reps) * 1000.0  # us


def gemm_bench():
    dev = torch.device("cuda")
    M = 12032
    shapes = [("ffn_up", 1024, 256, "swish", False, torch.bfloat16), ("ffn_down", 256, 1024, None, True, torch.float32),
              ("qkv", 768, 256, None, False, torch.bfloat16), ("out_proj", 256, 256, None, True, torch.float32),
              ("glu", 512, 256, "glu", False, torch.bfloat16), ("src", 256, 640, None, False, torch.float32)]
    for name, N, K, act, res, od in shapes:
        a = torch.randn(M, K, device=dev).to(torch.bfloat16)
        w = (torch.randn(N, K, device=dev) / K ** 0.5).to(torch.bfloat16)
        b = torch.randn(N, device=dev)
        r = torch.randn(M, N // 2 if act == "glu" else N, device=dev) if res else None
        fl = 2.0 * M * N * K
        line = f"{name:9s} M={M} N={N} K={K}:"
        for tile in (2, 4, 5, 6, 8, 9):
            us = timeit(lambda: _enc.gemm(a, w, bias=b, act=act, res=r, out_dtype=od, tile=tile))
            line += f" t{tile} {us:6.1f}us {fl / us / 1e6:6.0f}TF"
        # library reference point (plain GEMM, no fused epilogue): hipBLASLt via torch
        us = timeit(lambda: torch.mm(a, w.t()))
        line += f" | torch.mm {us:6.1f}us {fl / us / 1e6:6.0f}TF"
        print(line, flush=True)


def gemm_one(name="qkv", tile=2):
    """One GEMM shape/tile, 50 launches (for counter passes)."""
    dev = torch.device("cuda")
    M = 12032
    N, K = {"qkv": (768, 256), "out_proj": (256, 256), "ffn_down": (256, 1024)}[name]
    a = torch.randn(M, K, device=dev).to(torch.bfloat16)
    w = (torch.randn(N, K, device=dev) / K ** 0.5).to(torch.bfloat16)
    us = timeit(lambda: _enc.gemm(a, w, out_dtype=torch.bfloat16, tile=tile))
    print(f"{name} tile {tile}: {us:.1f}us", flush=True)


def gemmln_bench():
    dev = torch.device("cuda")
    M, N, K = 12032, 256, 256
    a = torch.randn(M, K, device=dev).to(torch.bfloat16)
    w = (torch.randn(N, K, device=dev) / 16).to(torch.bfloat16)
    bias = torch.randn(N, device=dev)
    res = torch.randn(M, N, device=dev)
    ln = (torch.ones(N, device=dev), torch.zeros(N, device=dev), 1e-5)
    for tile in (0, 1, 2):
        us = timeit(lambda: _enc.gemm_ln(a, w, ln, bias=bias, res=res, tile=tile))
        print(f"gemm_ln tile {tile}: {us:.1f}us", flush=True)
    us1 = timeit(lambda: _enc.gemm(a, w, bias=bias, res=res))
    out = _enc.gemm(a, w, bias=bias, res=res)
    us2 = timeit(lambda: _enc.layernorm(out, *ln, out1_dtype=torch.bfloat16))
    print(f"separate: gemm {us1:.1f}us + layernorm {us2:.1f}us", flush=True)


def convmod_bench():
    from speechbrain_amd.lobes.models.transformer.Conformer import ConvolutionModule
    dev = torch.device("cuda")
    B, T = 32, 376
    cm = ConvolutionModule(256, 31).to(dev).eval()
    x = torch.randn(B * T, 256, device=dev)
    with torch.no_grad():
        us = timeit(lambda: cm.run_fused(x, B, T, None))
        us2 = timeit(lambda: cm.run(x, B, T, torch.bfloat16, None, residual=x))
    print(f"conv_module fused {us:.1f}us | chain {us2:.1f}us", flush=True)


def attn_bench():
    dev = torch.device("cuda")
    B, T, H, dh = 32, 376, 4, 64
    d = H * dh
    qkv = torch.randn(B * T, 3 * d, device=dev).to(torch.bfloat16)
    pk = torch.randn(2 * T - 1, d, device=dev).to(torch.bfloat16)
    u = torch.randn(H * dh, device=dev)
    v = torch.randn(H * dh, device=dev)
    us = timeit(lambda: _enc.relpos_attention(qkv, pk, u, v, None, B, T, H, dh, 1 / 16.0))
    fl = B * H * (2 * T * T * dh * 2 + 2 * T * (T + 64) * dh)
    print(f"relpos_attn bf16 B={B} T={T}: {us:.1f}us  {fl / us / 1e6:.1f} TF (algorithmic)", flush=True)


def misc_bench():
    dev = torch.device("cuda")
    M, d = 12032, 256
    x = torch.randn(M, d, device=dev)
    w = torch.randn(d, device=dev)
    us = timeit(lambda: _enc.layernorm(x, w, w, 1e-5, torch.bfloat16))
    print(f"layernorm {M}x{d}: {us:.1f}us {(M * d * 6) / us / 1e3:.0f} GB/s", flush=True)
    g = torch.randn(M, d, device=dev).to(torch.bfloat16)
    cw = torch.randn(d, 1, 31, device=dev)
    us = timeit(lambda: _enc.dwconv_ln_swish(g, 32, 376, cw, w, False, w, w, 1e-5, torch.bfloat16))
    print(f"dwconv_ln_swish: {us:.1f}us {(M * d * 4) / us / 1e3:.0f} GB/s", flush=True)
    from speechbrain_amd.lobes.features import Fbank
    fb = Fbank(n_mels=80).to(dev)
    wav = torch.randn(32, 240000, device=dev) * 0.1
    us = timeit(lambda: fb(wav), reps=20)
    print(f"fbank 32x15s: {us:.1f}us {(32 * 240000 * 4 + 32 * 1501 * 80 * 4) / us / 1e3:.0f} GB/s", flush=True)


def ffn_bench():
    from speechbrain_amd.nnet.attention import PositionalwiseFeedForward
    from speechbrain_amd.nnet.activations import Swish
    dev = torch.device("cuda")
    for D, H in ((256, 1024), (256, 2048)):
        M = 12032
        ffn = PositionalwiseFeedForward(H, input_size=D, activation=Swish).to(dev).eval()
        x = torch.randn(M, D, device=dev)
        ln = (torch.ones(D, device=dev), torch.zeros(D, device=dev), 1e-5)
        with torch.no_grad():
            us = timeit(lambda: ffn.run_fused(x, ln, 0.5, next_ln=ln))
            u = _enc.layernorm(x, *ln, out1_dtype=torch.bfloat16)[0]
            us2 = timeit(lambda: ffn.run(u, torch.bfloat16, residual=x, alpha=0.5))
        fl = 4.0 * M * D * H
        print(f"ffn D={D} H={H} M={M}: fused {us:.1f}us {fl / us / 1e6:.0f} TF/s | 2 gemms {us2:.1f}us", flush=True)
        wp = (torch.randn(768, D, device=dev) / 16).to(torch.bfloat16)
        with torch.no_grad():
            us3 = timeit(lambda: ffn.run_fused_proj(x, ln, 0.5, ln, wp))
            u = ffn.run_fused(x, ln, 0.5, next_ln=ln)[1]
            us4 = timeit(lambda: _enc.gemm(u, wp, out_dtype=torch.bfloat16))
        print(f"ffn+qkv D={D} H={H}: fused {us3:.1f}us | ffn {us:.1f}us + qkv gemm {us4:.1f}us", flush=True)


if __name__ == "__main__":
    what = sys.argv[1] if len(sys.argv) > 1 else "all"
    if what in ("gemm", "all"):
        gemm_bench()
    if what in ("attn", "all"):
        attn_bench()
    if what in ("misc", "all"):
        misc_bench()
    if what == "gemm1":
        gemm_one(sys.argv[2] if len(sys.argv) > 2 else "qkv", int(sys.argv[3]) if len(sys.argv) > 3 else 2)
    if what in ("convmod", "all"):
        convmod_bench()
    if what in ("ffn", "all"):
        ffn_bench()
    if what in ("gemmln", "all"):
        gemmln_bench()
