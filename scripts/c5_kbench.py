"""Config-5 kernel microbenchmark: each MXFP8 GEMM shape of one step, the
attention kernel and the latent-extractor layer 0, timed with HIP events
over back-to-back launches on the launch stream (us per launch, TFLOP/s)."""
import sys
import os

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import speechbrain_amd._lib as _L  # noqa: E402
if os.environ.get("SBK_PROBE_LIB"):
    _L.LIB_PATH = os.path.abspath(os.environ["SBK_PROBE_LIB"])  # A/B of a probe build (never the product)
from speechbrain_amd import _w2v, _enc  # noqa: E402


def timeit(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return 1000.0 * e0.elapsed_time(e1) / reps


def main():
    dev = torch.device("cuda:0")
    M = 32 * 748
    d, ff = 1024, 4096
    g = torch.Generator(device=dev).manual_seed(0)
    rnd = lambda *s: torch.randn(*s, device=dev, generator=g)  # noqa: E731
    x = _w2v.mx_quant(rnd(M, d))
    h = _w2v.mx_quant(rnd(M, ff))
    res = rnd(M, d)
    W = {n: _w2v.mx_quant(rnd(N, K) * 0.03) for n, (N, K) in
         {"qkv": (3 * d, d), "out": (d, d), "ffn1": (ff, d), "ffn2": (d, ff)}.items()}
    b = {n: rnd(W[n].q.shape[0]) for n in W}
    cases = [("qkv  bf16 out", lambda: _w2v.mx_gemm(x, W["qkv"], bias=b["qkv"], out=torch.bfloat16), 2 * M * 3 * d * d),
             ("out  +res f32", lambda: _w2v.mx_gemm(x, W["out"], bias=b["out"], res=res), 2 * M * d * d),
             ("ffn1 gelu mx", lambda: _w2v.mx_gemm(x, W["ffn1"], bias=b["ffn1"], act="gelu", out="mx"), 2 * M * ff * d),
             ("ffn1 none f32", lambda: _w2v.mx_gemm(x, W["ffn1"], bias=b["ffn1"]), 2 * M * ff * d),
             ("ffn1 gelu bf16", lambda: _w2v.mx_gemm(x, W["ffn1"], bias=b["ffn1"], act="gelu", out=torch.bfloat16),
              2 * M * ff * d),
             ("ffn2 +res f32", lambda: _w2v.mx_gemm(h, W["ffn2"], bias=b["ffn2"], res=res), 2 * M * d * ff)]
    # conv layer 1 of the extractor: (32, 23998) x 512 from (32, 47998, 512)
    T_in, C = 47998, 512
    xc = _w2v.mx_quant(rnd(32 * T_in, C))
    wc = _w2v.mx_quant(rnd(C, 3 * C) * 0.03)
    T1 = (T_in - 3) // 2 + 1
    cases.append(("conv1 f32", lambda: _w2v.mx_conv_gemm(xc, 32, T_in, C, 3, 2, wc), 2 * 32 * T1 * C * 3 * C))
    for name, fn, fl in cases:
        us = timeit(fn)
        print(f"{name:16s} {us:9.1f} us  {fl / us / 1e6:8.1f} TFLOP/s", flush=True)
    # attention (rel-pos kernel with a zero band, as MultiheadAttention runs it)
    from speechbrain_amd.nnet.attention import MultiheadAttention
    mha = MultiheadAttention(16, d).to(dev)
    qkv = rnd(M, 3 * d).bfloat16()
    us = timeit(lambda: mha.attend(qkv, 32, 748, None, False))
    fl = 32 * 748 * 748 * d * 4
    print(f"{'attention':16s} {us:9.1f} us  {fl / us / 1e6:8.1f} TFLOP/s", flush=True)
    wav = 0.1 * rnd(32, 240000)
    st = _w2v.wav_stats(wav, 1e-5)
    w0, g0, b0 = rnd(512, 11), rnd(512), rnd(512)
    us = timeit(lambda: _w2v.conv0(wav, st, w0, g0, b0, 1e-5, 5, "mx"), reps=5)
    print(f"{'conv0 mx':16s} {us:9.1f} us  {32 * 47998 * 512 * (1 + 1 / 32) / us / 1e3:8.1f} GB/s out", flush=True)


if __name__ == "__main__":
    main()
