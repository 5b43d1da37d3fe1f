"""MXFP8 GEMM: sbk_mx_gemm (128x128 / 256x128 kernels of mxgemm.hip) vs
sbk_mx_gemm256 (the 256x256 multi-phase kernel of gemm256.hip) on the
config-5 shapes: outputs compared (fp32 bit-equality expected: same MFMA,
same K order) and device time per call (GPU box, not the product)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from speechbrain_amd import _w2v  # noqa: E402
from speechbrain_amd._lib import lib, ptr, stream_of  # noqa: E402
from scripts.kbench import timeit  # noqa: E402

dev = torch.device("cuda")
torch.manual_seed(0)


def call(fn, a, w, M, N, K, mode, bias=None, act=0, res=None):
    out, sc = _w2v._empty_out(M, N, mode, dev)
    rc = fn(ptr(a.q), ptr(a.s), a.q.stride(0), a.s.stride(0), M, 0, 0, ptr(w.q), ptr(w.s), w.q.stride(0),
            w.s.stride(0), M, N, K, ptr(bias), act, 1.0, ptr(res), res.stride(0) if res is not None else 0,
            ptr(out), out.stride(0), mode, ptr(sc) if mode == 2 else None, sc.stride(0) if mode == 2 else 0,
            stream_of(a.q))
    assert rc == 0, rc
    return out, sc


L = lib()

if __name__ == '__main__':
    for (M, N, K, tag) in ((23936, 4096, 1024, "c5 ffn1"), (23936, 1024, 4096, "c5 ffn2"),
                           (23936, 3072, 1024, "c5 in_proj"), (23936, 1024, 1024, "c5 out_proj"),
                           (1000, 512, 256, "tail"), (8192, 8192, 8192, "8k^3")):
        a = _w2v.mx_quant((torch.rand(M, K, device=dev) * 2 - 1))
        w = _w2v.mx_quant((torch.rand(N, K, device=dev) * 2 - 1))
        bias = torch.randn(N, device=dev)
        res = torch.randn(M, N, device=dev)
        for mode, act, r in ((0, 0, None), (0, 4, res), (1, 4, None), (2, 4, None)):
            o0, s0 = call(L.sbk_mx_gemm, a, w, M, N, K, mode, bias, act, r)
            o1, s1 = call(L.sbk_mx_gemm256, a, w, M, N, K, mode, bias, act, r)
            same = torch.equal(o0, o1) and (mode != 2 or torch.equal(s0, s1))
            diff = float((o0.float() - o1.float()).abs().max()) if mode != 2 else int((o0 != o1).sum())
            print(f"{tag} mode={mode} act={act} res={r is not None}: equal={same} maxdiff={diff}", flush=True)
        fl = 2.0 * M * N * K
        res_s = []
        for name, fn in (("mx", L.sbk_mx_gemm), ("mx256", L.sbk_mx_gemm256)):
            for mode in (1, 2):
                us = timeit(lambda: call(fn, a, w, M, N, K, mode, bias, 4), reps=20 if K < 8192 else 5)
                res_s.append(f"{name}/o{mode} {us:8.2f}us {fl / us / 1e6:6.0f}TF/s")
        print(f"{tag:11s} M={M} N={N} K={K}: " + " | ".join(res_s), flush=True)
