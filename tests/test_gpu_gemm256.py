"""The 256 x 256-tile GEMMs (csrc/gemm256.hip) on the GPU: bf16 (sbk_gemm
tile 30, and the automatic dispatch on a config-5 shape) against an fp32
matmul of the same bf16 operands, every epilogue (bias, Swish / GELU,
row mask, alpha, residual; fp32 / bf16 out), M tails; MXFP8
(sbk_mx_gemm256) against the dequantised operands' product, fp32 / bf16 /
MXFP8 outputs, and equal to sbk_mx_gemm's small-tile kernel where both run."""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu


def _rnd(dev, *s):
    return torch.rand(*s, device=dev) * 2 - 1


def _epi(x, b, act, mask, alpha, r):
    x = x + b
    if act == "swish":
        x = x * torch.sigmoid(x)
    elif act == "gelu":
        x = torch.nn.functional.gelu(x)
    x = torch.where(mask.bool()[:, None], torch.zeros_like(x), alpha * x)
    return x + r


@pytest.mark.parametrize("M,N,K", [(256, 256, 64), (300, 512, 128), (1000, 768, 256), (777, 256, 1024)])
def test_gemm256_bf16_epilogues(dev, M, N, K):
    from speechbrain_amd import _enc
    torch.manual_seed(M)
    a, w = _rnd(dev, M, K).to(torch.bfloat16), _rnd(dev, N, K).to(torch.bfloat16)
    b, r = _rnd(dev, N), _rnd(dev, M, N)
    mask = (torch.rand(M, device=dev) < 0.1).to(torch.uint8)
    ref = (a.double().cpu() @ w.double().cpu().t()).float().to(dev)  # exact-enough reference
    for act in (None, "swish", "gelu"):
        x = _epi(ref, b, act, mask, 0.5, r)
        for odt in (torch.float32, torch.bfloat16):
            o = _enc.gemm(a, w, bias=b, act=act, res=r, alpha=0.5, rowmask=mask, out_dtype=odt, tile=30)
            tol = (1e-5 * math.sqrt(K) + (3e-6 if act == "gelu" else 0.0)) if odt == torch.float32 else 8e-3
            err = float(((o.float() - x).abs() / x.abs().clamp(min=1.0)).max())
            assert err <= tol, (act, odt, err)


def test_gemm256_auto_dispatch_config5_shape(dev):
    """(M, N, K) = (4096, 4096, 1024) takes the 256 tile by default: the
    result equals tile 30 bit for bit and the fp32 product within 1e-5 rel."""
    from speechbrain_amd import _enc
    torch.manual_seed(1)
    a, w = _rnd(dev, 4096, 1024).to(torch.bfloat16), _rnd(dev, 4096, 1024).to(torch.bfloat16)
    o0 = _enc.gemm(a, w, out_dtype=torch.float32)
    o30 = _enc.gemm(a, w, out_dtype=torch.float32, tile=30)
    assert torch.equal(o0, o30)
    ref = (a.double().cpu() @ w.double().cpu().t()).float().to(dev)
    assert float(((o0 - ref).abs() / ref.abs().clamp(min=1.0)).max()) < 1e-5 * 32


def _mx_call(fn, a, w, M, N, K, mode, bias=None, act=0, res=None):
    from speechbrain_amd import _w2v
    from speechbrain_amd._lib import ptr, stream_of
    out, sc = _w2v._empty_out(M, N, mode, a.q.device)
    rc = fn(ptr(a.q), ptr(a.s), a.q.stride(0), a.s.stride(0), M, 0, 0, ptr(w.q), ptr(w.s), w.q.stride(0),
            w.s.stride(0), M, N, K, ptr(bias), act, 1.0, ptr(res), res.stride(0) if res is not None else 0,
            ptr(out), out.stride(0), mode, ptr(sc) if mode == 2 else None, sc.stride(0) if mode == 2 else 0,
            stream_of(a.q))
    assert rc == 0, rc
    return out, sc


@pytest.mark.parametrize("M,N,K", [(300, 256, 128), (1000, 512, 256), (2048, 768, 1024)])
def test_mx256_vs_dequantised_and_small_tile(dev, M, N, K):
    from speechbrain_amd import _w2v
    from speechbrain_amd._lib import lib
    L = lib()
    torch.manual_seed(K)
    a = _w2v.mx_quant(_rnd(dev, M, K))
    w = _w2v.mx_quant(_rnd(dev, N, K))
    ref = (_w2v.mx_dequant(a).double().cpu() @ _w2v.mx_dequant(w).double().cpu().t()).float().to(dev)
    bias, res = _rnd(dev, N), _rnd(dev, M, N)
    o, _ = _mx_call(L.sbk_mx_gemm256, a, w, M, N, K, 0, bias, 0, res)
    # the block-scaled MFMA's own accumulation is coarser than an fp32 sum of
    # the exact e4m3 products (measured 1.7e-4 .. 4.7e-4 of max(1, |ref|) at
    # K = 128 .. 1024, identical in the small-tile kernel): bound it, and
    # equality with that kernel below pins this one bit for bit
    err = float(((o - (ref + bias + res)).abs() / (ref + bias + res).abs().clamp(min=1.0)).max())
    assert err < 4e-5 * math.sqrt(K), err
    # fp32 / bf16 / MXFP8 outputs equal the 128-tile kernel's (same MFMA, same K order;
    # at these M sbk_mx_gemm runs its small-tile kernel)
    for mode, act in ((0, 4), (1, 4), (2, 4), (2, 0)):
        o0, s0 = _mx_call(L.sbk_mx_gemm, a, w, M, N, K, mode, bias, act)
        o1, s1 = _mx_call(L.sbk_mx_gemm256, a, w, M, N, K, mode, bias, act)
        if act == 4:  # the 256 tile's GELU is the 1.5e-7 erf approximation: compare values
            d0 = o0.float() if mode < 2 else _w2v.mx_dequant(_w2v.MX(o0, s0))
            d1 = o1.float() if mode < 2 else _w2v.mx_dequant(_w2v.MX(o1, s1))
            tol = 1e-5 if mode == 0 else (8e-3 if mode == 1 else 0.13)
            assert float(((d0 - d1).abs() / d0.abs().clamp(min=1.0)).max()) <= tol, mode
        else:
            assert torch.equal(o0, o1) and torch.equal(s0, s1), mode


@pytest.mark.parametrize("act,with_res,K", [(0, True, 2048), (4, False, 2048), (3, True, 2176)])
def test_mx256_split_k_tail(dev, act, with_res, K):
    """sbk_mx_gemm_ws: the tiles past the last full round of 256-tile
    workgroups run as two K halves + an epilogue pass (gemm256.hip
    split_tail).  At (M, N) = (17820, 1024) — 70 row tiles x 4 = 280
    tiles, a ragged last row tile; K = 2176 splits 17 K-tiles as 8 + 9; no
    activation, GELU, ReLU — the result equals the unsplit launch's up to the
    fp32 order of the halves' sum, and the workspace size is the rule's
    (2 x tail x 256 x 256 floats, fp32 out only)."""
    from speechbrain_amd import _w2v
    from speechbrain_amd._lib import lib, ptr, stream_of
    L = lib()
    M, N = 17820, 1024
    cus = torch.cuda.get_device_properties(dev).multi_processor_count
    nt = ((M + 255) // 256) * (N // 256)
    tail = nt % cus
    if not (nt > cus and 0 < tail and 2 * tail <= cus):
        pytest.skip(f"{cus} CUs: no split tail at this shape")
    nws = int(L.sbk_mx_gemm_ws_floats(M, N, K, 0))
    assert nws == 2 * tail * 65536, (nws, tail)
    assert int(L.sbk_mx_gemm_ws_floats(M, N, K, 1)) == 0 and int(L.sbk_mx_gemm_ws_floats(M, N, 1024, 0)) == 0
    torch.manual_seed(act + 7)
    a = _w2v.mx_quant(_rnd(dev, M, K))
    w = _w2v.mx_quant(_rnd(dev, N, K))
    bias = _rnd(dev, N)
    res = _rnd(dev, M, N) if with_res else None
    o0, _ = _mx_call(L.sbk_mx_gemm, a, w, M, N, K, 0, bias, act, res)
    ws = torch.full((nws,), float("nan"), device=dev)
    o1 = torch.full((M, N), float("nan"), device=dev)
    rc = L.sbk_mx_gemm_ws(ptr(a.q), ptr(a.s), a.q.stride(0), a.s.stride(0), M, 0, 0, ptr(w.q), ptr(w.s),
                          w.q.stride(0), w.s.stride(0), M, N, K, ptr(bias), act, 1.0, ptr(res),
                          res.stride(0) if res is not None else 0, ptr(o1), o1.stride(0), 0, None, 0, ptr(ws), nws,
                          stream_of(a.q))
    assert rc == 0, rc
    torch.cuda.synchronize()
    assert bool(torch.isfinite(o1).all())
    err = float(((o1 - o0).abs() / o0.abs().clamp(min=1.0)).max())
    assert err < 1e-5, err
    # whole tiles are the unsplit kernel's bit for bit: at most the tail's
    # tiles (tail x 65536 values) differ
    assert int((o1 != o0).sum()) <= tail * 65536
    # the op path (_w2v.mx_gemm's custom op) takes the workspace entry
    o2, _ = _w2v._mx_gemm_op(a.q, a.s, M, K, a.q.stride(0), a.s.stride(0), M, 0, 0, w.q, w.s, bias, act, 1.0, res, 0)
    assert torch.equal(o2, o1)


def test_mx256_split_k_tail_graph_replay(dev):
    """The split-K tail inside a captured HIP graph (the C5 bench's mode):
    the workspace comes from the graph's pool at capture, and a replay on new
    inputs equals the eager call on them bit for bit."""
    from speechbrain_amd import _w2v
    from speechbrain_amd._lib import lib
    M, N, K = 17820, 1024, 2048
    if not int(lib().sbk_mx_gemm_ws_floats(M, N, K, 0)):
        pytest.skip("no split tail at this shape on this device")
    torch.manual_seed(11)
    x = _rnd(dev, M, K)
    w = _w2v.mx_quant(_rnd(dev, N, K))
    bias, res = _rnd(dev, N), _rnd(dev, M, N)

    def step():
        return _w2v.mx_gemm(_w2v.mx_quant(x), w, bias=bias, res=res)

    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        step()  # warm-up outside the capture
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        out = step()
    x.copy_(_rnd(dev, M, K))
    g.replay()
    torch.cuda.synchronize()
    assert torch.equal(out, step())
