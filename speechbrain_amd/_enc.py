"""Thin Python wrappers over the encoder kernels of libsbk.so (gemm.hip,
conformer.hip, attention.hip).  Direct ctypes calls — no Python compute, no
fallback; used by the nn.Module drop-ins and capturable into HIP graphs
(no host sync, no allocation outside torch's caching allocator)."""
import torch

from ._lib import check, lib, ptr, require_device, stream_of

ACT = {None: 0, "none": 0, "swish": 1, "glu": 2, "leaky_relu": 3, "relu": 3, "gelu": 4}
_bf16 = torch.bfloat16
_f32 = torch.float32


def _is_bf16(t):
    return t.dtype == _bf16


def gemm(a, w, bias=None, act=None, slope=0.0, res=None, alpha=1.0, rowmask=None, out=None,
         out_dtype=_f32, tile=0):
    """out = res + alpha * act(a @ w.T + bias), rows with rowmask -> 0 before the
    residual.  a: (M, K), w: (N, K), both bf16 or both fp32."""
    require_device(a, w)
    if a.dtype != w.dtype:
        raise TypeError(f"gemm operand dtypes differ: {a.dtype} vs {w.dtype}")
    if a.stride(-1) != 1 or w.stride(-1) != 1:
        raise ValueError("gemm operands must be K-contiguous")
    M, K = a.shape
    N = w.shape[0]
    code = ACT[act]
    n_out = N // 2 if code == 2 else N
    if out is None:
        out = torch.empty(M, n_out, device=a.device, dtype=out_dtype)
    if res is not None and (res.dtype != _f32 or res.stride(-1) != 1):
        raise ValueError("residual must be fp32, row-contiguous")
    rc = lib().sbk_gemm(int(_is_bf16(a)), ptr(a), a.stride(0), ptr(w), w.stride(0), M, N, K, ptr(bias), code,
                        float(slope), ptr(res), res.stride(0) if res is not None else 0, float(alpha),
                        ptr(rowmask), ptr(out), out.stride(0), int(out.dtype == _bf16), int(tile), stream_of(a))
    check(rc, "sbk_gemm")
    return out


def length_mask(rel_len, T):
    """(B, T) uint8: t > floor(rel_len[b] * T) — one launch."""
    require_device(rel_len)
    rl = rel_len if (rel_len.dtype == _f32 and rel_len.is_contiguous()) else rel_len.float().contiguous()
    B = rl.shape[0]
    out = torch.empty(B, T, device=rl.device, dtype=torch.uint8)
    check(lib().sbk_length_mask(ptr(rl), B, int(T), ptr(out), stream_of(rl)), "sbk_length_mask")
    return out


def gemm_ln(a, w, ln, bias=None, res=None, alpha=1.0, rowmask=None, out=None, u_dtype=_bf16, tile=0):
    """out = res + alpha * (a @ w.T + bias) (fp32) and u = LN(out; *ln) in one
    launch (N == 256).  Returns (out, u)."""
    require_device(a, w)
    if a.dtype != w.dtype:
        raise TypeError(f"gemm operand dtypes differ: {a.dtype} vs {w.dtype}")
    M, K = a.shape
    N = w.shape[0]
    if out is None:
        out = torch.empty(M, N, device=a.device, dtype=_f32)
    u = torch.empty(M, N, device=a.device, dtype=u_dtype)
    if res is not None and (res.dtype != _f32 or res.stride(-1) != 1):
        raise ValueError("residual must be fp32, row-contiguous")
    g, b, eps = ln
    rc = lib().sbk_gemm_ln(int(_is_bf16(a)), ptr(a), a.stride(0), ptr(w), w.stride(0), M, N, K, ptr(bias), ptr(res),
                           res.stride(0) if res is not None else 0, float(alpha), ptr(rowmask), ptr(out),
                           out.stride(0), ptr(g), ptr(b), float(eps), ptr(u), u.stride(0), int(u_dtype == _bf16),
                           int(tile), stream_of(a))
    check(rc, "sbk_gemm_ln")
    return out, u


# The fused projection + LayerNorm (sbk_gemm_ln) measures the same as the two
# launches it replaces at M = 12032 (15.1 vs 8.5 + 6.3 us): off by default.
USE_GEMM_LN = False


def gemm_ln_supported(N):
    return int(N) == 256


def layernorm(x, w1, b1, eps1, out1_dtype=_f32, w2=None, b2=None, eps2=1e-5, out2_dtype=_bf16, out1=None):
    """y1 = LN(x; w1, b1) (returned unless out1_dtype is None); optionally
    y2 = LN(y1; w2, b2) in one pass.  x: (M, D) fp32."""
    require_device(x)
    M, D = x.shape
    if out1 is None and out1_dtype is not None:
        out1 = torch.empty(M, D, device=x.device, dtype=out1_dtype)
    out2 = torch.empty(M, D, device=x.device, dtype=out2_dtype) if w2 is not None else None
    rc = lib().sbk_layernorm(ptr(x), M, D, ptr(w1), ptr(b1), float(eps1), ptr(out1),
                             int(out1 is not None and out1.dtype == _bf16), ptr(w2), ptr(b2), float(eps2), ptr(out2),
                             int(out2 is not None and out2.dtype == _bf16), stream_of(x))
    check(rc, "sbk_layernorm")
    return out1, out2


def ffn_supported(D, H):
    return bool(lib().sbk_ffn_supported(int(D), int(H)))


def ffn(x, ln0, w1, b1, act, slope, w2, b2, alpha, post_ln=None, next_ln=None, next_dtype=_bf16, out=None):
    """Fused macaron FFN block (bf16 MFMA): z = x + alpha * FFN(LN0(x));
    out = post_ln(z) if given; u = next_ln(out) (returned) if given.
    x: (M, D) fp32; ln*: (weight, bias, eps); w1 (H, D), w2 (D, H) bf16.
    `out` may alias x."""
    require_device(x, w1, w2)
    M, D = x.shape
    H = w1.shape[0]
    if out is None:
        out = torch.empty_like(x)
    u = torch.empty(M, D, device=x.device, dtype=next_dtype) if next_ln is not None else None
    gp, bp, ep = post_ln if post_ln is not None else (None, None, 0.0)
    gn, bn, en = next_ln if next_ln is not None else (None, None, 0.0)
    rc = lib().sbk_ffn(ptr(x), M, D, H, ptr(ln0[0]), ptr(ln0[1]), float(ln0[2]), ptr(w1), ptr(b1), ACT[act],
                       float(slope), ptr(w2), ptr(b2), float(alpha), ptr(gp), ptr(bp), float(ep), ptr(out),
                       ptr(gn), ptr(bn), float(en), ptr(u), int(next_dtype == _bf16), stream_of(x))
    check(rc, "sbk_ffn")
    return out, u


def dwconv_ln_swish(x, B, T, w, bias, causal, ln_w, ln_b, eps, out_dtype):
    """Depthwise Conv1d over time + LayerNorm(C) + Swish.  x: (B*T, C)."""
    C = x.shape[-1]
    K = w.shape[-1]
    out = torch.empty(B * T, C, device=x.device, dtype=out_dtype)
    rc = lib().sbk_dwconv_ln_swish(int(_is_bf16(x)), ptr(x), B, T, C, ptr(w), ptr(bias), K, int(causal), ptr(ln_w),
                                   ptr(ln_b), float(eps), ptr(out), int(out_dtype == _bf16), stream_of(x))
    check(rc, "sbk_dwconv_ln_swish")
    return out


def conv_module_supported(D, K):
    return bool(lib().sbk_conv_module_supported(int(D), int(K)))


def conv_module(x, B, T, ln0, w1p, b1p, wc, bc, causal, ln1, w2, b2, kpm=None):
    """Fused Conformer convolution module (bf16 MFMA, one launch):
    x + rowmask0(after_conv(dwconv(GLU(pointwise(LN0(x)))))).  x: (B*T, 256) fp32."""
    require_device(x, w1p, w2)
    K = wc.shape[0]  # wc: (K, d) tap-major
    out = torch.empty_like(x)
    rc = lib().sbk_conv_module(ptr(x), ptr(out), B, T, x.shape[1], ptr(ln0[0]), ptr(ln0[1]), float(ln0[2]), ptr(w1p),
                               ptr(b1p), ptr(wc), ptr(bc), K, int(causal), ptr(ln1[0]), ptr(ln1[1]), float(ln1[2]),
                               ptr(w2), ptr(b2), ptr(kpm), stream_of(x))
    check(rc, "sbk_conv_module")
    return out


def conv_block_c1(x, w, bias, ln_w, ln_b, eps, slope, out_dtype):
    """ConvBlock with one input channel: x (B, T, F) fp32 → (B, T', F', C)."""
    require_device(x)
    B, Tin, Fin = x.shape
    Cout = w.shape[0]
    Tout, Fout = (Tin - 1) // 2 + 1, (Fin - 1) // 2 + 1
    out = torch.empty(B, Tout, Fout, Cout, device=x.device, dtype=out_dtype)
    rc = lib().sbk_conv_block_c1(ptr(x), B, Tin, Fin, Cout, ptr(w), ptr(bias), ptr(ln_w), ptr(ln_b), float(eps),
                                 float(slope), ptr(out), int(out_dtype == _bf16), None, None, stream_of(x))
    check(rc, "sbk_conv_block_c1")
    return out


def conv_block_mfma(x, wperm, bias, ln_w, ln_b, eps, slope, out_dtype):
    """ConvBlock implicit GEMM: x (B, T, F, Cin) → (B, T', F', Cout);
    wperm: (Cout, 3, 3, Cin) [time, freq] in x.dtype."""
    require_device(x, wperm)
    B, Tin, Fin, Cin = x.shape
    Cout = wperm.shape[0]
    Tout, Fout = (Tin - 1) // 2 + 1, (Fin - 1) // 2 + 1
    out = torch.empty(B, Tout, Fout, Cout, device=x.device, dtype=out_dtype)
    rc = lib().sbk_conv_block_mfma(int(_is_bf16(x)), ptr(x), B, Tin, Fin, Cin, Cout, ptr(wperm), ptr(bias),
                                   ptr(ln_w), ptr(ln_b), float(eps), float(slope), ptr(out),
                                   int(out_dtype == _bf16), None, None, stream_of(x))
    check(rc, "sbk_conv_block_mfma")
    return out


def conv_frontend2(x, blk1, blk2, wperm2, out_dtype):
    """Both ConvBlocks in one kernel: x (B, T, F) fp32 → (B, T2, F2, C2).
    blk*: (conv weight, bias, ln weight, ln bias, ln eps, leaky slope);
    wperm2: block-2 weights (C2, 3, 3, C1) in the compute dtype."""
    require_device(x, wperm2)
    B, Tin, Fin = x.shape
    w1, b1, g1, be1, e1, s1 = blk1
    _, b2, g2, be2, e2, s2 = blk2
    C1, C2 = w1.shape[0], wperm2.shape[0]
    T1, F1 = (Tin - 1) // 2 + 1, (Fin - 1) // 2 + 1
    T2, F2 = (T1 - 1) // 2 + 1, (F1 - 1) // 2 + 1
    out = torch.empty(B, T2, F2, C2, device=x.device, dtype=out_dtype)
    rc = lib().sbk_conv_frontend2(int(_is_bf16(wperm2)), ptr(x), B, Tin, Fin, ptr(w1), ptr(b1), ptr(g1), ptr(be1),
                                  float(e1), float(s1), C1, ptr(wperm2), ptr(b2), ptr(g2), ptr(be2), float(e2),
                                  float(s2), C2, ptr(out), int(out_dtype == _bf16), None, None, stream_of(x))
    check(rc, "sbk_conv_frontend2")
    return out


def relpos_attention(qkv, pk, pbu, pbv, kpm, B, T, H, dh, scale, need_probs=False):
    """Fused RelPosMHAXL core.  qkv: (B*T, 3d) head-interleaved, pk: (2T-1, d),
    both bf16 or fp32; returns (out (B*T, d) in qkv.dtype, probs or None)."""
    d = H * dh
    if pk.stride(-1) != 1 or pk.shape[-1] != d:
        raise ValueError("pk must be (2T-1, d) with unit column stride")
    out = torch.empty(B * T, d, device=qkv.device, dtype=qkv.dtype)
    probs = torch.empty(B, H, T, T, device=qkv.device, dtype=_f32) if need_probs else None
    rc = lib().sbk_relpos_attention_ld(int(_is_bf16(qkv)), ptr(qkv), ptr(pk), pk.stride(0), ptr(pbu), ptr(pbv),
                                       ptr(kpm), B, T, H, dh, float(scale), ptr(out), ptr(probs), stream_of(qkv))
    check(rc, "sbk_relpos_attention")
    return out, probs


def glu_group():
    """Channels per GLU pairing group (weights row-permuted in [a | gate] groups)."""
    return int(lib().sbk_gemm_glu_group(1))


def cast_bf16(x):
    out = torch.empty(x.shape, device=x.device, dtype=_bf16)
    check(lib().sbk_cast_bf16(ptr(x), ptr(out), x.numel(), stream_of(x)), "sbk_cast_bf16")
    return out


def to_compute(x, dtype):
    """Row-contiguous copy of x in the compute dtype (bf16 via the cast kernel)."""
    if dtype == _bf16:
        return x.contiguous() if x.dtype == _bf16 else cast_bf16(x.float().contiguous())
    if x.dtype != _f32:
        raise TypeError(f"fp32 compute path got {x.dtype}")
    return x.contiguous()


def compute_dtype():
    """bf16 MFMA under torch.autocast(device_type='cuda', dtype=bf16),
    exact-f32 MFMA otherwise.  fp16 autocast (the reference's
    `--auto_mix_prec`, core.py:905-919) has no kernels here and raises rather
    than silently computing in bf16."""
    if torch.is_autocast_enabled("cuda"):
        dt = torch.get_autocast_dtype("cuda")
        if dt != _bf16:
            raise NotImplementedError(
                f"speechbrain_amd kernels compute in bf16 or fp32; torch.autocast(dtype={dt}) is not supported. "
                "Use torch.autocast('cuda', dtype=torch.bfloat16) (Brain: auto_mix_prec='bf16') or no autocast.")
        return _bf16
    return _f32


class WeightCache:
    """Per-module cache of kernel-ready weight copies (bf16 casts, GLU row
    permutations), refreshed when a parameter's storage or version changes."""

    def __init__(self):
        self._d = {}

    def get(self, key, params, make):
        sig = tuple((p.data_ptr(), p._version, p.device) for p in params)
        hit = self._d.get(key)
        if hit is not None and hit[0] == sig:
            return hit[1]
        v = make()
        self._d[key] = (sig, v)
        return v
