"""Thin Python wrappers over the encoder kernels of libsbk.so (gemm.hip,
conformer.hip, attention.hip).  Direct ctypes calls — no Python compute, no
fallback; used by the nn.Module drop-ins and capturable into HIP graphs
(no host sync, no allocation outside torch's caching allocator)."""
import contextlib
import ctypes
import threading
import weakref
from typing import Optional

import torch

from ._lib import OPS, SbkError, check, custom_op, lib, ptr, require_device, stream_of

ACT = {None: 0, "none": 0, "swish": 1, "glu": 2, "leaky_relu": 3, "relu": 3, "gelu": 4}
_bf16 = torch.bfloat16
_f32 = torch.float32


def _is_bf16(t):
    return t.dtype == _bf16


# ---------------------------------------------------------------------------
# torch.library custom ops (sbk::*): every encoder kernel is a dispatcher op,
# so torch.jit.trace / torch.compile record the launches as graph nodes
# (instead of baking ctypes results in as constants) and HIP-graph capture
# sees ordinary stream work.  The Python wrappers below keep the call
# signatures the modules use.  Optional outputs are returned as 0-element
# tensors by the ops and mapped back to None by the wrappers.
# ---------------------------------------------------------------------------
@custom_op("sbk::gemm", mutates_args=())
def _gemm_op(a: torch.Tensor, w: torch.Tensor, bias: Optional[torch.Tensor], act: int, slope: float,
             res: Optional[torch.Tensor], alpha: float, rowmask: Optional[torch.Tensor], out_bf16: bool,
             tile: int) -> torch.Tensor:
    M, K = a.shape
    N = w.shape[0]
    n_out = N // 2 if act == 2 else N
    out = torch.empty(M, n_out, device=a.device, dtype=_bf16 if out_bf16 else _f32)
    rc = lib().sbk_gemm(int(_is_bf16(a)), ptr(a), a.stride(0), ptr(w), w.stride(0), M, N, K, ptr(bias), act,
                        float(slope), ptr(res), res.stride(0) if res is not None else 0, float(alpha),
                        ptr(rowmask), ptr(out), out.stride(0), int(out_bf16), int(tile), stream_of(a))
    check(rc, "sbk_gemm")
    return out


@_gemm_op.register_fake
def _(a, w, bias, act, slope, res, alpha, rowmask, out_bf16, tile):
    n = w.shape[0] // 2 if act == 2 else w.shape[0]
    return a.new_empty(a.shape[0], n, dtype=_bf16 if out_bf16 else _f32)


def gemm(a, w, bias=None, act=None, slope=0.0, res=None, alpha=1.0, rowmask=None, out=None,
         out_dtype=_f32, tile=0):
    """out = res + alpha * act(a @ w.T + bias), rows with rowmask -> 0 before the
    residual.  a: (M, K), w: (N, K), both bf16 or both fp32."""
    require_device(a, w)
    if out is not None:
        raise ValueError("gemm allocates its output (out= is not supported)")
    if a.dtype != w.dtype:
        raise TypeError(f"gemm operand dtypes differ: {a.dtype} vs {w.dtype}")
    if (a.stride(-1) != 1 and a.shape[-1] > 1) or (w.stride(-1) != 1 and w.shape[-1] > 1):
        raise ValueError("gemm operands must be K-contiguous")
    if res is not None and (res.dtype != _f32 or res.stride(-1) != 1):
        raise ValueError("residual must be fp32, row-contiguous")
    vec = 8 if a.dtype == _bf16 else 4
    if (a.shape[1] % vec or a.stride(0) % vec or w.stride(0) % vec
            or (a.data_ptr() | w.data_ptr()) % 16):
        # the MFMA tiles read K in 16-B vectors: zero-pad K (odd widths such
        # as a 10-unit prediction-network GRU; the hot-path shapes never pad)
        Kp = -(-a.shape[1] // vec) * vec
        a = torch.nn.functional.pad(a, (0, Kp - a.shape[1]))
        w = torch.nn.functional.pad(w, (0, Kp - w.shape[1]))
    return OPS.gemm(a, w, bias, ACT[act], float(slope), res, float(alpha), rowmask,
                              out_dtype == _bf16, int(tile))


@custom_op("sbk::gemm_tn", mutates_args=())
def _gemm_tn_op(a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    K, M = a.shape[-2], a.shape[-1]
    N = b.shape[-1]
    batch = a.shape[0] if a.dim() == 3 else 1
    out = torch.zeros(*([batch] if a.dim() == 3 else []), M, N, device=a.device, dtype=_f32)
    sa = a.stride(0) if a.dim() == 3 else 0
    sb = b.stride(0) if b.dim() == 3 else 0
    _tn_call(a, a.stride(-2), sa, b, b.stride(-2), sb, M, N, K, batch, out, N, M * N if a.dim() == 3 else 0)
    return out


def _tn_call(a, lda, sa, b, ldb, sb, M, N, K, batch, out, ldc, sc):
    """sbk_gemm_tn (bf16) / sbk_gemm_tn_f32; one token-range split (plain
    stores, run-to-run identical) under torch.use_deterministic_algorithms."""
    det = torch.are_deterministic_algorithms_enabled()
    L = lib()
    if a.dtype == _bf16:
        rc = (L.sbk_gemm_tn_cfg(ptr(a), lda, sa, ptr(b), ldb, sb, M, N, K, batch, ptr(out), ldc, sc, 0, 1, stream_of(a))
              if det else L.sbk_gemm_tn(ptr(a), lda, sa, ptr(b), ldb, sb, M, N, K, batch, ptr(out), ldc, sc, stream_of(a)))
    else:
        rc = L.sbk_gemm_tn_f32(ptr(a), lda, sa, ptr(b), ldb, sb, M, N, K, batch, ptr(out), ldc, sc, int(det),
                               stream_of(a))
    check(rc, "sbk_gemm_tn")


@_gemm_tn_op.register_fake
def _(a, b):
    return a.new_empty(*a.shape[:-2], a.shape[-1], b.shape[-1], dtype=_f32)


def gemm_tn(a, b):
    """a^T @ b in fp32 for a (K, M), b (K, N) (or batched (Bt, K, *)), both
    bf16 (sbk_gemm_tn: rows 16-B aligned, M, N % 8 == 0) or both fp32
    (sbk_gemm_tn_f32, exact-f32 MFMA, any shape): the weight gradient dY^T X
    without transposing the token-major operands.  Columns contiguous."""
    require_device(a, b)
    if a.dtype != b.dtype or a.dtype not in (_bf16, _f32):
        raise TypeError(f"gemm_tn takes two bf16 or two fp32 operands (got {a.dtype}, {b.dtype})")
    if a.stride(-1) != 1 or b.stride(-1) != 1:
        raise ValueError("gemm_tn operands must be column-contiguous")
    return OPS.gemm_tn(a, b)


def gemm_tn_into(a, b, out, ldc, sC):
    """out (fp32, caller-initialised) += a[z]^T b[z] with batch z of the
    result at out + z * sC, rows ldc apart (e.g. per-head blocks of one
    (rows, H*dh) matrix).  a (Bt, K, M), b (Bt, K, N), same dtype."""
    require_device(a, b, out)
    Bt, K, M = a.shape
    N = b.shape[-1]
    if a.dtype != b.dtype or out.dtype != _f32 or a.stride(-1) != 1 or b.stride(-1) != 1:
        raise ValueError("gemm_tn_into: same-dtype column-contiguous operands, fp32 out")
    if out.numel() < (Bt - 1) * sC + (M - 1) * ldc + N:
        raise ValueError("gemm_tn_into: output too small")
    _tn_call(a, a.stride(1), a.stride(0), b, b.stride(1), b.stride(0), M, N, K, Bt, out, ldc, sC)
    return out


@custom_op("sbk::gemm_batched", mutates_args=())
def _gemm_batched_op(a: torch.Tensor, w: torch.Tensor, out_bf16: bool, M: int, zdiv: int, ldc: int, sC: int,
                     sCo: int, rows: int) -> torch.Tensor:
    Bt, _, K = a.shape
    N = w.shape[1]
    if zdiv:
        out = torch.empty(rows, ldc, device=a.device, dtype=_bf16 if out_bf16 else _f32)
    else:
        out = torch.empty(Bt, M, N, device=a.device, dtype=_bf16 if out_bf16 else _f32)
        ldc, sC = N, M * N
    check(lib().sbk_gemm_batched(int(_is_bf16(a)), ptr(a), a.stride(1), a.stride(0), ptr(w), w.stride(1), w.stride(0),
                                 M, N, K, Bt, ptr(out), ldc, sC, zdiv, sCo, int(out_bf16), stream_of(a)),
          "sbk_gemm_batched")
    return out


@_gemm_batched_op.register_fake
def _(a, w, out_bf16, M, zdiv, ldc, sC, sCo, rows):
    dt = _bf16 if out_bf16 else _f32
    if zdiv:
        return a.new_empty(rows, ldc, dtype=dt)
    return a.new_empty(a.shape[0], M, w.shape[1], dtype=dt)


def gemm_batched(a, w, out_dtype=_f32, M=None, heads=None):
    """a[z] @ w[z]^T for a (Bt, Ma, K), w (Bt, N, K), both bf16 or both fp32,
    K-contiguous rows (batch strides arbitrary): (Bt, M, N) in out_dtype over
    the first M (default Ma) rows of each a[z].  heads=H: batch z = b*H + h is
    written into a (Bt/H * M, H*N) matrix at rows b*M.., columns h*N.. — the
    per-head products merged into the (B*T, H*dh) layout in the same launch."""
    require_device(a, w)
    if a.dtype != w.dtype or a.dtype not in (_bf16, _f32):
        raise TypeError(f"gemm_batched takes two bf16 or two fp32 operands (got {a.dtype}, {w.dtype})")
    if a.stride(-1) != 1 or w.stride(-1) != 1:
        raise ValueError("gemm_batched operands must be K-contiguous")
    Bt, Ma, _ = a.shape
    N = w.shape[1]
    M = Ma if M is None else int(M)
    if not 0 < M <= Ma:
        raise ValueError("gemm_batched: M out of range")
    if heads:
        H = int(heads)
        if Bt % H:
            raise ValueError("gemm_batched: batch not a multiple of heads")
        return OPS.gemm_batched(a, w, out_dtype == _bf16, M, H, H * N, N, M * H * N, Bt // H * M)
    return OPS.gemm_batched(a, w, out_dtype == _bf16, M, 0, 0, 0, 0, 0)


@custom_op("sbk::length_mask", mutates_args=())
def _length_mask_op(rel_len: torch.Tensor, T: int) -> torch.Tensor:
    B = rel_len.shape[0]
    out = torch.empty(B, T, device=rel_len.device, dtype=torch.uint8)
    check(lib().sbk_length_mask(ptr(rel_len), B, int(T), ptr(out), stream_of(rel_len)), "sbk_length_mask")
    return out


@_length_mask_op.register_fake
def _(rel_len, T):
    return rel_len.new_empty(rel_len.shape[0], T, dtype=torch.uint8)


def length_mask(rel_len, T):
    """(B, T) uint8: t > floor(rel_len[b] * T) — one launch."""
    require_device(rel_len)
    rl = rel_len if (rel_len.dtype == _f32 and rel_len.is_contiguous()) else rel_len.float().contiguous()
    return OPS.length_mask(rl, int(T))


@custom_op("sbk::gemm_ln", mutates_args=())
def _gemm_ln_op(a: torch.Tensor, w: torch.Tensor, g: torch.Tensor, b: torch.Tensor, eps: float,
                bias: Optional[torch.Tensor], res: Optional[torch.Tensor], alpha: float,
                rowmask: Optional[torch.Tensor], u_bf16: bool, tile: int) -> tuple[torch.Tensor, torch.Tensor]:
    M, K = a.shape
    N = w.shape[0]
    out = torch.empty(M, N, device=a.device, dtype=_f32)
    u = torch.empty(M, N, device=a.device, dtype=_bf16 if u_bf16 else _f32)
    rc = lib().sbk_gemm_ln(int(_is_bf16(a)), ptr(a), a.stride(0), ptr(w), w.stride(0), M, N, K, ptr(bias), ptr(res),
                           res.stride(0) if res is not None else 0, float(alpha), ptr(rowmask), ptr(out),
                           out.stride(0), ptr(g), ptr(b), float(eps), ptr(u), u.stride(0), int(u_bf16),
                           int(tile), stream_of(a))
    check(rc, "sbk_gemm_ln")
    return out, u


@_gemm_ln_op.register_fake
def _(a, w, g, b, eps, bias, res, alpha, rowmask, u_bf16, tile):
    return (a.new_empty(a.shape[0], w.shape[0], dtype=_f32),
            a.new_empty(a.shape[0], w.shape[0], dtype=_bf16 if u_bf16 else _f32))


def gemm_ln(a, w, ln, bias=None, res=None, alpha=1.0, rowmask=None, out=None, u_dtype=_bf16, tile=0):
    """out = res + alpha * (a @ w.T + bias) (fp32) and u = LN(out; *ln) in one
    launch (N == 256).  Returns (out, u)."""
    require_device(a, w)
    if out is not None:
        raise ValueError("gemm_ln allocates its output (out= is not supported)")
    if a.dtype != w.dtype:
        raise TypeError(f"gemm operand dtypes differ: {a.dtype} vs {w.dtype}")
    if res is not None and (res.dtype != _f32 or res.stride(-1) != 1):
        raise ValueError("residual must be fp32, row-contiguous")
    g, b, eps = ln
    return OPS.gemm_ln(a, w, g, b, float(eps), bias, res, float(alpha), rowmask, u_dtype == _bf16,
                                 int(tile))


# The fused projection + LayerNorm (sbk_gemm_ln) measures the same as the two
# launches it replaces at M = 12032 (15.1 vs 8.5 + 6.3 us): off by default.
USE_GEMM_LN = False


def gemm_ln_supported(N):
    return int(N) == 256


@custom_op("sbk::layernorm", mutates_args=())
def _layernorm_op(x: torch.Tensor, w1: torch.Tensor, b1: torch.Tensor, eps1: float, out1_mode: int,
                  w2: Optional[torch.Tensor], b2: Optional[torch.Tensor], eps2: float,
                  out2_bf16: bool) -> tuple[torch.Tensor, torch.Tensor]:
    """out1_mode: 0 no first output, 1 fp32, 2 bf16."""
    M, D = x.shape
    out1 = torch.empty(M, D, device=x.device, dtype=_bf16 if out1_mode == 2 else _f32) if out1_mode else None
    out2 = torch.empty(M, D, device=x.device, dtype=_bf16 if out2_bf16 else _f32) if w2 is not None else None
    rc = lib().sbk_layernorm(ptr(x), M, D, ptr(w1), ptr(b1), float(eps1), ptr(out1), int(out1_mode == 2),
                             ptr(w2), ptr(b2), float(eps2), ptr(out2), int(out2 is not None and out2_bf16),
                             stream_of(x))
    check(rc, "sbk_layernorm")
    e = x.new_empty(0)
    return (out1 if out1 is not None else e), (out2 if out2 is not None else e)


@_layernorm_op.register_fake
def _(x, w1, b1, eps1, out1_mode, w2, b2, eps2, out2_bf16):
    o1 = x.new_empty(x.shape, dtype=_bf16 if out1_mode == 2 else _f32) if out1_mode else x.new_empty(0)
    o2 = x.new_empty(x.shape, dtype=_bf16 if out2_bf16 else _f32) if w2 is not None else x.new_empty(0)
    return o1, o2


def layernorm(x, w1, b1, eps1, out1_dtype=_f32, w2=None, b2=None, eps2=1e-5, out2_dtype=_bf16, out1=None):
    """y1 = LN(x; w1, b1) (returned unless out1_dtype is None); optionally
    y2 = LN(y1; w2, b2) in one pass.  x: (M, D) fp32."""
    require_device(x)
    if out1 is not None:
        raise ValueError("layernorm allocates its output (out1= is not supported)")
    mode = 0 if out1_dtype is None else (2 if out1_dtype == _bf16 else 1)
    y1, y2 = OPS.layernorm(x, w1, b1, float(eps1), mode, w2, b2, float(eps2), out2_dtype == _bf16)
    return (y1 if mode else None), (y2 if w2 is not None else None)


def ffn_supported(D, H):
    return bool(lib().sbk_ffn_supported(int(D), int(H)))


class _ImageCache:
    """The fused FFN kernels stream their weights from one pre-laid-out image
    (sbk_ffn_image: 32-KB tiles in stream order, bank swizzle applied), built
    once per set of weight tensors and reused while none of them changes.

    An entry is keyed on its source tensors' (data_ptr, version) and holds
    them only weakly: the bf16 copies a module's WeightCache replaces after
    an optimizer step die with their last strong reference, and the entry
    (image included) is dropped with them by the weakref callback — before
    their storage can be recycled into a false hit, and without keeping dead
    images alive across a train / validate loop.  An image is built on the
    requesting stream; a hit from another stream waits on the event recorded
    after the build.  LRU-bounded as a backstop."""

    def __init__(self, cap=64):
        self.cap = cap
        self._d = {}

    def _drop(self, key):
        self._d.pop(key, None)

    def get(self, ws, np_, stream):
        key = tuple((w.data_ptr(), w._version) if w is not None else None for w in ws) + (np_,)
        hit = self._d.pop(key, None)
        if hit is None:
            w1, w2, w1b, w2b, wp = ws
            D, H = w1.shape[1], w1.shape[0]
            n = int(lib().sbk_ffn_image_elems(D, H, np_, int(w1b is not None)))
            if n <= 0:
                raise SbkError(f"sbk_ffn_image_elems: unsupported shape D={D} H={H} np={np_}")
            img = torch.empty(n, device=w1.device, dtype=_bf16)
            check(lib().sbk_ffn_image(ptr(w1), ptr(w2), ptr(w1b), ptr(w2b), ptr(wp), D, H, np_, ptr(img),
                                      ctypes.c_void_p(stream.cuda_stream)), "sbk_ffn_image")
            ev = torch.cuda.Event()
            ev.record(stream)
            refs = tuple(weakref.ref(w, lambda _r, k=key: self._drop(k)) for w in ws if w is not None)
            hit = (img, refs, ev, stream.cuda_stream)
            if len(self._d) >= self.cap:
                self._d.pop(next(iter(self._d)))
        elif hit[3] != stream.cuda_stream:
            stream.wait_event(hit[2])
        self._d[key] = hit
        return hit[0]


_FFN_IMAGES = _ImageCache()


def ffn_image(w1, w2, w1b=None, w2b=None, wp=None):
    """The weight-stream image of one FFN block (w1 (H, D), w2 (D, H) bf16),
    or of a chain (w1b, w2b), with the projection wp (np, D) bf16 appended."""
    for t in (w1, w2, w1b, w2b, wp):
        if t is not None and (t.dtype != _bf16 or not t.is_contiguous()):
            raise TypeError("ffn_image: contiguous bf16 weights")
    img = _FFN_IMAGES.get((w1, w2, w1b, w2b, wp), 0 if wp is None else wp.shape[0], torch.cuda.current_stream(w1.device))
    return img


@custom_op("sbk::ffn", mutates_args=())
def _ffn_op(x: torch.Tensor, g0: torch.Tensor, b0: torch.Tensor, e0: float, w1: torch.Tensor, b1: torch.Tensor,
            act: int, slope: float, w2: torch.Tensor, b2: torch.Tensor, alpha: float, gp: Optional[torch.Tensor],
            bp: Optional[torch.Tensor], ep: float, gn: Optional[torch.Tensor], bn: Optional[torch.Tensor], en: float,
            next_bf16: bool, deff: int) -> tuple[torch.Tensor, torch.Tensor]:
    M, D = x.shape
    H = w1.shape[0]
    img = ffn_image(w1, w2)
    out = torch.empty_like(x)
    u = torch.empty(M, D, device=x.device, dtype=_bf16 if next_bf16 else _f32) if gn is not None else None
    rc = lib().sbk_ffn(ptr(x), M, D, deff, H, ptr(g0), ptr(b0), float(e0), ptr(img), img.numel(), ptr(b1), act,
                       float(slope), ptr(b2), float(alpha), ptr(gp), ptr(bp), float(ep), ptr(out), ptr(gn), ptr(bn), float(en),
                       ptr(u), int(next_bf16), stream_of(x))
    check(rc, "sbk_ffn")
    return out, (u if u is not None else x.new_empty(0))


@_ffn_op.register_fake
def _(x, g0, b0, e0, w1, b1, act, slope, w2, b2, alpha, gp, bp, ep, gn, bn, en, next_bf16, deff):
    return (torch.empty_like(x),
            x.new_empty(x.shape, dtype=_bf16 if next_bf16 else _f32) if gn is not None else x.new_empty(0))


@custom_op("sbk::ffn_proj", mutates_args=())
def _ffn_proj_op(x: torch.Tensor, g0: torch.Tensor, b0: torch.Tensor, e0: float, w1: torch.Tensor,
                 b1: torch.Tensor, act: int, slope: float, w2: torch.Tensor, b2: torch.Tensor, alpha: float,
                 gp: Optional[torch.Tensor], bp: Optional[torch.Tensor], ep: float, gn: torch.Tensor,
                 bn: torch.Tensor, en: float, wp: torch.Tensor, deff: int) -> tuple[torch.Tensor, torch.Tensor]:
    M, D = x.shape
    H, NP = w1.shape[0], wp.shape[0]
    img = ffn_image(w1, w2, wp=wp)
    out = torch.empty_like(x)
    y = torch.empty(M, NP, device=x.device, dtype=_bf16)
    rc = lib().sbk_ffn_proj(ptr(x), M, D, deff, H, ptr(g0), ptr(b0), float(e0), ptr(img), img.numel(), ptr(b1), act,
                            float(slope), ptr(b2), float(alpha), ptr(gp), ptr(bp), float(ep), ptr(out), ptr(gn), ptr(bn),
                            float(en), None, 1, NP, ptr(y), stream_of(x))
    check(rc, "sbk_ffn_proj")
    return out, y


@_ffn_proj_op.register_fake
def _(x, g0, b0, e0, w1, b1, act, slope, w2, b2, alpha, gp, bp, ep, gn, bn, en, wp, deff):
    return torch.empty_like(x), x.new_empty((x.shape[0], wp.shape[0]), dtype=_bf16)


def ffn_proj_supported(D, H, NP):
    return ffn_supported(D, H) and NP > 0 and NP % 256 == 0


def ffn_proj(x, ln0, w1, b1, act, slope, w2, b2, alpha, next_ln, wp, post_ln=None, deff=None):
    """sbk_ffn with the following block's input projection fused on chip:
    returns (out fp32, next_ln(out) · wp^T in bf16).  wp: (NP, D) bf16, no
    bias (RelPosMHAXL's in_proj).  deff: LayerNorm statistics over the first
    deff columns (the rest zero-padded channels; default all)."""
    require_device(x, w1, w2, wp)
    gp, bp, ep = post_ln if post_ln is not None else (None, None, 0.0)
    return OPS.ffn_proj(x, ln0[0], ln0[1], float(ln0[2]), w1, b1, ACT[act], float(slope), w2, b2,
                                  float(alpha), gp, bp, float(ep), next_ln[0], next_ln[1], float(next_ln[2]), wp,
                       int(deff or x.shape[1]))


@custom_op("sbk::ffn_chain", mutates_args=())
def _ffn_chain_op(x: torch.Tensor, act: int, slope: float, g0: torch.Tensor, b0: torch.Tensor, e0: float,
                  w1: torch.Tensor, b1: torch.Tensor, w2: torch.Tensor, b2: torch.Tensor, alpha: float,
                  gp: Optional[torch.Tensor], bp: Optional[torch.Tensor], ep: float, g0b: torch.Tensor,
                  b0b: torch.Tensor, e0b: float, w1b: torch.Tensor, b1b: torch.Tensor, w2b: torch.Tensor,
                  b2b: torch.Tensor, alphab: float, gn: torch.Tensor, bn: torch.Tensor, en: float,
                  wp: torch.Tensor, deff: int) -> tuple[torch.Tensor, torch.Tensor]:
    M, D = x.shape
    H, NP = w1.shape[0], wp.shape[0]
    img = ffn_image(w1, w2, w1b, w2b, wp)
    out = torch.empty_like(x)
    y = torch.empty(M, NP, device=x.device, dtype=_bf16)
    rc = lib().sbk_ffn_chain(ptr(x), M, D, deff, H, act, float(slope), ptr(g0), ptr(b0), float(e0), ptr(b1), ptr(b2),
                             float(alpha), ptr(gp), ptr(bp), float(ep), ptr(g0b), ptr(b0b), float(e0b), ptr(b1b),
                             ptr(b2b), float(alphab), ptr(out), ptr(gn), ptr(bn), float(en), None, 1, ptr(img), img.numel(), NP,
                             ptr(y), stream_of(x))
    check(rc, "sbk_ffn_chain")
    return out, y


@_ffn_chain_op.register_fake
def _(x, act, slope, g0, b0, e0, w1, b1, w2, b2, alpha, gp, bp, ep, g0b, b0b, e0b, w1b, b1b, w2b, b2b, alphab, gn,
      bn, en, wp, deff):
    return torch.empty_like(x), x.new_empty((x.shape[0], wp.shape[0]), dtype=_bf16)


def ffn_chain(x, a, b, act, slope, next_ln, wp, deff=None):
    """Two FFN blocks in one launch — a = (ln0, w1, b1, w2, b2, alpha,
    post_ln) then b = (ln0, w1, b1, w2, b2, alpha) on a's output, which stays
    on chip — followed by next_ln and the projection wp (bf16, no bias):
    returns (b's output fp32, next_ln(out) · wp^T bf16).  The Conformer's
    FFN2 + norm2 of layer i with FFN1 + norm1 + in_proj of layer i+1."""
    require_device(x, a[1], b[1], wp)
    # one H and activation for both blocks (the kernel takes H from block a)
    if b[1].shape != a[1].shape or b[3].shape != a[3].shape:
        raise ValueError(f"ffn_chain: block shapes differ ({tuple(a[1].shape)}/{tuple(a[3].shape)} vs "
                         f"{tuple(b[1].shape)}/{tuple(b[3].shape)})")
    gp, bp, ep = a[6] if a[6] is not None else (None, None, 0.0)
    return OPS.ffn_chain(x, ACT[act], float(slope), a[0][0], a[0][1], float(a[0][2]), a[1], a[2], a[3],
                                   a[4], float(a[5]), gp, bp, float(ep), b[0][0], b[0][1], float(b[0][2]), b[1], b[2],
                                   b[3], b[4], float(b[5]), next_ln[0], next_ln[1], float(next_ln[2]), wp,
                         int(deff or x.shape[1]))


def ffn(x, ln0, w1, b1, act, slope, w2, b2, alpha, post_ln=None, next_ln=None, next_dtype=_bf16, out=None, deff=None):
    """Fused macaron FFN block (bf16 MFMA): z = x + alpha * FFN(LN0(x));
    out = post_ln(z) if given; u = next_ln(out) (returned) if given.
    x: (M, D) fp32; ln*: (weight, bias, eps); w1 (H, D), w2 (D, H) bf16.
    `out` is accepted for API compatibility and ignored (a new tensor is
    returned; the op does not alias its input)."""
    require_device(x, w1, w2)
    gp, bp, ep = post_ln if post_ln is not None else (None, None, 0.0)
    gn, bn, en = next_ln if next_ln is not None else (None, None, 0.0)
    y, u = OPS.ffn(x, ln0[0], ln0[1], float(ln0[2]), w1, b1, ACT[act], float(slope), w2, b2, float(alpha),
                             gp, bp, float(ep), gn, bn, float(en), next_dtype == _bf16, int(deff or x.shape[1]))
    return y, (u if next_ln is not None else None)


@custom_op("sbk::dwconv_ln_swish", mutates_args=())
def _dwconv_op(x: torch.Tensor, B: int, T: int, w: torch.Tensor, bias: Optional[torch.Tensor], causal: bool,
               ln_w: torch.Tensor, ln_b: torch.Tensor, eps: float, out_bf16: bool) -> torch.Tensor:
    C = x.shape[-1]
    K = w.shape[-1]
    out = torch.empty(B * T, C, device=x.device, dtype=_bf16 if out_bf16 else _f32)
    rc = lib().sbk_dwconv_ln_swish(int(_is_bf16(x)), ptr(x), B, T, C, ptr(w), ptr(bias), K, int(causal), ptr(ln_w),
                                   ptr(ln_b), float(eps), ptr(out), int(out_bf16), stream_of(x))
    check(rc, "sbk_dwconv_ln_swish")
    return out


@_dwconv_op.register_fake
def _(x, B, T, w, bias, causal, ln_w, ln_b, eps, out_bf16):
    return x.new_empty(B * T, x.shape[-1], dtype=_bf16 if out_bf16 else _f32)


def dwconv_ln_swish(x, B, T, w, bias, causal, ln_w, ln_b, eps, out_dtype):
    """Depthwise Conv1d over time + LayerNorm(C) + Swish.  x: (B*T, C)."""
    return OPS.dwconv_ln_swish(x, int(B), int(T), w, bias, bool(causal), ln_w, ln_b, float(eps),
                                         out_dtype == _bf16)


def conv_module_supported(D, K):
    return bool(lib().sbk_conv_module_supported(int(D), int(K)))


@custom_op("sbk::conv_module", mutates_args=())
def _conv_module_op(x: torch.Tensor, B: int, T: int, g0: torch.Tensor, b0: torch.Tensor, e0: float,
                    w1p: torch.Tensor, b1p: torch.Tensor, wc: torch.Tensor, bc: Optional[torch.Tensor], causal: bool,
                    g1: torch.Tensor, b1: torch.Tensor, e1: float, w2: torch.Tensor, b2: Optional[torch.Tensor],
                    kpm: Optional[torch.Tensor], o: Optional[torch.Tensor], wo: Optional[torch.Tensor],
                    bo: Optional[torch.Tensor], deff: int) -> torch.Tensor:
    K = wc.shape[0]  # wc: (K, d) tap-major
    out = torch.empty_like(x)
    rc = lib().sbk_conv_module_pre(ptr(x), ptr(o), ptr(wo), ptr(bo), ptr(out), B, T, x.shape[1], deff, ptr(g0),
                                   ptr(b0),
                                   float(e0), ptr(w1p), ptr(b1p), ptr(wc), ptr(bc), K, int(causal), ptr(g1), ptr(b1),
                                   float(e1), ptr(w2), ptr(b2), ptr(kpm), stream_of(x))
    check(rc, "sbk_conv_module_pre")
    return out


@_conv_module_op.register_fake
def _(x, B, T, g0, b0, e0, w1p, b1p, wc, bc, causal, g1, b1, e1, w2, b2, kpm, o, wo, bo, deff):
    return torch.empty_like(x)


def conv_module(x, B, T, ln0, w1p, b1p, wc, bc, causal, ln1, w2, b2, kpm=None, pre=None, deff=None):
    """Fused Conformer convolution module (bf16 MFMA, one launch):
    x + rowmask0(after_conv(dwconv(GLU(pointwise(LN0(x)))))).  x: (B*T, 256) fp32.
    pre = (o, wo, bo): the module runs on x + o wo^T + bo (the MHSA output
    projection and residual fused in; o (B*T, 256) bf16)."""
    require_device(x, w1p, w2)
    o, wo, bo = pre if pre is not None else (None, None, None)
    return OPS.conv_module(x, int(B), int(T), ln0[0], ln0[1], float(ln0[2]), w1p, b1p, wc, bc,
                                     bool(causal), ln1[0], ln1[1], float(ln1[2]), w2, b2, kpm, o, wo, bo,
                            int(deff or x.shape[1]))


@custom_op("sbk::conv_block_c1", mutates_args=())
def _conv_block_c1_op(x: torch.Tensor, w: torch.Tensor, bias: torch.Tensor, ln_w: torch.Tensor, ln_b: torch.Tensor,
                      eps: float, slope: float, out_bf16: bool) -> torch.Tensor:
    B, Tin, Fin = x.shape
    Cout = w.shape[0]
    Tout, Fout = (Tin - 1) // 2 + 1, (Fin - 1) // 2 + 1
    out = torch.empty(B, Tout, Fout, Cout, device=x.device, dtype=_bf16 if out_bf16 else _f32)
    rc = lib().sbk_conv_block_c1(ptr(x), B, Tin, Fin, Cout, ptr(w), ptr(bias), ptr(ln_w), ptr(ln_b), float(eps),
                                 float(slope), ptr(out), int(out_bf16), None, None, stream_of(x))
    check(rc, "sbk_conv_block_c1")
    return out


@_conv_block_c1_op.register_fake
def _(x, w, bias, ln_w, ln_b, eps, slope, out_bf16):
    B, Tin, Fin = x.shape
    return x.new_empty(B, (Tin - 1) // 2 + 1, (Fin - 1) // 2 + 1, w.shape[0], dtype=_bf16 if out_bf16 else _f32)


def conv_block_c1(x, w, bias, ln_w, ln_b, eps, slope, out_dtype):
    """ConvBlock with one input channel: x (B, T, F) fp32 → (B, T', F', C)."""
    require_device(x)
    return OPS.conv_block_c1(x, w, bias, ln_w, ln_b, float(eps), float(slope), out_dtype == _bf16)


@custom_op("sbk::conv_block_mfma", mutates_args=())
def _conv_block_mfma_op(x: torch.Tensor, wperm: torch.Tensor, bias: torch.Tensor, ln_w: torch.Tensor,
                        ln_b: torch.Tensor, eps: float, slope: float, out_bf16: bool) -> torch.Tensor:
    B, Tin, Fin, Cin = x.shape
    Cout = wperm.shape[0]
    Tout, Fout = (Tin - 1) // 2 + 1, (Fin - 1) // 2 + 1
    out = torch.empty(B, Tout, Fout, Cout, device=x.device, dtype=_bf16 if out_bf16 else _f32)
    rc = lib().sbk_conv_block_mfma(int(_is_bf16(x)), ptr(x), B, Tin, Fin, Cin, Cout, ptr(wperm), ptr(bias),
                                   ptr(ln_w), ptr(ln_b), float(eps), float(slope), ptr(out), int(out_bf16), None,
                                   None, stream_of(x))
    check(rc, "sbk_conv_block_mfma")
    return out


@_conv_block_mfma_op.register_fake
def _(x, wperm, bias, ln_w, ln_b, eps, slope, out_bf16):
    B, Tin, Fin, _ = x.shape
    return x.new_empty(B, (Tin - 1) // 2 + 1, (Fin - 1) // 2 + 1, wperm.shape[0],
                       dtype=_bf16 if out_bf16 else _f32)


def conv_block_mfma(x, wperm, bias, ln_w, ln_b, eps, slope, out_dtype):
    """ConvBlock implicit GEMM: x (B, T, F, Cin) → (B, T', F', Cout);
    wperm: (Cout, 3, 3, Cin) [time, freq] in x.dtype."""
    require_device(x, wperm)
    return OPS.conv_block_mfma(x, wperm, bias, ln_w, ln_b, float(eps), float(slope), out_dtype == _bf16)


@custom_op("sbk::conv_frontend2", mutates_args=())
def _conv_frontend2_op(x: torch.Tensor, w1: torch.Tensor, b1: torch.Tensor, g1: torch.Tensor, be1: torch.Tensor,
                       e1: float, s1: float, wperm2: torch.Tensor, b2: torch.Tensor, g2: torch.Tensor,
                       be2: torch.Tensor, e2: float, s2: float, out_bf16: bool, slot_max: Optional[torch.Tensor],
                       top_db: float) -> torch.Tensor:
    B, Tin, Fin = x.shape
    C1, C2 = w1.shape[0], wperm2.shape[0]
    T1, F1 = (Tin - 1) // 2 + 1, (Fin - 1) // 2 + 1
    T2, F2 = (T1 - 1) // 2 + 1, (F1 - 1) // 2 + 1
    out = torch.empty(B, T2, F2, C2, device=x.device, dtype=_bf16 if out_bf16 else _f32)
    rc = lib().sbk_conv_frontend2(int(_is_bf16(wperm2)), ptr(x), B, Tin, Fin, ptr(w1), ptr(b1), ptr(g1), ptr(be1),
                                  float(e1), float(s1), C1, ptr(wperm2), ptr(b2), ptr(g2), ptr(be2), float(e2),
                                  float(s2), C2, ptr(out), int(out_bf16), ptr(slot_max),
                                  slot_max.shape[1] if slot_max is not None else 0, float(top_db), None, None,
                                  stream_of(x))
    check(rc, "sbk_conv_frontend2")
    return out


@_conv_frontend2_op.register_fake
def _(x, w1, b1, g1, be1, e1, s1, wperm2, b2, g2, be2, e2, s2, out_bf16, slot_max, top_db):
    B, Tin, Fin = x.shape
    T1, F1 = (Tin - 1) // 2 + 1, (Fin - 1) // 2 + 1
    return x.new_empty(B, (T1 - 1) // 2 + 1, (F1 - 1) // 2 + 1, wperm2.shape[0], dtype=_bf16 if out_bf16 else _f32)


def conv_frontend2(x, blk1, blk2, wperm2, out_dtype, topdb=None):
    """Both ConvBlocks in one kernel: x (B, T, F) fp32 → (B, T2, F2, C2).
    blk*: (conv weight, bias, ln weight, ln bias, ln eps, leaky slope);
    wperm2: block-2 weights (C2, 3, 3, C1) in the compute dtype; topdb =
    (slot_max (B, nslot), top_db): x is an Fbank output before its top_db
    floor, applied on load (ops.fbank_deferred)."""
    require_device(x, wperm2)
    w1, b1, g1, be1, e1, s1 = blk1
    _, b2, g2, be2, e2, s2 = blk2
    sm, tdb = topdb if topdb is not None else (None, 0.0)
    return OPS.conv_frontend2(x, w1, b1, g1, be1, float(e1), float(s1), wperm2, b2, g2, be2, float(e2),
                                        float(s2), out_dtype == _bf16, sm, float(tdb))


@custom_op("sbk::relpos_attention", mutates_args=())
def _relpos_attention_op(qkv: torch.Tensor, pk: torch.Tensor, pbu: torch.Tensor, pbv: torch.Tensor,
                         kpm: Optional[torch.Tensor], B: int, T: int, H: int, dh: int, scale: float,
                         need_probs: bool, am: Optional[torch.Tensor], am_sb: int,
                         am_sh: int) -> tuple[torch.Tensor, torch.Tensor]:
    d = H * dh
    out = torch.empty(B * T, d, device=qkv.device, dtype=qkv.dtype)
    probs = torch.empty(B, H, T, T, device=qkv.device, dtype=_f32) if need_probs else qkv.new_empty(0, dtype=_f32)
    if am is None:
        rc = lib().sbk_relpos_attention_ld(int(_is_bf16(qkv)), ptr(qkv), ptr(pk), pk.stride(0), ptr(pbu), ptr(pbv),
                                           ptr(kpm), B, T, H, dh, float(scale), ptr(out),
                                           ptr(probs) if need_probs else None, stream_of(qkv))
    else:
        rc = lib().sbk_relpos_attention_mask(int(_is_bf16(qkv)), ptr(qkv), ptr(pk), pk.stride(0), ptr(pbu), ptr(pbv),
                                             ptr(kpm), ptr(am), am_sb, am_sh, B, T, H, dh, float(scale), ptr(out),
                                             ptr(probs) if need_probs else None, stream_of(qkv))
    check(rc, "sbk_relpos_attention")
    return out, probs


@_relpos_attention_op.register_fake
def _(qkv, pk, pbu, pbv, kpm, B, T, H, dh, scale, need_probs, am, am_sb, am_sh):
    return (qkv.new_empty(B * T, H * dh),
            qkv.new_empty(B, H, T, T, dtype=_f32) if need_probs else qkv.new_empty(0, dtype=_f32))


def attn_mask_arg(attn_mask, B, T, H, device, Lk=None):
    """RelPosMHAXL's attn_mask (attention.py:598-611) as the kernel's additive
    fp32 mask: (mask (Lq, Lk) or (B|1, H, Lq, Lk), batch stride, head stride),
    bool masks as 0 / -inf (masked_fill(-inf) == adding -inf); None -> None.
    Lq = T; Lk defaults to T (self-attention)."""
    if attn_mask is None:
        return None
    Lk = T if Lk is None else Lk
    m = attn_mask.to(device)
    if m.dtype == torch.bool:
        m = torch.zeros(m.shape, device=device, dtype=_f32).masked_fill_(m, -float("inf"))
    else:
        m = m.to(_f32)
    if m.dim() == 2:
        if tuple(m.shape) != (T, Lk):
            raise ValueError(f"attn_mask {tuple(m.shape)} != ({T}, {Lk})")
        return m.contiguous(), 0, 0
    m = m.reshape(-1, H, T, Lk).contiguous()  # the reference's view(-1, num_heads, qlen, klen)
    if m.shape[0] not in (1, B):
        raise ValueError(f"attn_mask batch {m.shape[0]} does not broadcast to {B}")
    return m, (H * T * Lk if m.shape[0] == B else 0), T * Lk


def relpos_attention(qkv, pk, pbu, pbv, kpm, B, T, H, dh, scale, need_probs=False, am=None):
    """Fused RelPosMHAXL core.  qkv: (B*T, 3d) head-interleaved, pk: (2T-1, d),
    both bf16 or fp32; am: attn_mask_arg(...) or None.  Returns (out (B*T, d)
    in qkv.dtype, probs or None)."""
    d = H * dh
    if pk.stride(-1) != 1 or pk.shape[-1] != d:
        raise ValueError("pk must be (2T-1, d) with unit column stride")
    m, sb, sh = am if am is not None else (None, 0, 0)
    out, probs = OPS.relpos_attention(qkv, pk, pbu, pbv, kpm, int(B), int(T), int(H), int(dh),
                                                float(scale), bool(need_probs), m, int(sb), int(sh))
    return out, (probs if need_probs else None)


@custom_op("sbk::relpos_xattn", mutates_args=())
def _relpos_xattn_op(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor, pk: Optional[torch.Tensor],
                     pbu: Optional[torch.Tensor], pbv: Optional[torch.Tensor], kpm: Optional[torch.Tensor],
                     am: Optional[torch.Tensor], am_sb: int, am_sh: int, B: int, Lq: int, Lk: int, H: int, dh: int,
                     scale: float, mpf: bool, p: float, seed: int) -> tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
    out = torch.empty(B * Lq, H * dh, device=q.device, dtype=q.dtype)
    probs = torch.empty(B, H, Lq, Lk, device=q.device, dtype=_f32)
    attn = torch.empty_like(probs) if p > 0 else probs.new_empty(0)
    P = pk.shape[0] if pk is not None else 2 * Lk - 1
    rc = lib().sbk_relpos_xattn_fwd(int(_is_bf16(q)), ptr(q), q.stride(0), ptr(k), k.stride(0), ptr(v), v.stride(0),
                                    ptr(pk), pk.stride(0) if pk is not None else 0, P, ptr(pbu), ptr(pbv), ptr(kpm),
                                    ptr(am), int(am_sb), int(am_sh), B, Lq, Lk, H, dh, float(scale), int(mpf),
                                    float(p), int(seed), ptr(out), out.stride(0), ptr(probs),
                                    ptr(attn) if p > 0 else None, stream_of(q))
    check(rc, "sbk_relpos_xattn_fwd")
    return out, probs, attn


@_relpos_xattn_op.register_fake
def _(q, k, v, pk, pbu, pbv, kpm, am, am_sb, am_sh, B, Lq, Lk, H, dh, scale, mpf, p, seed):
    probs = q.new_empty(B, H, Lq, Lk, dtype=_f32)
    return q.new_empty(B * Lq, H * dh), probs, (q.new_empty(B, H, Lq, Lk, dtype=_f32) if p > 0 else
                                                  q.new_empty(0, dtype=_f32))


def relpos_xattn(q, k, v, pk, pbu, pbv, kpm, B, Lq, Lk, H, dh, scale, mask_pos_future=False, am=None, p=0.0,
                 seed=0):
    """RelPosMHAXL core for query != key/value (sbk_relpos_xattn_fwd): q
    (B*Lq, d), k / v (B*Lk, d), pk (P, d) with P // 2 + 1 == Lk, unit
    column stride, bf16 or fp32 alike; pbu / pbv fp32 (H*dh); am:
    attn_mask_arg(..., Lk=Lk) or None.  pk = pbu = pbv = None: plain scaled
    dot-product attention (no positional term).  Returns (out (B*Lq, d) in
    q.dtype, probs (B, H, Lq, Lk) fp32, attention weights after dropout)."""
    for t in (q, k, v) + ((pk,) if pk is not None else ()):
        if t.stride(-1) != 1 or t.shape[-1] != H * dh or t.dtype != q.dtype:
            raise ValueError("relpos_xattn: q / k / v / pk must be (rows, H*dh), unit column stride, one dtype")
    if pk is not None and pk.shape[0] // 2 + 1 != Lk:
        raise ValueError(f"pos_embs has {pk.shape[0]} rows: rel_shift keeps {pk.shape[0] // 2 + 1} != k_len {Lk}")
    m, sb, sh = am if am is not None else (None, 0, 0)
    out, probs, attn = OPS.relpos_xattn(q, k, v, pk, pbu, pbv, kpm, m, int(sb), int(sh), int(B), int(Lq), int(Lk),
                                        int(H), int(dh), float(scale), bool(mask_pos_future), float(p), int(seed))
    return out, probs, (attn if p > 0 else probs)


@custom_op("sbk::mha_attention", mutates_args=())
def _mha_attention_op(qkv: torch.Tensor, kpm: Optional[torch.Tensor], B: int, T: int, H: int, dh: int,
                      scale: float) -> torch.Tensor:
    out = torch.empty(B * T, H * dh, device=qkv.device, dtype=qkv.dtype)
    check(lib().sbk_mha_attention(ptr(qkv), ptr(kpm), B, T, H, dh, float(scale), ptr(out), stream_of(qkv)),
          "sbk_mha_attention")
    return out


@_mha_attention_op.register_fake
def _(qkv, kpm, B, T, H, dh, scale):
    return qkv.new_empty(B * T, H * dh)


def mha_fast_ok(qkv, T, dh):
    """The band-free kernel's envelope (sbk_mha_attention)."""
    return qkv.dtype == _bf16 and dh == 64 and T <= 4096 and qkv.is_contiguous() and qkv.data_ptr() % 16 == 0


def mha_attention(qkv, kpm, B, T, H, dh, scale):
    """Plain attention core (no positional band): qkv (B*T, 3d) head-interleaved
    bf16 -> out (B*T, d) bf16.  Inside mha_fast_ok's envelope only."""
    return OPS.mha_attention(qkv, kpm, int(B), int(T), int(H), int(dh), float(scale))


def glu_group():
    """Channels per GLU pairing group (weights row-permuted in [a | gate] groups)."""
    return int(lib().sbk_gemm_glu_group(1))


@custom_op("sbk::cast_bf16", mutates_args=())
def _cast_bf16_op(x: torch.Tensor) -> torch.Tensor:
    out = torch.empty(x.shape, device=x.device, dtype=_bf16)
    check(lib().sbk_cast_bf16(ptr(x), ptr(out), x.numel(), stream_of(x)), "sbk_cast_bf16")
    return out


@_cast_bf16_op.register_fake
def _(x):
    return x.new_empty(x.shape, dtype=_bf16)


def cast_bf16(x):
    """fp32 → bf16 (round to nearest even), contiguous input."""
    return OPS.cast_bf16(x)


def to_compute(x, dtype):
    """Row-contiguous copy of x in the compute dtype (bf16 via the cast kernel;
    fp16 / bf16 activations of library ops under fp16 autocast -> fp32)."""
    if dtype == _bf16:
        return x.contiguous() if x.dtype == _bf16 else cast_bf16(x.float().contiguous())
    if x.dtype in (torch.float16, _bf16):
        return x.float().contiguous()
    if x.dtype != _f32:
        raise TypeError(f"fp32 compute path got {x.dtype}")
    return x.contiguous()


def compute_dtype():
    """bf16 MFMA under torch.autocast(device_type='cuda', dtype=bf16),
    exact-f32 MFMA otherwise — including fp16 autocast (the reference's
    `--auto_mix_prec`, core.py:905-919): there are no fp16 kernels, and the
    fp32 ones are at least as precise as the fp16 GEMMs the request stands
    for (computing bf16 instead would lose precision without telling the
    caller).  Library ops around these modules still run in fp16."""
    if torch.is_autocast_enabled("cuda"):
        dt = torch.get_autocast_dtype("cuda")
        if dt == _bf16:
            return _bf16
        if dt != torch.float16:
            raise NotImplementedError(f"speechbrain_amd kernels compute in bf16 or fp32; torch.autocast(dtype={dt})")
    return _f32


_MX = threading.local()


@contextlib.contextmanager
def mxfp8(enabled=True):
    """Run the config-5 encoder's GEMMs (wav2vec2 latent-extractor convs,
    TransformerEncoder projections) on MXFP8 operands — e4m3 elements with
    one power-of-two scale per 32 contraction elements, the block-scaled
    MFMA at 2x the bf16 rate — and the rest of the path in bf16.  GEMMs whose
    K or N is not a multiple of 128 (the MXFP8 kernel's tile) run in bf16."""
    prev = getattr(_MX, "on", False)
    _MX.on = bool(enabled)
    try:
        yield
    finally:
        _MX.on = prev


def mx_enabled():
    return getattr(_MX, "on", False)


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
