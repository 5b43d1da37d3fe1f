"""Autograd functions of the training path (config 4: Conformer-Transducer
under Brain DDP).

The inference path (``_enc`` + the nn.Module drop-ins) fuses whole
sub-blocks into single kernels and keeps nothing.  When gradients are
needed the modules run this chain instead: every forward op is still a
libsbk.so HIP kernel (MFMA GEMM, rel-pos attention, LayerNorm, activations,
depthwise conv, im2col), and each ``backward`` pairs HIP kernels
(csrc/backward.hip: LayerNorm / activation / depthwise-conv / softmax
backward, col2im, joint reductions) with the MFMA GEMMs for the dense
contractions: dX = dY·W on sbk_gemm, dW = dYᵀ·X on sbk_gemm_tn (bf16) /
sbk_gemm_tn_f32 (fp32), the attention products on sbk_gemm_batched.  No
library GEMM runs in either dtype.

Numerics follow torch.autocast: under bf16 the GEMM operands and the
activations saved for them are bf16, reductions, LayerNorm statistics and the
residual stream are fp32, and weight gradients are formed from bf16
operands and returned in fp32.  Without autocast everything is fp32 — the
parity path checked against autograd of the oracle restatement.
"""
import torch
from torch.autograd import Function

from . import _enc
from ._lib import check, lib, ptr, stream_of

_f32 = torch.float32
_bf16 = torch.bfloat16

ACT_CODE = {"swish": 1, "glu": 2, "leaky_relu": 3, "gelu": 4}


def _bf(t):
    return int(t.dtype == _bf16)


def _cont(t):
    return t if t.is_contiguous() else t.contiguous()


def _as(t, dtype):
    """Row-contiguous t in dtype (fp32 -> bf16 through the HIP cast kernel)."""
    t = _cont(t)
    if t.dtype == dtype:
        return t
    if dtype == _bf16 and t.dtype == _f32:
        return _enc.cast_bf16(t)
    return t.to(dtype)


def rowsum(x, out=None, accumulate=False):
    """(rows, cols) fp32/bf16 -> (cols,) fp32 column sums (Linear bias grads)."""
    x = _cont(x)
    rows, cols = x.shape
    L = lib()
    part = torch.empty(int(L.sbk_rowsum_chunks(rows)) * cols, device=x.device, dtype=_f32)
    if out is None:
        out = torch.empty(cols, device=x.device, dtype=_f32)
    check(L.sbk_rowsum(ptr(x), _bf(x), rows, cols, ptr(part), ptr(out), int(accumulate), stream_of(x)), "sbk_rowsum")
    return out


def rowsum_batched(x):
    """(batch, rows, cols) fp32/bf16 -> (batch, cols) fp32 sums over rows."""
    x = _cont(x)
    bt, rows, cols = x.shape
    L = lib()
    part = torch.empty(int(L.sbk_rowsum_chunks(rows)) * bt * cols, device=x.device, dtype=_f32)
    out = torch.empty(bt, cols, device=x.device, dtype=_f32)
    check(L.sbk_rowsum_batched(ptr(x), _bf(x), bt, rows, cols, ptr(part), ptr(out), 0, stream_of(x)),
          "sbk_rowsum_batched")
    return out


def colsum(part, rows, cols):
    out = torch.empty(cols, device=part.device, dtype=_f32)
    check(lib().sbk_colsum(ptr(part), rows, cols, ptr(out), 0, stream_of(part)), "sbk_colsum")
    return out


# ------------------------------------------------------- dropout / residual
def wgrad(g, a):
    """dW = g^T a in fp32 for g (M, N), a (M, K) — the weight gradient of a
    Linear — on the token-major weight-gradient GEMM: sbk_gemm_tn for bf16
    (16-B rows: N, K padded to multiples of 8 when they are not), the
    exact-f32 sbk_gemm_tn_f32 for fp32 (any shape)."""
    M, N = g.shape
    K = a.shape[1]
    if g.dtype == _bf16:
        a = a if a.dtype == _bf16 else _as(a, _bf16)
        if (N % 8 or K % 8 or g.stride(0) % 8 or a.stride(0) % 8 or (g.data_ptr() | a.data_ptr()) % 16
                or g.stride(1) != 1 or a.stride(1) != 1):
            # F.pad with a zero pad returns a clone that keeps the input's
            # strides: .contiguous() makes the rows dense in every case
            gp = torch.nn.functional.pad(g, (0, -N % 8)).contiguous()
            ap = torch.nn.functional.pad(a, (0, -K % 8)).contiguous()
            return _enc.gemm_tn(gp, ap)[:N, :K]
        return _enc.gemm_tn(g, a)
    return _enc.gemm_tn(_cont(g), _cont(_as(a, _f32)))


def dgrad(g, wk):
    """dX = g @ wk for g (M, N), wk (N, K) — the input gradient of a Linear —
    on the MFMA GEMM (A @ W^T with W = wk^T, a (K, N) copy of the weight)."""
    return _enc.gemm(_cont(g), _cont(wk.t()), out_dtype=g.dtype)


def drop_add(x, res=None, alpha=1.0, rowmask=None, p=0.0, seed=0, out_dtype=_f32):
    """out = res + alpha * rowmask0(dropout_p(x)) — one HIP launch (sbk_dropout_add)."""
    x = _cont(x)
    cols = x.shape[-1]
    rows = x.numel() // cols
    out = torch.empty(x.shape, device=x.device, dtype=out_dtype)
    if res is not None and (res.dtype != _f32 or not res.is_contiguous()):
        raise ValueError("residual must be fp32, contiguous")
    check(lib().sbk_dropout_add(ptr(x), _bf(x), ptr(res), rows, cols, ptr(rowmask), float(alpha), float(p),
                                int(seed), ptr(out), _bf(out), stream_of(x)), "sbk_dropout_add")
    return out


def new_seed():
    """Dropout seed drawn from torch's default CPU generator (no device sync;
    reproducible under torch.manual_seed)."""
    return int(torch.randint(0, 2 ** 62, (1,)).item())


class DropAddFn(Function):
    """res + alpha * rowmask0(Dropout(p)(x)): nn.Dropout followed by the
    residual adds / masked_fill_ of Conformer.py:242-259, :113-114."""

    @staticmethod
    def forward(ctx, x, res, alpha, rowmask, p, out_dtype):
        seed = new_seed() if p > 0 else 0
        ctx.cfg = (alpha, p, seed, x.dtype)
        ctx.save_for_backward(rowmask)
        ctx.has_res = res is not None
        return drop_add(x, res.detach() if res is not None else None, alpha, rowmask, p, seed, out_dtype)

    @staticmethod
    def backward(ctx, dy):
        (rowmask,) = ctx.saved_tensors
        alpha, p, seed, xdt = ctx.cfg
        dx = drop_add(dy, None, alpha, rowmask, p, seed, xdt) if ctx.needs_input_grad[0] else None
        return dx, (dy if ctx.has_res else None), None, None, None, None


def dropout(x, p, training, out_dtype=None):
    out_dtype = x.dtype if out_dtype is None else out_dtype
    if not training or p == 0:
        return x if x.dtype == out_dtype else _as(x, out_dtype)
    return DropAddFn.apply(x, None, 1.0, None, float(p), out_dtype)


class CastFn(Function):
    """Differentiable fp32 <-> bf16 cast (HIP cast kernel forward)."""

    @staticmethod
    def forward(ctx, x, dtype):
        ctx.src = x.dtype
        return _as(x, dtype)

    @staticmethod
    def backward(ctx, dy):
        return _as(dy, ctx.src), None


def to_dtype(x, dtype):
    x = _cont(x)
    return x if x.dtype == dtype else CastFn.apply(x, dtype)


# --------------------------------------------------------------------- Linear
class LinearFn(Function):
    """y = res + alpha * rowmask0(a @ w.T + b) (nn.Linear / 1x1 Conv1d;
    linear.py:15-76, attention.py:549-553,581,636,823-839, Conformer.py:73-92),
    residual, scale and row mask fused into the MFMA GEMM epilogue.
    a (M, K) in the compute dtype; w the fp32 parameter; wk its kernel copy."""

    @staticmethod
    def forward(ctx, a, w, bias, wk, out_dtype, res, alpha, rowmask):
        out = _enc.gemm(a, wk, bias=None if bias is None else bias.detach(), res=None if res is None else
                        res.detach(), alpha=alpha, rowmask=rowmask, out_dtype=out_dtype)
        ctx.save_for_backward(a, wk, rowmask)
        ctx.wshape = tuple(w.shape)
        ctx.has_bias = bias is not None
        ctx.has_res = res is not None
        ctx.alpha = alpha
        return out

    @staticmethod
    def backward(ctx, dy):
        a, wk, rowmask = ctx.saved_tensors
        if ctx.alpha != 1.0 or rowmask is not None:
            g = drop_add(dy, None, ctx.alpha, rowmask, 0.0, 0, a.dtype)
            gb = g if a.dtype == _f32 else None
        else:
            g = _as(dy, a.dtype)
            gb = dy
        da = dgrad(g, wk) if ctx.needs_input_grad[0] else None
        dw = wgrad(g, a).view(ctx.wshape) if ctx.needs_input_grad[1] else None
        db = None
        if ctx.has_bias and ctx.needs_input_grad[2]:
            db = rowsum(gb if gb is not None else drop_add(dy, None, ctx.alpha, rowmask, 0.0, 0, _f32))
        dres = dy if ctx.has_res and ctx.needs_input_grad[5] else None
        return da, dw, db, None, None, dres, None, None


def kernel_weight(w, dtype, cache, key):
    """Kernel-ready copy of a weight (bf16 cast cached per parameter version)."""
    w2 = w.detach().reshape(w.shape[0], -1)  # Conv1d (N, K, 1) weights as (N, K)
    if dtype == _f32:
        return _cont(w2)
    return cache.get(key, [w], lambda: _enc.cast_bf16(_cont(w2)))


def linear(a, w, bias, dtype, cache, key, out_dtype=_f32, res=None, alpha=1.0, rowmask=None):
    """Linear through LinearFn; a is cast to the compute dtype first."""
    return LinearFn.apply(to_dtype(a, dtype), w, bias, kernel_weight(w, dtype, cache, key), out_dtype, res, alpha,
                          rowmask)


# ------------------------------------------------------------------ LayerNorm
class LayerNormFn(Function):
    """Row LayerNorm of fp32 x (M, D) (normalization.py:172-223, nn.LayerNorm)."""

    @staticmethod
    def forward(ctx, x, w, b, eps, out_dtype):
        x = _cont(x)
        M, D = x.shape
        if D <= 1024:
            y, _ = _enc.layernorm(x, w.detach().reshape(-1), b.detach().reshape(-1), eps, out1_dtype=out_dtype)
        else:
            y = torch.empty(M, D, device=x.device, dtype=out_dtype)
            check(lib().sbk_layernorm_wide(ptr(x), M, D, ptr(w.detach()), ptr(b.detach()), float(eps), ptr(y),
                                           _bf(y), stream_of(x)), "sbk_layernorm_wide")
        ctx.save_for_backward(x, w)
        ctx.eps = eps
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        dy = _cont(dy)
        M, D = x.shape
        L = lib()
        nblk = int(L.sbk_layernorm_bwd_blocks(M))
        part = torch.empty(nblk * 2 * D, device=x.device, dtype=_f32)
        dx = torch.empty(M, D, device=x.device, dtype=_f32)
        check(L.sbk_layernorm_bwd(ptr(x), ptr(dy), _bf(dy), M, D, ptr(w.detach()), float(ctx.eps), None, ptr(dx),
                                  ptr(part), stream_of(x)), "sbk_layernorm_bwd")
        gb = colsum(part, nblk, 2 * D)
        return dx, gb[:D].view_as(w), gb[D:].view_as(w), None, None


def layer_norm(x, mod, out_dtype=_f32):
    return LayerNormFn.apply(x, mod.weight, mod.bias, mod.eps, out_dtype)


# ---------------------------------------------------------------- activations
class ActFn(Function):
    """Swish / GLU / LeakyReLU (activations.py:111-142, Conformer.py:73-79,
    convolution.py:169-175).  GLU halves the last dim ([a | gate])."""

    @staticmethod
    def forward(ctx, x, mode, slope, out_dtype):
        x = _cont(x)
        rows = x.shape[0]
        cols = x.shape[1] // 2 if mode == 2 else x.shape[1]
        y = torch.empty(rows, cols, device=x.device, dtype=out_dtype)
        check(lib().sbk_act_fwd(mode, ptr(x), _bf(x), rows, cols, ptr(y), _bf(y), float(slope), stream_of(x)),
              "sbk_act_fwd")
        ctx.save_for_backward(x)
        ctx.mode, ctx.slope, ctx.cols = mode, slope, cols
        return y

    @staticmethod
    def backward(ctx, dy):
        (x,) = ctx.saved_tensors
        dy = _cont(dy)
        dx = torch.empty_like(x)
        check(lib().sbk_act_bwd(ctx.mode, ptr(x), _bf(x), ptr(dy), _bf(dy), x.shape[0], ctx.cols, ptr(dx), _bf(dx),
                                float(ctx.slope), stream_of(x)), "sbk_act_bwd")
        return dx, None, None, None


def act(x, name, slope=0.0, out_dtype=None):
    return ActFn.apply(x, ACT_CODE[name], slope, x.dtype if out_dtype is None else out_dtype)


# ------------------------------------------------------------ depthwise conv
class DwConvFn(Function):
    """Depthwise Conv1d over time + bias (Conformer.py:80-86,106).
    g (B*T, C) in the compute dtype -> (B*T, C) fp32."""

    @staticmethod
    def forward(ctx, g, w, bias, B, T, causal):
        g = _cont(g)
        C = g.shape[1]
        K = w.shape[-1]
        y = torch.empty(B * T, C, device=g.device, dtype=_f32)
        wk = _cont(w.detach().reshape(C, K))
        check(lib().sbk_dwconv_fwd(ptr(g), _bf(g), B, T, C, ptr(wk), ptr(None if bias is None else bias.detach()), K,
                                   int(causal), ptr(y), 0, stream_of(g)), "sbk_dwconv_fwd")
        ctx.save_for_backward(g, wk)
        ctx.dims = (B, T, C, K, causal, bias is not None, tuple(w.shape))
        return y

    @staticmethod
    def backward(ctx, dy):
        g, wk = ctx.saved_tensors
        B, T, C, K, causal, has_bias, wshape = ctx.dims
        dy = _as(dy, _f32)
        L = lib()
        nch = int(L.sbk_dwconv_wgrad_chunks(B, T))
        part = torch.empty(nch * C * (K + 1), device=g.device, dtype=_f32)
        dg = torch.empty_like(g) if ctx.needs_input_grad[0] else None
        check(L.sbk_dwconv_bwd(ptr(g), _bf(g), ptr(dy), B, T, C, ptr(wk), K, int(causal), ptr(dg),
                               _bf(g), ptr(part), stream_of(g)), "sbk_dwconv_bwd")
        red = colsum(part, nch, C * (K + 1)).view(C, K + 1)
        dw = red[:, :K].reshape(wshape)
        db = red[:, K].contiguous() if has_bias else None
        return dg, dw, db, None, None, None


# ------------------------------------------------------ rel-pos attention
def _rup8(n):
    return (n + 7) // 8 * 8


class RelPosAttentionFn(Function):
    """RelPosMHAXL core (attention.py:566-633, rel_shift :468-483) with
    attention dropout.  qkv (B*T, 3d) head-interleaved, pk (2T-1, d), both in
    the compute dtype (bf16 or fp32); pbu / pbv the (dh, H) parameters (read
    as (H, dh), attention.py:584-590).  Returns (out (B*T, d), attention
    weights after dropout (B, H, T, T) fp32, no grad).

    Forward: the fused attention kernel (probabilities kept); with dropout,
    drop(P)·V on sbk_gemm_batched.  Backward: per-(b, h) products on
    sbk_gemm_batched / sbk_gemm_tn{,_f32} around the softmax / dropout /
    rel_shift backward kernel.  Every per-(b, h) operand is laid out over
    T and dh rounded up to 8 (zero-filled), so any T and head size takes the
    same kernels in both dtypes."""

    @staticmethod
    def forward(ctx, qkv, pk, pbu, pbv, kpm, B, T, H, dh, scale, p=0.0, am=None):
        qkv, pk = _cont(qkv), _cont(pk)
        dt = qkv.dtype
        # am: additive attn_mask (_enc.attn_mask_arg), a constant: masked
        # probabilities are 0, so the backward needs nothing of it
        o, P = _enc.relpos_attention(qkv, pk, pbu.detach(), pbv.detach(), kpm, B, T, H, dh, scale, need_probs=True,
                                     am=am)
        seed = 0
        attn = P
        if p > 0:
            # attention-probability dropout (attention.py:626): o = drop(P) V
            seed = new_seed()
            Tp, dhp = _rup8(T), _rup8(dh)
            L = lib()
            s = stream_of(qkv)
            attn = torch.empty_like(P)
            Pd = torch.empty(B * H, Tp, Tp, device=qkv.device, dtype=dt)
            check(L.sbk_attn_probs_pad(ptr(P), B * H, T, Tp, float(p), int(seed), ptr(attn), ptr(Pd), _bf(Pd), s),
                  "sbk_attn_probs_pad")
            vT = torch.empty(B * H, dhp, Tp, device=qkv.device, dtype=dt)
            check(L.sbk_attn_prep(_bf(qkv), ptr(qkv), None, None, 0, None, None, B, H, T, dh, Tp, dhp, _rup8(2 * T - 1),
                                  None, None, None, None, ptr(vT), None, None, s), "sbk_attn_prep")
            o = _enc.gemm_batched(Pd, vT[:, :dh], out_dtype=dt, M=T, heads=H)   # (B*T, H*dh)
        ctx.save_for_backward(qkv, pk, pbu, pbv, P)
        ctx.dims = (B, T, H, dh, scale, p, seed)
        ctx.mark_non_differentiable(attn)
        return o, attn

    @staticmethod
    def backward(ctx, do, _dattn_unused):
        qkv, pk, pbu, pbv, P = ctx.saved_tensors
        B, T, H, dh, scale, p, seed = ctx.dims
        dt = qkv.dtype
        W = 2 * T - 1
        Tp, dhp, Wp = _rup8(T), _rup8(dh), _rup8(W)
        BH = B * H
        dev = qkv.device
        L = lib()
        s = stream_of(qkv)
        mk = lambda *shape: torch.empty(*shape, device=dev, dtype=dt)  # noqa: E731
        # per-(b, h) operands, zero-padded to (Tp, dhp), in one launch
        qu, v, do_h, kT, qv, pkT = mk(BH, Tp, dhp), mk(BH, Tp, dhp), mk(BH, Tp, dhp), mk(BH, dhp, Tp), \
            mk(H, B * T, dhp), mk(H, dhp, Wp)
        do_c = _as(do, dt)
        check(L.sbk_attn_prep(_bf(qkv), ptr(qkv), ptr(do_c), ptr(pk), pk.stride(0), ptr(_cont(pbu.detach().float())),
                              ptr(_cont(pbv.detach().float())), B, H, T, dh, Tp, dhp, Wp, ptr(qu), ptr(qv), ptr(kT),
                              ptr(v), None, ptr(do_h), ptr(pkT), s), "sbk_attn_prep")
        dP = _enc.gemm_batched(do_h, v, out_dtype=dt)            # dO V^T  (BH, Tp, Tp)
        dS, Pd = mk(BH, Tp, Tp), mk(BH, Tp, Tp)
        dBD = mk(H, B * T, Wp)                                    # head-major, zero outside the band
        check(L.sbk_relpos_softmax_bwd_pad(_bf(dP), ptr(P), ptr(dP), B, H, T, Tp, Wp, float(scale), float(p),
                                           int(seed), ptr(dS), ptr(Pd), ptr(dBD), s), "sbk_relpos_softmax_bwd_pad")
        dv = _enc.gemm_tn(Pd, do_h)                               # Pd^T dO  (BH, Tp, dhp)
        dq_ac = _enc.gemm_batched(dS, kT)                         # dS K     (BH, Tp, dhp)
        dq_bd = _enc.gemm_batched(dBD, pkT)                       # dBD P_k  (H, B*T, dhp)
        dk = _enc.gemm_tn(dS, qu)                                 # dS^T (q + u)
        dpk = torch.zeros(Wp, H * dhp, device=dev, dtype=_f32)    # dBD^T (q + v), head h at columns h*dhp
        _enc.gemm_tn_into(dBD, qv, dpk, H * dhp, dhp)
        dqkv = torch.empty(B * T, 3 * H * dh, device=dev, dtype=dt)
        check(L.sbk_attn_dqkv(ptr(dq_ac), ptr(dq_bd), ptr(dk), ptr(dv), B, H, T, dh, Tp, dhp, ptr(dqkv), _bf(dqkv), s),
              "sbk_attn_dqkv")
        dpk = dpk[:W].view(W, H, dhp)[:, :, :dh].reshape(W, H * dh)
        dpk = _as(dpk, dt)
        # pos-bias gradients: sums of dq_ac / dq_bd over (b, t) (padded rows are zero)
        dpbv = rowsum_batched(dq_bd)[:, :dh].reshape(pbv.shape)
        dpbu = rowsum_batched(rowsum(dq_ac.view(B, H * Tp * dhp)).view(H, Tp, dhp))[:, :dh].reshape(pbu.shape)
        return dqkv, dpk, dpbu, dpbv, None, None, None, None, None, None, None, None


class RelPosCrossAttnFn(Function):
    """RelPosMHAXL core with query != key/value and q_len != k_len
    (attention.py:554-639, rel_shift :468-483) on csrc/xattn.hip: q (B*Lq, d),
    k / v (B*Lk, d), pk (P, d) in the compute dtype; pbu / pbv the (dh, H)
    parameters.  pk = pbu = pbv = None: plain scaled dot-product attention
    (the MultiheadAttention drop-in; no positional term computed or
    differentiated).  Returns (out (B*Lq, d), attention weights after dropout,
    no grad).  Backward: sbk_relpos_xattn_bwd (score, query, key / value and,
    with a band, the band passes) and the pos-bias column sums on sbk_rowsum."""

    @staticmethod
    def forward(ctx, q, k, v, pk, pbu, pbv, kpm, am, B, Lq, Lk, H, dh, scale, mpf, p):
        q, k, v = _cont(q), _cont(k), _cont(v)
        seed = new_seed() if p > 0 else 0
        nopos = pk is None
        if nopos:
            u = vb = None
        else:
            pk = _cont(pk)
            u, vb = _cont(pbu.detach().float()), _cont(pbv.detach().float())
        o, probs, attn = _enc.relpos_xattn(q, k, v, pk, u, vb, kpm, B, Lq, Lk, H, dh, scale, mpf, am, p, seed)
        ctx.save_for_backward(q, k, v, pk, u, vb, probs)
        ctx.dims = (B, Lq, Lk, H, dh, scale, mpf, p, seed, None if nopos else tuple(pbu.shape),
                    None if nopos else tuple(pbv.shape))
        ctx.mark_non_differentiable(attn)
        return o, attn

    @staticmethod
    def backward(ctx, do, _dattn_unused):
        q, k, v, pk, u, vb, probs = ctx.saved_tensors
        B, Lq, Lk, H, dh, scale, mpf, p, seed, ushape, vshape = ctx.dims
        d = H * dh
        nopos = pk is None
        P = 2 * Lk - 1 if nopos else pk.shape[0]
        dt = q.dtype
        dev = q.device
        f32 = lambda *shape: torch.empty(*shape, device=dev, dtype=_f32)  # noqa: E731
        G, dq, dk, dv = f32(B * H * Lq * Lk), f32(B * Lq, d), f32(B * Lk, d), f32(B * Lk, d)
        dqu = dqv = dpk = None
        if not nopos:
            dqu, dqv, dpk = f32(B * Lq, d), f32(B * Lq, d), f32(P, d)
        do_c = _as(do, dt)
        check(lib().sbk_relpos_xattn_bwd(_bf(q), ptr(q), q.stride(0), ptr(k), k.stride(0), ptr(v), v.stride(0),
                                         ptr(pk), 0 if nopos else pk.stride(0), P, ptr(u), ptr(vb), ptr(probs),
                                         ptr(do_c), do_c.stride(0), B, Lq, Lk, H, dh, float(scale), int(mpf),
                                         float(p), int(seed), ptr(G), ptr(dqu), ptr(dqv), ptr(dq), ptr(dk), ptr(dv),
                                         ptr(dpk), stream_of(q)), "sbk_relpos_xattn_bwd")
        if nopos:
            return (_as(dq, dt), _as(dk, dt), _as(dv, dt), None, None, None) + (None,) * 10
        dpbu = rowsum(dqu).view(ushape)
        dpbv = rowsum(dqv).view(vshape)
        return (_as(dq, dt), _as(dk, dt), _as(dv, dt), _as(dpk, dt), dpbu, dpbv) + (None,) * 10


# --------------------------------------------------------------- ConvBlock
class ConvBlockFn(Function):
    """One ConvBlock layer (convolution.py:112-175): Conv2d with "same"
    reflect padding (CNN.py:616-700) -> [LayerNorm over (freq, chan)] ->
    [LeakyReLU], as im2col (HIP) + MFMA GEMM + wide LayerNorm + activation.
    geom = (kT, kF, sT, sF[, pT, pF]): time / freq kernel and stride, and
    the reflect padding per side (default (k - 1) / 2 for odd kernels,
    get_padding_elem :1459-1481; 0 = "valid").  ln_w None: no norm
    (ln_b, eps ignored); slope None: no activation (the residual branch's
    1x1 conv + norm).  x (B, Ti, Fi, Ci) -> (B, To, Fo, Co)."""

    @staticmethod
    def forward(ctx, x, w, bias, ln_w, ln_b, eps, slope, dtype, out_dtype, geom):
        x = _cont(x)
        kt, kf, st, sf = geom[:4]
        pt, pf = geom[4:] if len(geom) == 6 else ((kt - 1) // 2, (kf - 1) // 2)
        B, Ti, Fi, Ci = x.shape
        Co = w.shape[0]
        To, Fo = (Ti + 2 * pt - kt) // st + 1, (Fi + 2 * pf - kf) // sf + 1
        vec = 8 if dtype == _bf16 else 4
        K = kt * kf * Ci
        ldcol = -(-K // vec) * vec
        N = B * To * Fo
        L = lib()
        s = stream_of(x)
        col = torch.empty(N, ldcol, device=x.device, dtype=dtype)
        check(L.sbk_im2col(ptr(x), _bf(x), B, Ti, Fi, Ci, kt, kf, st, sf, pt, pf, ldcol, ptr(col), _bf(col), s),
              "sbk_im2col")
        # weight (Co, Ci, kF, kT) -> (Co, kT, kF, Ci) -> (Co, ldcol)
        wp = torch.zeros(Co, ldcol, device=x.device, dtype=_f32)
        wp[:, :K] = w.detach().permute(0, 3, 2, 1).reshape(Co, K)
        wk = _as(wp, dtype)
        D = Fo * Co
        has_ln, has_act = ln_w is not None, slope is not None
        c = _enc.gemm(col, wk, bias=None if bias is None else bias.detach(),
                      out_dtype=_f32 if (has_ln or has_act) else out_dtype)
        c2 = c.view(B * To, D)
        n = c2
        if has_ln:
            n = torch.empty(B * To, D, device=x.device, dtype=_f32 if has_act else out_dtype)
            check(L.sbk_layernorm_wide(ptr(c2), B * To, D, ptr(ln_w.detach()), ptr(ln_b.detach()), float(eps),
                                       ptr(n), _bf(n), s), "sbk_layernorm_wide")
        y = n
        if has_act:
            y = torch.empty(B * To, D, device=x.device, dtype=out_dtype)
            check(L.sbk_act_fwd(3, ptr(n), 0, B * To, D, ptr(y), _bf(y), float(slope), s), "sbk_act_fwd")
        ctx.save_for_backward(col, wk, c2 if has_ln else None, n if has_act else None, ln_w)
        ctx.dims = (B, Ti, Fi, Ci, Co, To, Fo, ldcol, eps, slope, bias is not None, tuple(w.shape), x.dtype,
                    (kt, kf, st, sf, pt, pf))
        return y.view(B, To, Fo, Co)

    @staticmethod
    def backward(ctx, dy):
        col, wk, c2, n, ln_w = ctx.saved_tensors
        B, Ti, Fi, Ci, Co, To, Fo, ldcol, eps, slope, has_bias, wshape, xdt, (kt, kf, st, sf, pt, pf) = ctx.dims
        L = lib()
        s = stream_of(col)
        D = Fo * Co
        dy = _cont(dy).view(B * To, D)
        dn = dy
        if slope is not None:
            dn = torch.empty(B * To, D, device=col.device, dtype=_f32)
            check(L.sbk_act_bwd(3, ptr(n), _bf(n), ptr(dy), _bf(dy), B * To, D, ptr(dn), 0, float(slope), s),
                  "sbk_act_bwd")
        dlw = dlb = None
        dc = dn
        if ln_w is not None:
            nblk = int(L.sbk_layernorm_bwd_blocks(B * To))
            part = torch.empty(nblk * 2 * D, device=col.device, dtype=_f32)
            dc = torch.empty(B * To, D, device=col.device, dtype=_f32)
            check(L.sbk_layernorm_bwd(ptr(c2), ptr(dn), _bf(dn), B * To, D, ptr(ln_w.detach()), float(eps), None,
                                      ptr(dc), ptr(part), s), "sbk_layernorm_bwd")
            gb = colsum(part, nblk, 2 * D)
            dlw, dlb = gb[:D].view_as(ln_w), gb[D:].view_as(ln_w)
        dc = _cont(dc).view(B * To * Fo, Co)
        g = _as(dc, col.dtype)
        K = kt * kf * Ci
        dwp = wgrad(g, col)  # (Co, ldcol)
        dw = dwp[:, :K].reshape(Co, kt, kf, Ci).permute(0, 3, 2, 1).reshape(wshape)
        db = rowsum(dc) if has_bias else None
        dx = None
        if ctx.needs_input_grad[0]:
            dcol = dgrad(g, wk)  # (N, ldcol)
            dx = torch.empty(B, Ti, Fi, Ci, device=col.device, dtype=xdt)
            check(L.sbk_col2im(ptr(dcol), _bf(dcol), B, Ti, Fi, Ci, kt, kf, st, sf, pt, pf, ldcol, ptr(dx), _bf(dx),
                               s), "sbk_col2im")
        return dx, dw, db, dlw, dlb, None, None, None, None, None


class Conv2dXFn(Function):
    """The standalone Conv2d's general geometry (CNN.py:616-700): dilation,
    per-side padding and the F.pad modes, as sbk_im2col_x + the MFMA GEMM.
    geom = (kT, kF, sT, sF, dT, dF, pT, pF, To, Fo, mode) with pT / pF the
    leading pads and mode 0 reflect, 1 zeros, 2 replicate, 3 circular.
    x (B, Ti, Fi, Ci) -> (B, To, Fo, Co); w (Co, Ci, kF, kT)."""

    @staticmethod
    def forward(ctx, x, w, bias, dtype, out_dtype, geom):
        x = _cont(x)
        kt, kf, st, sf, dt, df, pt, pf, To, Fo, mode = geom
        B, Ti, Fi, Ci = x.shape
        Co = w.shape[0]
        vec = 8 if dtype == _bf16 else 4
        K = kt * kf * Ci
        ldcol = -(-K // vec) * vec
        L = lib()
        s = stream_of(x)
        col = torch.empty(B * To * Fo, ldcol, device=x.device, dtype=dtype)
        check(L.sbk_im2col_x(ptr(x), _bf(x), B, Ti, Fi, Ci, kt, kf, st, sf, dt, df, pt, pf, To, Fo, mode, ldcol,
                             ptr(col), _bf(col), s), "sbk_im2col_x")
        wp = torch.zeros(Co, ldcol, device=x.device, dtype=_f32)
        wp[:, :K] = w.detach().permute(0, 3, 2, 1).reshape(Co, K)
        wk = _as(wp, dtype)
        c = _enc.gemm(col, wk, bias=None if bias is None else bias.detach(), out_dtype=out_dtype)
        ctx.save_for_backward(col, wk)
        ctx.dims = (B, Ti, Fi, Ci, Co, ldcol, bias is not None, tuple(w.shape), x.dtype, geom)
        return c.view(B, To, Fo, Co)

    @staticmethod
    def backward(ctx, dy):
        col, wk = ctx.saved_tensors
        B, Ti, Fi, Ci, Co, ldcol, has_bias, wshape, xdt, geom = ctx.dims
        kt, kf, st, sf, dt, df, pt, pf, To, Fo, mode = geom
        dc = _cont(dy).view(B * To * Fo, Co)
        g = _as(dc, col.dtype)
        K = kt * kf * Ci
        dw = wgrad(g, col)[:, :K].reshape(Co, kt, kf, Ci).permute(0, 3, 2, 1).reshape(wshape)
        db = rowsum(dc) if has_bias else None
        dx = None
        if ctx.needs_input_grad[0]:
            dcol = dgrad(g, wk)
            Tp, Fp = (To - 1) * st + (kt - 1) * dt + 1, (Fo - 1) * sf + (kf - 1) * df + 1
            dxpad = torch.empty(B * Tp * Fp * Ci, device=col.device, dtype=_f32)
            dx = torch.empty(B, Ti, Fi, Ci, device=col.device, dtype=xdt)
            check(lib().sbk_col2im_x(ptr(dcol), _bf(dcol), B, Ti, Fi, Ci, kt, kf, st, sf, dt, df, pt, pf, To, Fo,
                                     mode, ldcol, ptr(dxpad), ptr(dx), _bf(dx), stream_of(col)), "sbk_col2im_x")
        return dx, dw, db, None, None, None


# ---------------------------------------------------------- transducer joint
class JointFn(Function):
    """Transducer_joint "sum" + nonlinearity (transducer_joint.py:57-95):
    tn (B, T, J), pn (B, U1, J) fp32 -> z (B, T, U1, J)."""

    @staticmethod
    def forward(ctx, tn, pn, act_code, slope, out_dtype):
        tn, pn = _as(tn, _f32), _as(pn, _f32)
        B, T, J = tn.shape
        U1 = pn.shape[1]
        z = torch.empty(B, T, U1, J, device=tn.device, dtype=out_dtype)
        check(lib().sbk_joint_fwd(ptr(tn), ptr(pn), B, T, U1, J, act_code, float(slope), ptr(z), _bf(z),
                                  stream_of(tn)), "sbk_joint_fwd")
        ctx.save_for_backward(tn, pn)
        ctx.a = (act_code, slope)
        return z

    @staticmethod
    def backward(ctx, dz):
        tn, pn = ctx.saved_tensors
        B, T, J = tn.shape
        U1 = pn.shape[1]
        dz = _cont(dz)
        dtn = torch.empty_like(tn)
        dpn = torch.empty_like(pn)
        L = lib()
        ws = torch.empty(int(L.sbk_joint_bwd_workspace_floats(B, T, U1, J)), device=tn.device, dtype=_f32)
        check(L.sbk_joint_bwd(ptr(tn), ptr(pn), ptr(dz), _bf(dz), B, T, U1, J, ctx.a[0], float(ctx.a[1]), ptr(dtn),
                              ptr(dpn), ptr(ws), stream_of(tn)), "sbk_joint_bwd")
        return dtn, dpn, None, None, None


def needs_grad(*tensors_or_modules):
    """True when autograd must see this call (grad mode on and something requires grad)."""
    if not torch.is_grad_enabled():
        return False
    for t in tensors_or_modules:
        if isinstance(t, torch.Tensor):
            if t.requires_grad:
                return True
        elif isinstance(t, torch.nn.Module):
            if any(p.requires_grad for p in t.parameters()):
                return True
    return False
