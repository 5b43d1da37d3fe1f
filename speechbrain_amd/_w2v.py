"""torch.library custom ops over the config-5 kernels (csrc/w2v.hip,
csrc/mxgemm.hip): the wav2vec2 latent extractor's layer 0, the row
LayerNorm / activation / MXFP8 quantisation kernel and the MXFP8 GEMM.

MXFP8 tensors travel as two tensors: e4m3 bytes (uint8, (M, K)) and one
E8M0 scale byte per 32 consecutive K elements (uint8, (M, K/32)).  `MX`
bundles them for the module code.  No op has a CPU path."""
import functools
from typing import NamedTuple, Optional

import torch

from ._lib import OPS, check, custom_op, lib, ptr, require_device, stream_of

_f32, _bf16, _u8 = torch.float32, torch.bfloat16, torch.uint8
OUT = {_f32: 0, _bf16: 1, "mx": 2}
ACT = {None: 0, "none": 0, "relu": 3, "gelu": 4}


class MX(NamedTuple):
    """An MXFP8 matrix: q (M, K) e4m3 bytes, s (M, K/32) E8M0 bytes."""
    q: torch.Tensor
    s: torch.Tensor


def _empty_out(M, N, mode, dev):
    if mode == 2:
        return torch.empty(M, N, device=dev, dtype=_u8), torch.empty(M, N // 32, device=dev, dtype=_u8)
    return torch.empty(M, N, device=dev, dtype=_bf16 if mode == 1 else _f32), torch.empty(0, device=dev, dtype=_u8)


def _fake_out(x, M, N, mode):
    if mode == 2:
        return x.new_empty(M, N, dtype=_u8), x.new_empty(M, N // 32, dtype=_u8)
    return x.new_empty(M, N, dtype=_bf16 if mode == 1 else _f32), x.new_empty(0, dtype=_u8)


# ---------------------------------------------------------------------------
@custom_op("sbk::w2v_wav_stats", mutates_args=())
def wav_stats(wav: torch.Tensor, eps: float) -> torch.Tensor:
    """(B, 2) [mean, rstd] of F.layer_norm(wav, wav.shape[1:]) (wav2vec.py:92-93)."""
    B, S = wav.shape
    st = torch.empty(B, 2, device=wav.device, dtype=_f32)
    check(lib().sbk_w2v_wav_stats(ptr(wav), B, S, float(eps), ptr(st), stream_of(wav)), "sbk_w2v_wav_stats")
    return st


@wav_stats.register_fake
def _(wav, eps):
    return wav.new_empty(wav.shape[0], 2)


@custom_op("sbk::w2v_conv0", mutates_args=())
def _conv0_op(wav: torch.Tensor, stats: Optional[torch.Tensor], w: torch.Tensor, g: torch.Tensor, b: torch.Tensor,
              eps: float, stride: int, out_mode: int) -> tuple[torch.Tensor, torch.Tensor]:
    B, S = wav.shape
    C, K = w.shape
    T0 = (S - K) // stride + 1
    out, sc = _empty_out(B * T0, C, out_mode, wav.device)
    check(lib().sbk_w2v_conv0(ptr(wav), ptr(stats), B, S, T0, C, K, stride, ptr(w), ptr(g), ptr(b), float(eps),
                              ptr(out), out_mode, ptr(sc) if out_mode == 2 else None, stream_of(wav)),
          "sbk_w2v_conv0")
    return out, sc


@_conv0_op.register_fake
def _(wav, stats, w, g, b, eps, stride, out_mode):
    T0 = (wav.shape[1] - w.shape[1]) // stride + 1
    return _fake_out(wav, wav.shape[0] * T0, w.shape[0], out_mode)


def conv0(wav, stats, w, g, b, eps, stride, out):
    """Layer 0 of the latent extractor: (B, S) → (B*T0, C) in `out`
    (torch.float32 | torch.bfloat16 | "mx")."""
    require_device(wav, w)
    y, s = OPS.w2v_conv0(wav.contiguous(), stats, w.contiguous(), g, b, float(eps), int(stride), OUT[out])
    return MX(y, s) if out == "mx" else y


@custom_op("sbk::ln_act", mutates_args=())
def _ln_act_op(x: torch.Tensor, g: Optional[torch.Tensor], b: Optional[torch.Tensor], eps: float, act: int,
               out_mode: int) -> tuple[torch.Tensor, torch.Tensor]:
    M, D = x.shape
    out, sc = _empty_out(M, D, out_mode, x.device)
    check(lib().sbk_ln_act(ptr(x), int(x.dtype == _bf16), x.stride(0), M, D, ptr(g), ptr(b), float(eps), act,
                           ptr(out), out.stride(0), out_mode, ptr(sc) if out_mode == 2 else None,
                           sc.stride(0) if out_mode == 2 else 0, stream_of(x)), "sbk_ln_act")
    return out, sc


@_ln_act_op.register_fake
def _(x, g, b, eps, act, out_mode):
    return _fake_out(x, x.shape[0], x.shape[1], out_mode)


def ln_act(x, ln=None, act=None, out=_f32):
    """Row LayerNorm (ln = (weight, bias, eps) or None) → activation → output
    fp32 / bf16 / "mx".  x: (M, D) fp32 or bf16, unit column stride."""
    require_device(x)
    if x.stride(-1) != 1:
        x = x.contiguous()
    g, b, eps = ln if ln is not None else (None, None, 0.0)
    y, s = OPS.ln_act(x, g, b, float(eps), ACT[act], OUT[out])
    return MX(y, s) if out == "mx" else y


@custom_op("sbk::mx_quant", mutates_args=())
def _mx_quant_op(x: torch.Tensor) -> tuple[torch.Tensor, torch.Tensor]:
    M, K = x.shape
    q = torch.empty(M, K, device=x.device, dtype=_u8)
    s = torch.empty(M, K // 32, device=x.device, dtype=_u8)
    check(lib().sbk_mx_quant(ptr(x), int(x.dtype == _bf16), x.stride(0), M, K, ptr(q), q.stride(0), ptr(s),
                             s.stride(0), stream_of(x)), "sbk_mx_quant")
    return q, s


@_mx_quant_op.register_fake
def _(x):
    return x.new_empty(x.shape, dtype=_u8), x.new_empty(x.shape[0], x.shape[1] // 32, dtype=_u8)


def mx_quant(x):
    """fp32 / bf16 (M, K) → MX (power-of-two block scales, e4m3 elements)."""
    require_device(x)
    q, s = OPS.mx_quant(x if x.stride(-1) == 1 else x.contiguous())
    return MX(q, s)


def mx_dequant(m):
    """MX → fp32 (tests)."""
    M, K = m.q.shape
    out = torch.empty(M, K, device=m.q.device, dtype=_f32)
    check(lib().sbk_mx_dequant(ptr(m.q), m.q.stride(0), ptr(m.s), m.s.stride(0), M, K, ptr(out),
                               stream_of(m.q)), "sbk_mx_dequant")
    return out


@custom_op("sbk::mx_gemm", mutates_args=())
def _mx_gemm_op(aq: torch.Tensor, asc: torch.Tensor, M: int, K: int, lda: int, ldsa: int, rpb: int, a_bs: int,
                s_bs: int, wq: torch.Tensor, wsc: torch.Tensor, bias: Optional[torch.Tensor], act: int, alpha: float,
                res: Optional[torch.Tensor], out_mode: int) -> tuple[torch.Tensor, torch.Tensor]:
    N = wq.shape[0]
    out, sc = _empty_out(M, N, out_mode, aq.device)
    # the 256-tile kernel's split-K tail workspace (config 5's FFN
    # down-projection); 0 floats at shapes that do not split
    nws = _ws_floats(M, N, K, out_mode)
    ws = torch.empty(nws, device=aq.device, dtype=_f32) if nws else None
    check(lib().sbk_mx_gemm_ws(ptr(aq), ptr(asc), lda, ldsa, rpb, a_bs, s_bs, ptr(wq), ptr(wsc), wq.stride(0),
                               wsc.stride(0), M, N, K, ptr(bias), act, float(alpha), ptr(res),
                               res.stride(0) if res is not None else 0, ptr(out), out.stride(0), out_mode,
                               ptr(sc) if out_mode == 2 else None, sc.stride(0) if out_mode == 2 else 0, ptr(ws), nws,
                               stream_of(aq)), "sbk_mx_gemm_ws")
    return out, sc


@functools.lru_cache(maxsize=None)
def _ws_floats(M, N, K, out_mode):
    return int(lib().sbk_mx_gemm_ws_floats(M, N, K, out_mode))


@_mx_gemm_op.register_fake
def _(aq, asc, M, K, lda, ldsa, rpb, a_bs, s_bs, wq, wsc, bias, act, alpha, res, out_mode):
    return _fake_out(aq, M, wq.shape[0], out_mode)


def mx_gemm(a, w, bias=None, act=None, alpha=1.0, res=None, out=_f32):
    """out = res + alpha * act(A·Wᵀ + bias), A and W as MX (row-major, K-contiguous)."""
    require_device(a.q, w.q)
    M, K = a.q.shape
    if w.q.shape[1] != K:
        raise ValueError(f"mx_gemm K mismatch {K} vs {w.q.shape[1]}")
    if res is not None and (res.dtype != _f32 or res.stride(-1) != 1):
        raise ValueError("residual must be fp32, row-contiguous")
    y, s = OPS.mx_gemm(a.q, a.s, M, K, a.q.stride(0), a.s.stride(0), M, 0, 0, w.q, w.s, bias, ACT[act],
                                 float(alpha), res, OUT[out])
    return MX(y, s) if out == "mx" else y


def mx_conv_gemm(x, B, T_in, C, k, stride, w, out=_f32):
    """Conv1d(C → N, kernel k, stride, "valid", no bias) over channels-last
    MX rows x (B*T_in, C) as ONE GEMM: output row (b, t) reads the k
    consecutive input rows from (b, stride*t) — K = k*C, lda = stride*C,
    batch stride T_in*C (scales likewise); w: MX of the weight permuted to
    [out][tap][in] (CNN.py:309-516, padding "valid")."""
    T_out = (T_in - k) // stride + 1
    M = B * T_out
    y, s = OPS.mx_gemm(x.q, x.s, M, k * C, stride * C, stride * C // 32, T_out, T_in * C,
                                 T_in * C // 32, w.q, w.s, None, 0, 1.0, None, OUT[out])
    return (MX(y, s) if out == "mx" else y), T_out


@custom_op("sbk::add_posenc", mutates_args=("x",))
def add_posenc(x: torch.Tensor, pe: torch.Tensor, T: int) -> None:
    """x (B*T, D) fp32 += pe[t] (EncoderWrapper: latents + positional_encoding,
    wav2vec.py:222)."""
    M, D = x.shape
    check(lib().sbk_add_rows_periodic(ptr(x), M, D, ptr(pe), int(T), stream_of(x)), "sbk_add_rows_periodic")


@add_posenc.register_fake
def _(x, pe, T):
    return None
