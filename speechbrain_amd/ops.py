"""torch.library custom ops over the sbk C ABI.

Every op launches hand-written HIP kernels (libsbk.so) on the current stream
of the input's device; none has a CPU or eager-PyTorch implementation.  The
`register_fake` rules only describe output shapes, so modules stay
traceable (torch.jit.trace / torch.compile graph capture) as the reference's
tests require (tests/unittests/test_features.py:14,39,56,66,97,107).
"""
import ctypes

import numpy as np
import torch

from . import _lib
from ._lib import check, custom_op, ptr, require_device, stream_of

_f32 = torch.float32


def _c(t):
    return t if t.is_contiguous() else t.contiguous()


# ---------------------------------------------------------------------------
# spectral front-end
# ---------------------------------------------------------------------------

PAD_MODES = {"constant": 0, "reflect": 1, "replicate": 2, "circular": 3}


def n_frames(S, n_fft, hop, center):
    pad = n_fft // 2 if center else 0
    return 1 + (S + 2 * pad - n_fft) // hop


@custom_op("sbk::stft", mutates_args=())
def stft(x: torch.Tensor, window: torch.Tensor, tw_nc: torch.Tensor, tw_nfft: torch.Tensor,
         n_fft: int, hop: int, center: bool, pad_mode: int, onesided: bool, normalized: bool) -> torch.Tensor:
    """torch.stft(return_complex=False) layout (features.py:161-183):
    (B,S)->(B,T,F,2); (B,S,C)->(B,T,F,2,C)."""
    require_device(x, window, tw_nc, tw_nfft)
    x = _c(x.to(_f32))
    B, S = x.shape[0], x.shape[1]
    C = x.shape[2] if x.dim() == 3 else 1
    T = n_frames(S, n_fft, hop, center)
    Fo = n_fft // 2 + 1 if onesided else n_fft
    if x.dim() == 3:
        out = torch.empty(B, T, Fo, 2, C, device=x.device, dtype=_f32)
        strides = [T * Fo * 2 * C, 1, Fo * 2 * C, 2 * C, C]
    else:
        out = torch.empty(B, T, Fo, 2, device=x.device, dtype=_f32)
        strides = [T * Fo * 2, 0, Fo * 2, 2, 1]
    st = np.array(strides, dtype=np.int64)
    st_p = st.ctypes.data_as(ctypes.c_void_p)
    scale = float(n_fft) ** -0.5 if normalized else 1.0
    rc = _lib.lib().sbk_spectrum(0, ptr(x), B, S, C, n_fft, hop, int(center), pad_mode, T, ptr(window),
                                 ptr(tw_nc), ptr(tw_nfft), int(onesided), scale, 1.0, 0.0, 0, st_p,
                                 None, None, None, None, 0, 0, 0, 0.0, 0.0, 0.0, ptr(out), None, stream_of(x))
    check(rc, "sbk_spectrum(stft)")
    return out


@stft.register_fake
def _(x, window, tw_nc, tw_nfft, n_fft, hop, center, pad_mode, onesided, normalized):
    T = n_frames(x.shape[1], n_fft, hop, center)
    Fo = n_fft // 2 + 1 if onesided else n_fft
    if x.dim() == 3:
        return x.new_empty(x.shape[0], T, Fo, 2, x.shape[2])
    return x.new_empty(x.shape[0], T, Fo, 2)


@custom_op("sbk::power_spectrum", mutates_args=())
def power_spectrum(x: torch.Tensor, window: torch.Tensor, tw_nc: torch.Tensor, tw_nfft: torch.Tensor,
                   n_fft: int, hop: int, center: bool, pad_mode: int, normalized: bool,
                   power: float, eps: float, log_mag: bool) -> torch.Tensor:
    """Fused STFT → spectral_magnitude for mono (B,S) input → (B,T,F)."""
    require_device(x, window, tw_nc, tw_nfft)
    x = _c(x.to(_f32))
    B, S = x.shape
    T = n_frames(S, n_fft, hop, center)
    Fo = n_fft // 2 + 1
    out = torch.empty(B, T, Fo, device=x.device, dtype=_f32)
    st = np.array([T * Fo, 0, Fo, 1, 0], dtype=np.int64)
    scale = float(n_fft) ** -0.5 if normalized else 1.0
    rc = _lib.lib().sbk_spectrum(1, ptr(x), B, S, 1, n_fft, hop, int(center), pad_mode, T, ptr(window),
                                 ptr(tw_nc), ptr(tw_nfft), 1, scale, float(power), float(eps), int(log_mag),
                                 st.ctypes.data_as(ctypes.c_void_p), None, None, None, None, 0, 0, 0, 0.0, 0.0,
                                 0.0, ptr(out), None, stream_of(x))
    check(rc, "sbk_spectrum(power)")
    return out


@power_spectrum.register_fake
def _(x, window, tw_nc, tw_nfft, n_fft, hop, center, pad_mode, normalized, power, eps, log_mag):
    return x.new_empty(x.shape[0], n_frames(x.shape[1], n_fft, hop, center), n_fft // 2 + 1)


@custom_op("sbk::fbank", mutates_args=())
def fbank(x: torch.Tensor, window: torch.Tensor, tw_nc: torch.Tensor, tw_nfft: torch.Tensor,
          mel_start: torch.Tensor, mel_len: torch.Tensor, mel_off: torch.Tensor, mel_w: torch.Tensor,
          n_fft: int, hop: int, center: bool, pad_mode: int, n_mels: int, log_mel: bool,
          multiplier: float, db_offset: float, amin: float, top_db: float) -> torch.Tensor:
    """Fused Fbank: wav (B,S) → STFT → |X|^2 → mel → dB → top_db (B,T,M).
    lobes/features.py:130-147 with processing/features.py:133-188,327-356,490-560,691-712."""
    require_device(x, window, tw_nc, tw_nfft, mel_start, mel_len, mel_off, mel_w)
    x = _c(x.to(_f32))
    B, S = x.shape
    T = n_frames(S, n_fft, hop, center)
    out = torch.empty(B, T, n_mels, device=x.device, dtype=_f32)
    L = _lib.lib()
    nslot = L.sbk_spectrum_slots(n_fft, hop, T, n_mels, mel_w.numel())
    slot_max = torch.empty(B, max(nslot, 1), device=x.device, dtype=_f32)
    s = stream_of(x)
    rc = L.sbk_spectrum(2, ptr(x), B, S, 1, n_fft, hop, int(center), pad_mode, T, ptr(window), ptr(tw_nc),
                        ptr(tw_nfft), 1, 1.0, 1.0, 0.0, 0, None, ptr(mel_start), ptr(mel_len), ptr(mel_off),
                        ptr(mel_w), mel_w.numel(), n_mels, int(log_mel), multiplier, db_offset, amin, ptr(out),
                        ptr(slot_max), s)
    check(rc, "sbk_spectrum(fbank)")
    if log_mel:
        check(L.sbk_topdb_clamp(ptr(out), ptr(slot_max), nslot, T * n_mels, B, top_db, s), "sbk_topdb_clamp")
    return out


@fbank.register_fake
def _(x, window, tw_nc, tw_nfft, mel_start, mel_len, mel_off, mel_w, n_fft, hop, center, pad_mode, n_mels,
      log_mel, multiplier, db_offset, amin, top_db):
    return x.new_empty(x.shape[0], n_frames(x.shape[1], n_fft, hop, center), n_mels)


@custom_op("sbk::fbank_deferred", mutates_args=())
def fbank_deferred(x: torch.Tensor, window: torch.Tensor, tw_nc: torch.Tensor, tw_nfft: torch.Tensor,
                   mel_start: torch.Tensor, mel_len: torch.Tensor, mel_off: torch.Tensor, mel_w: torch.Tensor,
                   n_fft: int, hop: int, center: bool, pad_mode: int, n_mels: int, multiplier: float,
                   db_offset: float, amin: float) -> tuple[torch.Tensor, torch.Tensor]:
    """fbank (log_mel) WITHOUT the top_db floor: (dB features (B,T,M), the
    per-workgroup partial maxima (B, nslot)).  The consumer applies
    max(x, max_b - top_db) as it loads the rows (sbk_conv_frontend2), so the
    clamp pass over the features never runs; features.py:691-712 otherwise."""
    require_device(x, window, tw_nc, tw_nfft, mel_start, mel_len, mel_off, mel_w)
    x = _c(x.to(_f32))
    B, S = x.shape
    T = n_frames(S, n_fft, hop, center)
    out = torch.empty(B, T, n_mels, device=x.device, dtype=_f32)
    L = _lib.lib()
    nslot = L.sbk_spectrum_slots(n_fft, hop, T, n_mels, mel_w.numel())
    slot_max = torch.empty(B, max(nslot, 1), device=x.device, dtype=_f32)
    rc = L.sbk_spectrum(2, ptr(x), B, S, 1, n_fft, hop, int(center), pad_mode, T, ptr(window), ptr(tw_nc),
                        ptr(tw_nfft), 1, 1.0, 1.0, 0.0, 0, None, ptr(mel_start), ptr(mel_len), ptr(mel_off),
                        ptr(mel_w), mel_w.numel(), n_mels, 1, multiplier, db_offset, amin, ptr(out),
                        ptr(slot_max), stream_of(x))
    check(rc, "sbk_spectrum(fbank)")
    return out, slot_max


@fbank_deferred.register_fake
def _(x, window, tw_nc, tw_nfft, mel_start, mel_len, mel_off, mel_w, n_fft, hop, center, pad_mode, n_mels,
      multiplier, db_offset, amin):
    B = x.shape[0]
    T = n_frames(x.shape[1], n_fft, hop, center)
    nslot = _lib.lib().sbk_spectrum_slots(n_fft, hop, T, n_mels, mel_w.numel())
    return x.new_empty(B, T, n_mels), x.new_empty(B, max(nslot, 1))


@custom_op("sbk::topdb_clamp", mutates_args=())
def topdb_clamp(x: torch.Tensor, slot_max: torch.Tensor, top_db: float) -> torch.Tensor:
    """max(x, max_b - top_db) per sequence b of fbank_deferred's output
    (features.py:706-711), into a new tensor."""
    require_device(x, slot_max)
    y = _c(x.to(_f32)).clone()
    B = y.shape[0]
    check(_lib.lib().sbk_topdb_clamp(ptr(y), ptr(slot_max), slot_max.shape[1], y.numel() // B, B, float(top_db),
                                     stream_of(y)), "sbk_topdb_clamp")
    return y


@topdb_clamp.register_fake
def _(x, slot_max, top_db):
    return torch.empty_like(x, dtype=_f32)


@custom_op("sbk::filterbank", mutates_args=())
def filterbank(spec: torch.Tensor, mel_start: torch.Tensor, mel_len: torch.Tensor, mel_off: torch.Tensor,
               mel_w: torch.Tensor, n_mels: int, log_mel: bool, multiplier: float, db_offset: float,
               amin: float, top_db: float) -> torch.Tensor:
    """Filterbank.forward on a (N,T,F) spectrogram (features.py:490-560)."""
    require_device(spec, mel_start, mel_len, mel_off, mel_w)
    spec = _c(spec.to(_f32))
    N, T, Fd = spec.shape
    out = torch.empty(N, T, n_mels, device=spec.device, dtype=_f32)
    L = _lib.lib()
    nslot = L.sbk_filterbank_slots(T, Fd)
    slot_max = torch.empty(N, max(nslot, 1), device=spec.device, dtype=_f32)
    s = stream_of(spec)
    rc = L.sbk_filterbank(ptr(spec), N, T, Fd, ptr(mel_start), ptr(mel_len), ptr(mel_off), ptr(mel_w), None,
                          n_mels, int(log_mel), multiplier, db_offset, amin, ptr(out), ptr(slot_max), s)
    check(rc, "sbk_filterbank")
    if log_mel:
        check(L.sbk_topdb_clamp(ptr(out), ptr(slot_max), nslot, T * n_mels, N, top_db, s), "sbk_topdb_clamp")
    return out


@filterbank.register_fake
def _(spec, mel_start, mel_len, mel_off, mel_w, n_mels, log_mel, multiplier, db_offset, amin, top_db):
    return spec.new_empty(spec.shape[0], spec.shape[1], n_mels)


@custom_op("sbk::filterbank_dense", mutates_args=())
def filterbank_dense(spec: torch.Tensor, mat: torch.Tensor, log_mel: bool, multiplier: float,
                     db_offset: float, amin: float, top_db: float) -> torch.Tensor:
    """Filterbank with a dense (F, M) matrix (learnable filters, freeze=False)."""
    require_device(spec, mat)
    spec = _c(spec.to(_f32))
    mat = _c(mat.to(_f32))
    N, T, Fd = spec.shape
    M = mat.shape[1]
    out = torch.empty(N, T, M, device=spec.device, dtype=_f32)
    L = _lib.lib()
    nslot = L.sbk_filterbank_slots(T, Fd)
    slot_max = torch.empty(N, max(nslot, 1), device=spec.device, dtype=_f32)
    s = stream_of(spec)
    rc = L.sbk_filterbank(ptr(spec), N, T, Fd, None, None, None, None, ptr(mat), M, int(log_mel), multiplier,
                          db_offset, amin, ptr(out), ptr(slot_max), s)
    check(rc, "sbk_filterbank(dense)")
    if log_mel:
        check(L.sbk_topdb_clamp(ptr(out), ptr(slot_max), nslot, T * M, N, top_db, s), "sbk_topdb_clamp")
    return out


@filterbank_dense.register_fake
def _(spec, mat, log_mel, multiplier, db_offset, amin, top_db):
    return spec.new_empty(spec.shape[0], spec.shape[1], mat.shape[1])


@custom_op("sbk::magnitude", mutates_args=())
def magnitude(x: torch.Tensor, power: float, eps: float, log_mag: bool) -> torch.Tensor:
    """spectral_magnitude: reduce the last axis by sum of squares (features.py:347-356)."""
    require_device(x)
    x = _c(x.to(_f32))
    L = x.shape[-1]
    out = torch.empty(x.shape[:-1], device=x.device, dtype=_f32)
    n = out.numel()
    check(_lib.lib().sbk_magnitude(ptr(x), ptr(out), n, L, float(power), float(eps), int(log_mag),
                                   stream_of(x)), "sbk_magnitude")
    return out


@magnitude.register_fake
def _(x, power, eps, log_mag):
    return x.new_empty(x.shape[:-1])


@custom_op("sbk::dct", mutates_args=())
def dct(x: torch.Tensor, mat: torch.Tensor) -> torch.Tensor:
    """x (..., n_in) @ mat (n_in, n_out) (features.py:765-786)."""
    require_device(x, mat)
    x = _c(x.to(_f32))
    mat = _c(mat.to(_f32))
    n_in, n_out = mat.shape
    out = torch.empty(*x.shape[:-1], n_out, device=x.device, dtype=_f32)
    rows = x.numel() // n_in
    check(_lib.lib().sbk_dct(ptr(x), ptr(mat), ptr(out), rows, n_in, n_out, stream_of(x)), "sbk_dct")
    return out


@dct.register_fake
def _(x, mat):
    return x.new_empty(*x.shape[:-1], mat.shape[1])


@custom_op("sbk::deltas", mutates_args=())
def deltas(x: torch.Tensor, window_length: int, concat: bool) -> torch.Tensor:
    """Deltas along dim 1 of (N,T,F) (features.py:829-852); concat=True
    returns [x | Δx | ΔΔx] in one pass (lobes/features.py:141-144)."""
    require_device(x)
    x = _c(x.to(_f32))
    N, T, Fd = x.shape
    out = torch.empty(N, T, 3 * Fd if concat else Fd, device=x.device, dtype=_f32)
    check(_lib.lib().sbk_deltas(ptr(x), ptr(out), N, T, Fd, window_length, int(concat), stream_of(x)),
          "sbk_deltas")
    return out


@deltas.register_fake
def _(x, window_length, concat):
    return x.new_empty(x.shape[0], x.shape[1], 3 * x.shape[2] if concat else x.shape[2])


@custom_op("sbk::deltas_floor", mutates_args=())
def deltas_floor(x: torch.Tensor, window_length: int, slot_max: torch.Tensor, top_db: float) -> torch.Tensor:
    """[max(x, max_b - top_db) | Δ | ΔΔ] of fbank_deferred's output: the
    top_db floor (features.py:706-711) applied as the concat deltas kernel
    loads its rows (lobes/features.py:141-144), no clamp pass."""
    require_device(x, slot_max)
    x = _c(x.to(_f32))
    N, T, Fd = x.shape
    out = torch.empty(N, T, 3 * Fd, device=x.device, dtype=_f32)
    check(_lib.lib().sbk_deltas_floor(ptr(x), ptr(out), N, T, Fd, window_length, ptr(slot_max), slot_max.shape[1],
                                      float(top_db), stream_of(x)), "sbk_deltas_floor")
    return out


@deltas_floor.register_fake
def _(x, window_length, slot_max, top_db):
    return x.new_empty(x.shape[0], x.shape[1], 3 * x.shape[2])


@custom_op("sbk::context_window", mutates_args=())
def context_window(x: torch.Tensor, left: int, right: int) -> torch.Tensor:
    """ContextWindow on (N,T,F) → (N,T,F·(l+r+1)) (features.py:917-937)."""
    require_device(x)
    x = _c(x.to(_f32))
    N, T, Fd = x.shape
    out = torch.empty(N, T, Fd * (left + right + 1), device=x.device, dtype=_f32)
    check(_lib.lib().sbk_context_window(ptr(x), ptr(out), N, T, Fd, left, right, stream_of(x)),
          "sbk_context_window")
    return out


@context_window.register_fake
def _(x, left, right):
    return x.new_empty(x.shape[0], x.shape[1], x.shape[2] * (left + right + 1))


# ---------------------------------------------------------------------------
# autograd for the learnable-filter path (Filterbank(freeze=False),
# Fbank/MFCC(requires_grad=True); features.py:476-482): the reference gets
# these gradients from torch autograd; here they are HIP kernels too
# ---------------------------------------------------------------------------

@custom_op("sbk::filterbank_dense_bwd", mutates_args=())
def filterbank_dense_bwd(grad: torch.Tensor, spec: torch.Tensor, mat: torch.Tensor, log_mel: bool,
                         multiplier: float, db_offset: float, amin: float,
                         top_db: float) -> tuple[torch.Tensor, torch.Tensor]:
    """(dL/dspec, dL/dmat) of filterbank_dense: the linear energies are
    recomputed by the forward's own kernel (bit-identical dB values for the
    top_db tie rule), sbk_filterbank_db_bwd differentiates dB + top_db,
    dspec = dx·matᵀ runs on the dense filterbank kernel with matᵀ, and dmat
    is a chunked specᵀ·dx reduced by sbk_colsum (deterministic)."""
    require_device(grad, spec, mat)
    spec = _c(spec.to(_f32))
    mat = _c(mat.to(_f32))
    grad = _c(grad.to(_f32))
    N, T, Fd = spec.shape
    M = mat.shape[1]
    L = _lib.lib()
    s = stream_of(spec)
    x = torch.empty(N, T, M, device=spec.device, dtype=_f32)
    check(L.sbk_filterbank(ptr(spec), N, T, Fd, None, None, None, None, ptr(mat), M, 0, multiplier, db_offset, amin,
                           ptr(x), None, s), "sbk_filterbank(recompute)")
    dx = torch.empty_like(x)
    stats = torch.empty(3 * N, device=spec.device, dtype=_f32)
    check(L.sbk_filterbank_db_bwd(ptr(x), ptr(grad), N, T * M, int(log_mel), multiplier, db_offset, amin, top_db,
                                  ptr(stats), ptr(dx), s), "sbk_filterbank_db_bwd")
    matT = mat.t().contiguous()
    dspec = torch.empty(N, T, Fd, device=spec.device, dtype=_f32)
    check(L.sbk_filterbank(ptr(dx), N, T, M, None, None, None, None, ptr(matT), Fd, 0, 1.0, 0.0, 0.0, ptr(dspec),
                           None, s), "sbk_filterbank(dx·matT)")
    rows = N * T
    chunk = 256
    nch = (rows + chunk - 1) // chunk
    part = torch.empty(nch, Fd * M, device=spec.device, dtype=_f32)
    check(L.sbk_filterbank_wgrad(ptr(spec), ptr(dx), rows, Fd, M, chunk, ptr(part), s), "sbk_filterbank_wgrad")
    dmat = torch.empty(Fd, M, device=spec.device, dtype=_f32)
    check(L.sbk_colsum(ptr(part), nch, Fd * M, ptr(dmat), 0, s), "sbk_colsum")
    return dspec, dmat


@filterbank_dense_bwd.register_fake
def _(grad, spec, mat, log_mel, multiplier, db_offset, amin, top_db):
    return spec.new_empty(spec.shape), mat.new_empty(mat.shape)


def _fbd_setup(ctx, inputs, output):
    spec, mat, log_mel, mult, off, amin, top_db = inputs
    ctx.save_for_backward(spec, mat)
    ctx.args = (log_mel, mult, off, amin, top_db)


def _fbd_backward(ctx, grad):
    spec, mat = ctx.saved_tensors
    dspec, dmat = filterbank_dense_bwd(grad, spec, mat, *ctx.args)
    return (dspec if ctx.needs_input_grad[0] else None, dmat if ctx.needs_input_grad[1] else None,
            None, None, None, None, None)


filterbank_dense.register_autograd(_fbd_backward, setup_context=_fbd_setup)


def _dct_setup(ctx, inputs, output):
    ctx.save_for_backward(inputs[1])


def _dct_backward(ctx, grad):
    """y = x·D is linear: dx = g·Dᵀ on the same kernel (the DCT matrix is a
    fixed buffer in the reference, so it gets no gradient)."""
    (mat,) = ctx.saved_tensors
    return dct(grad, mat.t().contiguous()), None


dct.register_autograd(_dct_backward, setup_context=_dct_setup)
