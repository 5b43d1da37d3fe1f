"""Drop-in for speechbrain.processing.features (STFT, spectral_magnitude,
Filterbank, DCT, Deltas, ContextWindow) on HIP kernels.

Constructor arguments, attributes, buffers (state_dict keys) and forward
signatures follow the reference (speechbrain/processing/features.py:50-937);
the arithmetic runs in libsbk.so (speechbrain_amd/csrc/features.hip).
"""
import logging
import math

import torch

from .. import ops
from .._lib import check as _check, lib as _lib, ptr as _ptr, require_device as _require_device, stream_of as _stream_of

logger = logging.getLogger(__name__)

__all__ = ["STFT", "spectral_magnitude", "Filterbank", "DCT", "Deltas", "ContextWindow", "InputNormalization"]


class _DevCache:
    """Per-device cache of small constant tables (window, twiddles, mel CSR)."""

    def __init__(self):
        self._d = {}

    def get(self, key, device, make):
        k = (key, str(device))
        v = self._d.get(k)
        if v is None:
            v = make()
            v = tuple(t.to(device) for t in v) if isinstance(v, tuple) else v.to(device)
            self._d[k] = v
        return v


def fft_twiddles(n_fft):
    """(W_{n_fft/2}^m for m < n_fft/2, W_{n_fft}^k for k <= n_fft/2) as float32
    (re, im) pairs, computed in float64 on the host."""
    nc = n_fft // 2
    m = torch.arange(nc, dtype=torch.float64)
    a = -2.0 * math.pi * m / nc
    tw1 = torch.stack([torch.cos(a), torch.sin(a)], -1).to(torch.float32).contiguous()
    k = torch.arange(nc + 1, dtype=torch.float64)
    b = -2.0 * math.pi * k / n_fft
    tw2 = torch.stack([torch.cos(b), torch.sin(b)], -1).to(torch.float32).contiguous()
    return tw1, tw2


class STFT(torch.nn.Module):
    """Short-Term Fourier Transform (features.py:50-188): a mixed-radix LDS
    FFT kernel; (B,S)→(B,T,F,2), (B,S,C)→(B,T,F,2,C)."""

    def __init__(self, sample_rate, win_length=25, hop_length=10, n_fft=400,
                 window_fn=torch.hamming_window, normalized_stft=False, center=True,
                 pad_mode="constant", onesided=True):
        super().__init__()
        self.sample_rate = sample_rate
        self.win_length = win_length
        self.hop_length = hop_length
        self.n_fft = n_fft
        self.normalized_stft = normalized_stft
        self.center = center
        self.pad_mode = pad_mode
        self.onesided = onesided
        self.win_length = int(round((self.sample_rate / 1000.0) * self.win_length))
        self.hop_length = int(round((self.sample_rate / 1000.0) * self.hop_length))
        self.window = window_fn(self.win_length)
        if pad_mode not in ops.PAD_MODES:
            raise ValueError(f"unsupported pad_mode {pad_mode}")
        self._cache = _DevCache()

    def _tables(self, device):
        def make():
            w = torch.zeros(self.n_fft, dtype=torch.float32)
            left = (self.n_fft - self.win_length) // 2
            w[left:left + self.win_length] = self.window.to(torch.float32)
            tw1, tw2 = fft_twiddles(self.n_fft)
            return (w, tw1, tw2)
        return self._cache.get("stft", device, make)

    def forward(self, x):
        """Returns the STFT of a batch of waveforms (features.py:133-188)."""
        w, tw1, tw2 = self._tables(x.device)
        return ops.stft(x, w, tw1, tw2, self.n_fft, self.hop_length, self.center,
                        ops.PAD_MODES[self.pad_mode], self.onesided, self.normalized_stft)

    def power_spectrum(self, x, power=1, eps=1e-14, log=False):
        """Fused STFT → spectral_magnitude for mono input (one kernel)."""
        w, tw1, tw2 = self._tables(x.device)
        return ops.power_spectrum(x, w, tw1, tw2, self.n_fft, self.hop_length, self.center,
                                  ops.PAD_MODES[self.pad_mode], self.normalized_stft,
                                  float(power), float(eps), bool(log))


def spectral_magnitude(stft, power=1, log=False, eps=1e-14):
    """features.py:327-356: sum of squares over the last axis, ^power, log."""
    return ops.magnitude(stft, float(power), float(eps), bool(log))


def _mel_csr(mat):
    """(F, M) dense filter matrix → per-filter contiguous nonzero runs."""
    Fd, M = mat.shape
    starts, lens, offs, ws = [], [], [], []
    off = 0
    for j in range(M):
        nz = torch.nonzero(mat[:, j] != 0).flatten()
        if nz.numel() == 0:
            s, L = 0, 0
        else:
            s, e = int(nz[0]), int(nz[-1]) + 1
            L = e - s
            ws.append(mat[s:e, j])
        starts.append(s)
        lens.append(L)
        offs.append(off)
        off += L
    w = torch.cat(ws) if ws else torch.zeros(1)
    i32 = torch.int32
    return (torch.tensor(starts, dtype=i32), torch.tensor(lens, dtype=i32),
            torch.tensor(offs, dtype=i32), w.to(torch.float32).contiguous())


class Filterbank(torch.nn.Module):
    """Mel filterbank + dB (features.py:359-712).  Frozen filters use a
    per-filter sparse (CSR) table; learnable filters (freeze=False) a dense
    matrix kernel."""

    def __init__(self, n_mels=40, log_mel=True, filter_shape="triangular", f_min=0, f_max=8000,
                 n_fft=400, sample_rate=16000, power_spectrogram=2, amin=1e-10, ref_value=1.0,
                 top_db=80.0, param_change_factor=1.0, param_rand_factor=0.0, freeze=True):
        super().__init__()
        self.n_mels = n_mels
        self.log_mel = log_mel
        self.filter_shape = filter_shape
        self.f_min = f_min
        self.f_max = f_max
        self.n_fft = n_fft
        self.sample_rate = sample_rate
        self.power_spectrogram = power_spectrogram
        self.amin = amin
        self.ref_value = ref_value
        self.top_db = top_db
        self.freeze = freeze
        self.n_stft = self.n_fft // 2 + 1
        self.db_multiplier = math.log10(max(self.amin, self.ref_value))
        self.device_inp = torch.device("cpu")
        self.param_change_factor = param_change_factor
        self.param_rand_factor = param_rand_factor
        self.multiplier = 10 if self.power_spectrogram == 2 else 20
        if self.f_min >= self.f_max:
            logger.error("Require f_min: %f < f_max: %f" % (self.f_min, self.f_max), exc_info=True)
        mel = torch.linspace(self._to_mel(self.f_min), self._to_mel(self.f_max), self.n_mels + 2)
        hz = self._to_hz(mel)
        band = hz[1:] - hz[:-1]
        self.band = band[:-1]
        self.f_central = hz[1:-1]
        if not self.freeze:
            self.f_central = torch.nn.Parameter(self.f_central / (self.sample_rate * self.param_change_factor))
            self.band = torch.nn.Parameter(self.band / (self.sample_rate * self.param_change_factor))
        all_freqs = torch.linspace(0, self.sample_rate // 2, self.n_stft)
        self.all_freqs_mat = all_freqs.repeat(self.f_central.shape[0], 1)
        self._cache = _DevCache()

    @staticmethod
    def _to_mel(hz):
        return 2595 * math.log10(1 + hz / 700)

    @staticmethod
    def _to_hz(mel):
        return 700 * (10 ** (mel / 2595) - 1)

    def _matrix(self, f_central, band):
        """(n_stft, n_mels) filter matrix (features.py:586-689)."""
        f = self.all_freqs_mat.to(f_central.device)
        fc = f_central.unsqueeze(1)
        bd = band.unsqueeze(1)
        if self.filter_shape == "triangular":
            slope = (f - fc) / bd
            # torch.max against a zero tensor (not clamp): at a filter edge
            # slope = ±1 exactly (the first filter at 0 Hz) the reference's
            # maximum splits the gradient in half, clamp would pass it whole
            zero = torch.zeros(1, device=f.device)
            m = torch.max(zero, torch.min(slope + 1.0, -slope + 1.0))
        elif self.filter_shape == "rectangular":
            m = ((f >= fc - bd) & (f <= fc + bd)).float()
        else:
            m = torch.exp(-0.5 * ((f - fc) / (bd / 2)) ** 2)
        return m.transpose(0, 1)

    def _params(self):
        fc, bd = self.f_central, self.band
        if not self.freeze:
            s = self.sample_rate * self.param_change_factor * self.param_change_factor
            return fc * s, bd * s, True
        if self.param_rand_factor != 0 and self.training:
            rc = 1.0 + torch.rand(2) * 2 * self.param_rand_factor - self.param_rand_factor
            return fc * rc[0], bd * rc[1], True
        return fc, bd, False

    def csr_tables(self, device):
        fc, bd, dynamic = self._params()
        if dynamic:
            return tuple(t.to(device) for t in _mel_csr(self._matrix(fc.detach().cpu(), bd.detach().cpu())))
        return self._cache.get("mel", device, lambda: _mel_csr(self._matrix(fc, bd)))

    def _db_args(self):
        return (bool(self.log_mel), float(self.multiplier), float(self.multiplier * self.db_multiplier),
                float(self.amin), float(self.top_db))

    def forward(self, spectrogram):
        """Returns the FBANKs of (B,T,F) or (B,T,F,C) spectrograms."""
        sp_shape = spectrogram.shape
        if len(sp_shape) == 4:
            spectrogram = spectrogram.permute(0, 3, 1, 2).reshape(
                sp_shape[0] * sp_shape[3], sp_shape[1], sp_shape[2])
        log_mel, mult, off, amin, top_db = self._db_args()
        if not self.freeze:
            fc, bd, _ = self._params()
            mat = self._matrix(fc, bd)
            fb = ops.filterbank_dense(spectrogram, mat.to(spectrogram.device), log_mel, mult, off, amin, top_db)
        else:
            st, ln, of, w = self.csr_tables(spectrogram.device)
            fb = ops.filterbank(spectrogram, st, ln, of, w, self.n_mels, log_mel, mult, off, amin, top_db)
        if len(sp_shape) == 4:
            fb = fb.reshape(sp_shape[0], sp_shape[3], fb.shape[1], fb.shape[2]).permute(0, 2, 3, 1)
        return fb


class DCT(torch.nn.Module):
    """Discrete cosine transform (features.py:715-786)."""

    def __init__(self, input_size, n_out=20, ortho_norm=True):
        super().__init__()
        if n_out > input_size:
            raise ValueError("Cannot select more DCT coefficients than inputs "
                             "(n_out=%i, n_in=%i)" % (n_out, input_size))
        n = torch.arange(float(input_size))
        k = torch.arange(float(n_out)).unsqueeze(1)
        dct = torch.cos(math.pi / float(input_size) * (n + 0.5) * k)
        if ortho_norm:
            dct[0] *= 1.0 / math.sqrt(2.0)
            dct *= math.sqrt(2.0 / float(input_size))
        else:
            dct *= 2.0
        self.dct_mat = dct.t()
        self._cache = _DevCache()

    def forward(self, x):
        input_shape = x.shape
        if len(input_shape) == 4:
            x = x.reshape(x.shape[0] * x.shape[3], x.shape[1], x.shape[2])
        mat = self._cache.get("dct", x.device, lambda: self.dct_mat.contiguous())
        y = ops.dct(x, mat)
        if len(input_shape) == 4:
            y = y.reshape(input_shape[0], y.shape[1], y.shape[2], input_shape[3])
        return y


class Deltas(torch.nn.Module):
    """Time derivatives (features.py:789-852) as a one-pass stencil kernel."""

    def __init__(self, input_size, window_length=5):
        super().__init__()
        self.n = (window_length - 1) // 2
        self.denom = self.n * (self.n + 1) * (2 * self.n + 1) / 3
        self.window_length = window_length
        self.register_buffer(
            "kernel", torch.arange(-self.n, self.n + 1, dtype=torch.float32).repeat(input_size, 1, 1))

    def forward(self, x):
        if x.dim() == 4:
            # the reference's per-(freq, channel) time derivative (features.py:829-850)
            B, T, Fd, C = x.shape
            y = ops.deltas(x.reshape(B, T, Fd * C), 2 * self.n + 1, False)
            return y.reshape(B, T, Fd, C)
        return ops.deltas(x, 2 * self.n + 1, False)


class ContextWindow(torch.nn.Module):
    """Context stacking (features.py:855-937) as a gather kernel."""

    def __init__(self, left_frames=0, right_frames=0):
        super().__init__()
        self.left_frames = left_frames
        self.right_frames = right_frames
        self.context_len = self.left_frames + self.right_frames + 1
        self.kernel_len = 2 * max(self.left_frames, self.right_frames) + 1
        self.kernel = torch.eye(self.context_len, self.kernel_len)
        if self.right_frames > self.left_frames:
            lag = self.right_frames - self.left_frames
            self.kernel = torch.roll(self.kernel, lag, 1)
        self.first_call = True

    def forward(self, x):
        if x.dim() == 4:
            # reference: conv1d over the LAST axis of (B*T, F, C) (features.py:917-935)
            B, Tn, Fd, C = x.shape
            xr = x.transpose(1, 2).reshape(B * Tn, Fd, C)  # same regroup as the reference
            y = ops.context_window(xr.transpose(1, 2).contiguous(), self.left_frames, self.right_frames)
            y = y.transpose(1, 2).reshape(B, Fd * self.context_len, Tn, C)
            return y.transpose(1, 2)
        return ops.context_window(x, self.left_frames, self.right_frames)


class InputNormalization(torch.nn.Module):
    """Mean / variance normalisation (features.py:940-1231) on HIP
    (csrc/norm.hip): the per-utterance statistics of the whole batch in two
    launches (fp64 Welford slices, then the merge — no per-utterance host
    loop and no host sync), the normalisation in a third.  norm_type
    "sentence" | "batch" | "global" | "speaker" with the reference's moving
    averages; sentence and speaker modes write into x and return it, batch and
    global return a new tensor, as the reference does.  The statistics state
    (count, glob_mean, glob_std, spk_dict_*) round-trips through
    _statistics_dict / _load_statistics_dict / _save / _load."""

    def __init__(self, mean_norm=True, std_norm=True, norm_type="global", avg_factor=None, requires_grad=False,
                 update_until_epoch=3):
        super().__init__()
        self.mean_norm = mean_norm
        self.std_norm = std_norm
        self.norm_type = norm_type
        self.avg_factor = avg_factor
        self.requires_grad = requires_grad
        self.glob_mean = torch.tensor([0])
        self.glob_std = torch.tensor([0])
        self.spk_dict_mean = {}
        self.spk_dict_std = {}
        self.spk_dict_count = {}
        self.weight = 1.0
        self.count = 0
        self.eps = 1e-10
        self.update_until_epoch = update_until_epoch

    def _batch_stats(self, x, lengths, glob_update=None):
        """Per-utterance (B, F) mean / std, and for batch / global also the
        batch means (F,) with the global moving average applied in place."""
        _require_device(x)
        B, T = x.shape[0], x.shape[1]
        F = x[0, 0].numel()
        lib = _lib()
        lens = lengths.to(device=x.device, dtype=torch.float32).contiguous()
        part = torch.empty(B * int(lib.sbk_inorm_slices(T)) * F * 3, device=x.device, dtype=torch.float64)
        s = _stream_of(x)
        _check(lib.sbk_inorm_partials(_ptr(x), _ptr(lens), B, T, F, _ptr(part), s), "sbk_inorm_partials")
        mean = torch.empty(B, F, device=x.device, dtype=torch.float32)
        std = torch.empty(B, F, device=x.device, dtype=torch.float32)
        cur = None
        upd, keep, w, gm, gs = 0, 0.0, 0.0, None, None
        if self.norm_type in ("batch", "global"):
            cur = (torch.empty(F, device=x.device, dtype=torch.float32),
                   torch.empty(F, device=x.device, dtype=torch.float32))
            if glob_update is not None:
                upd, w = glob_update
                keep = 1.0 - w
                if upd == 1:
                    gm = torch.empty(F, device=x.device, dtype=torch.float32)
                    gs = torch.empty(F, device=x.device, dtype=torch.float32)
                else:  # blended in place; a (1,) state (mean_norm / std_norm off) is widened first
                    gm = self.glob_mean.to(device=x.device, dtype=torch.float32).expand(F).contiguous()
                    gs = self.glob_std.to(device=x.device, dtype=torch.float32).expand(F).contiguous()
        _check(lib.sbk_inorm_stats(_ptr(part), B, T, F, int(self.mean_norm), int(self.std_norm),
                                      float(self.eps), _ptr(mean), _ptr(std),
                                      _ptr(cur[0] if cur else None), _ptr(cur[1] if cur else None), upd,
                                      float(keep), float(w), _ptr(gm), _ptr(gs), s), "sbk_inorm_stats")
        if upd:
            # the reference's statistics are (1,) tensors when that normalisation is off
            self.glob_mean = gm if self.mean_norm else gm[:1].clone()
            self.glob_std = gs if self.std_norm else gs[:1].clone()
        return mean, std, cur

    def _normalize(self, x, mean, std, per_utt, out):
        B, T = x.shape[0], x.shape[1]
        F = x[0, 0].numel()
        _check(_lib().sbk_inorm_apply(_ptr(x), B, T, F, _ptr(mean), _ptr(std), int(per_utt),
                                            _ptr(out), _stream_of(x)), "sbk_inorm_apply")
        return out

    def forward(self, x, lengths, spk_ids=torch.tensor([]), epoch=0):
        if x.dtype != torch.float32 or not x.is_contiguous():
            raise TypeError("InputNormalization kernels take contiguous fp32 features")
        glob_update = None
        if self.norm_type == "global" and self.training:
            if self.count == 0:
                glob_update = (1, 1.0)
            elif epoch < self.update_until_epoch:
                self.weight = 1 / (self.count + 1) if self.avg_factor is None else self.avg_factor
                glob_update = (2, float(self.weight))
        mean, std, cur = self._batch_stats(x, lengths, glob_update)
        if self.norm_type == "sentence":
            return self._normalize(x, mean, std, True, x)
        if self.norm_type == "speaker":
            sm, ss = [], []
            for b in range(x.shape[0]):
                k = int(spk_ids[b][0])
                m, s = mean[b], std[b]
                if self.training:
                    if k not in self.spk_dict_mean:
                        self.spk_dict_mean[k], self.spk_dict_std[k], self.spk_dict_count[k] = m, s, 1
                    else:
                        self.spk_dict_count[k] += 1
                        self.weight = 1 / self.spk_dict_count[k] if self.avg_factor is None else self.avg_factor
                        self.spk_dict_mean[k] = (1 - self.weight) * self.spk_dict_mean[k] + self.weight * m
                        self.spk_dict_std[k] = (1 - self.weight) * self.spk_dict_std[k] + self.weight * s
                    sm.append(self.spk_dict_mean[k])
                    ss.append(self.spk_dict_std[k])
                else:
                    sm.append(self.spk_dict_mean.get(k, m))
                    ss.append(self.spk_dict_std.get(k, s))
            return self._normalize(x, torch.stack(sm).contiguous(), torch.stack(ss).contiguous(), True, x)
        if self.norm_type == "batch":
            return self._normalize(x, cur[0], cur[1], False, torch.empty_like(x))
        if self.norm_type == "global":
            if self.training:
                self.count = self.count + 1
            gm = self.glob_mean.to(device=x.device, dtype=torch.float32).expand(mean.shape[1]).contiguous()
            gs = self.glob_std.to(device=x.device, dtype=torch.float32).expand(mean.shape[1]).contiguous()
            return self._normalize(x, gm, gs, False, torch.empty_like(x))
        return x

    # statistics state (features.py:1147-1231)
    def _statistics_dict(self):
        return {"count": self.count, "glob_mean": self.glob_mean, "glob_std": self.glob_std,
                "spk_dict_mean": self.spk_dict_mean, "spk_dict_std": self.spk_dict_std,
                "spk_dict_count": self.spk_dict_count}

    def _load_statistics_dict(self, state):
        self.count = state["count"]
        self.glob_mean = state["glob_mean"]
        self.glob_std = state["glob_std"]
        self.spk_dict_mean = dict(state["spk_dict_mean"])
        self.spk_dict_std = dict(state["spk_dict_std"])
        self.spk_dict_count = dict(state["spk_dict_count"])
        return state

    def to(self, device):
        self = super().to(device)
        if isinstance(self.glob_mean, torch.Tensor):
            self.glob_mean = self.glob_mean.to(device)
            self.glob_std = self.glob_std.to(device)
        for k in self.spk_dict_mean:
            self.spk_dict_mean[k] = self.spk_dict_mean[k].to(device)
            self.spk_dict_std[k] = self.spk_dict_std[k].to(device)
        return self

    def _save(self, path):
        torch.save(self._statistics_dict(), path)

    def _load(self, path, end_of_epoch=False, device=None):
        del end_of_epoch
        self._load_statistics_dict(torch.load(path, map_location=device, weights_only=True))

