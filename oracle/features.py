"""CPU restatement of the SpeechBrain feature front-end (test infrastructure).

Restates speechbrain/processing/features.py (STFT, spectral_magnitude,
Filterbank, DCT, Deltas, ContextWindow) and speechbrain/lobes/features.py
(Fbank, MFCC) as plain functions over CPU tensors.  See oracle/__init__.py
for who may import this module.
"""
import math

import torch

__all__ = [
    "ms_to_samples", "hamming_periodic", "stft", "spectral_magnitude",
    "mel_filter_params", "fbank_matrix", "amplitude_to_db", "filterbank",
    "dct_matrix", "dct", "deltas", "context_window", "fbank", "mfcc",
]


def ms_to_samples(sample_rate, ms):
    """features.py:124-129 — int(round(sr/1000 * ms))."""
    return int(round((sample_rate / 1000.0) * ms))


def hamming_periodic(n, dtype=torch.float32):
    """torch.hamming_window(n) default (periodic): 0.54 - 0.46 cos(2πk/n).

    features.py:131 uses `window_fn(self.win_length)` with
    window_fn=torch.hamming_window."""
    k = torch.arange(n, dtype=torch.float64)
    return (0.54 - 0.46 * torch.cos(2.0 * math.pi * k / n)).to(dtype)


def stft(x, sample_rate=16000, win_length=25, hop_length=10, n_fft=400,
         normalized=False, center=True, pad_mode="constant", onesided=True,
         compute_dtype=torch.float32):
    """features.py:133-188 (STFT.forward) with torch.stft semantics.

    Frames of n_fft samples every `hop` samples (after n_fft//2 padding on
    both sides when center=True), the win-sample window zero-padded to n_fft
    and centred, real DFT, output (B, T, F, 2) or (B, T, F, 2, C) for a
    (B, S, C) input (features.py:143-146, :175-183)."""
    win = ms_to_samples(sample_rate, win_length)
    hop = ms_to_samples(sample_rate, hop_length)
    or_shape = x.shape
    if x.dim() == 3:
        x = x.transpose(1, 2).reshape(or_shape[0] * or_shape[2], or_shape[1])
    x = x.to(compute_dtype)
    if center:
        p = n_fft // 2
        mode = {"constant": "constant", "reflect": "reflect",
                "replicate": "replicate", "circular": "circular"}[pad_mode]
        x = torch.nn.functional.pad(x[:, None, :], (p, p), mode=mode)[:, 0]
    w = torch.zeros(n_fft, dtype=compute_dtype)
    left = (n_fft - win) // 2
    w[left:left + win] = hamming_periodic(win, compute_dtype)
    frames = x.unfold(-1, n_fft, hop) * w  # (N, T, n_fft)
    spec = torch.fft.rfft(frames, dim=-1) if onesided else torch.fft.fft(frames, dim=-1)
    if normalized:
        spec = spec * (n_fft ** -0.5)
    out = torch.view_as_real(spec).to(torch.float32)  # (N, T, F, 2)
    if len(or_shape) == 3:
        out = out.reshape(or_shape[0], or_shape[2], *out.shape[1:])
        out = out.permute(0, 2, 3, 4, 1)  # (B, T, F, 2, C)
    return out


def spectral_magnitude(stft_out, power=1, log=False, eps=1e-14):
    """features.py:327-356: sum of squares over the LAST axis, eps when
    power < 1, ^power, optional log(x + eps)."""
    s = stft_out.pow(2).sum(-1)
    if power < 1:
        s = s + eps
    s = s.pow(power)
    if log:
        return torch.log(s + eps)
    return s


def _to_mel(hz):
    return 2595 * math.log10(1 + hz / 700)  # features.py:562-572


def mel_filter_params(n_mels=40, f_min=0, f_max=8000):
    """features.py:464-474: fp32 linspace on the mel axis, back to Hz,
    central frequencies and bands of the n_mels filters."""
    mel = torch.linspace(_to_mel(f_min), _to_mel(f_max), n_mels + 2)
    hz = 700 * (10 ** (mel / 2595) - 1)  # features.py:574-584
    band = (hz[1:] - hz[:-1])[:-1]
    f_central = hz[1:-1]
    return f_central, band


def fbank_matrix(f_central, band, n_fft=400, sample_rate=16000,
                 filter_shape="triangular"):
    """(n_stft, n_mels) matrix: features.py:586-689.

    triangular: max(0, min(slope+1, 1-slope)), slope=(f-fc)/band;
    rectangular: 1 on [fc-band, fc+band]; gaussian: exp(-0.5((f-fc)/(band/2))^2).
    """
    n_stft = n_fft // 2 + 1
    all_freqs = torch.linspace(0, sample_rate // 2, n_stft)
    f = all_freqs[None, :]
    fc = f_central[:, None]
    bd = band[:, None]
    if filter_shape == "triangular":
        slope = (f - fc) / bd
        m = torch.clamp(torch.minimum(slope + 1.0, -slope + 1.0), min=0.0)
    elif filter_shape == "rectangular":
        m = ((f >= fc - bd) & (f <= fc + bd)).to(torch.float32)
    else:
        m = torch.exp(-0.5 * ((f - fc) / (bd / 2)) ** 2)
    return m.t().contiguous()


def amplitude_to_db(x, multiplier=10.0, amin=1e-10, ref_value=1.0, top_db=80.0):
    """features.py:691-712: multiplier*log10(clamp(x, amin)) minus the ref
    offset, floored at (per-sequence max over the last two axes) - top_db."""
    db_mult = math.log10(max(amin, ref_value))
    x_db = multiplier * torch.log10(torch.clamp(x, min=amin))
    x_db = x_db - multiplier * db_mult
    floor = x_db.amax(dim=(-2, -1)) - top_db
    return torch.maximum(x_db, floor.view(x_db.shape[0], 1, 1))


def filterbank(spectrogram, n_mels=40, log_mel=True, filter_shape="triangular",
               f_min=0, f_max=8000, n_fft=400, sample_rate=16000,
               power_spectrogram=2, amin=1e-10, ref_value=1.0, top_db=80.0,
               f_central=None, band=None):
    """features.py:490-560 (Filterbank.forward, frozen filters).

    4-D (B, T, F, C) input is folded to (B*C, T, F) and unfolded back
    (features.py:538-558)."""
    if f_central is None:
        f_central, band = mel_filter_params(n_mels, f_min, f_max)
    mat = fbank_matrix(f_central, band, n_fft, sample_rate, filter_shape)
    sp_shape = spectrogram.shape
    if len(sp_shape) == 4:
        spectrogram = spectrogram.permute(0, 3, 1, 2).reshape(
            sp_shape[0] * sp_shape[3], sp_shape[1], sp_shape[2])
    fb = torch.matmul(spectrogram, mat)
    if log_mel:
        mult = 10.0 if power_spectrogram == 2 else 20.0
        fb = amplitude_to_db(fb, mult, amin, ref_value, top_db)
    if len(sp_shape) == 4:
        fb = fb.reshape(sp_shape[0], sp_shape[3], fb.shape[1], fb.shape[2])
        fb = fb.permute(0, 2, 3, 1)
    return fb


def dct_matrix(input_size, n_out=20, ortho_norm=True):
    """features.py:740-763: cos(π/n (n+0.5) k), ortho-normalised; (n_in, n_out)."""
    if n_out > input_size:
        raise ValueError("Cannot select more DCT coefficients than inputs "
                         "(n_out=%i, n_in=%i)" % (n_out, input_size))
    n = torch.arange(float(input_size))
    k = torch.arange(float(n_out)).unsqueeze(1)
    m = torch.cos(math.pi / float(input_size) * (n + 0.5) * k)
    if ortho_norm:
        m[0] *= 1.0 / math.sqrt(2.0)
        m *= math.sqrt(2.0 / float(input_size))
    else:
        m *= 2.0
    return m.t().contiguous()


def dct(x, n_out=20, ortho_norm=True):
    """features.py:765-786 (DCT.forward)."""
    shp = x.shape
    if len(shp) == 4:
        x = x.reshape(shp[0] * shp[3], shp[1], shp[2])
    y = torch.matmul(x, dct_matrix(x.shape[-1], n_out, ortho_norm))
    if len(shp) == 4:
        y = y.reshape(shp[0], y.shape[1], y.shape[2], shp[3])
    return y


def deltas(x, window_length=5):
    """features.py:806-852: δ[t] = Σ_{k=-n..n} k·x[clamp(t+k)] / (n(n+1)(2n+1)/3).

    Works on the time axis (dim 1) of (B, T, F) or (B, T, F, C) input; the
    4-D fold mirrors the reference's transpose/reshape sequence."""
    n = (window_length - 1) // 2
    denom = n * (n + 1) * (2 * n + 1) / 3
    x = x.transpose(1, 2).transpose(2, -1)
    or_shape = x.shape
    if len(or_shape) == 4:
        x = x.reshape(or_shape[0] * or_shape[2], or_shape[1], or_shape[3])
    T = x.shape[-1]
    idx = torch.arange(T)
    acc = torch.zeros_like(x)
    for k in range(-n, n + 1):
        if k == 0:
            continue
        acc = acc + k * x[..., torch.clamp(idx + k, 0, T - 1)]
    d = acc / denom
    if len(or_shape) == 4:
        d = d.reshape(or_shape[0], or_shape[1], or_shape[2], or_shape[3])
    return d.transpose(1, -1).transpose(2, -1)


def context_window(x, left_frames=0, right_frames=0):
    """features.py:879-937 for (B, T, F) input: output feature c*L + k holds
    x[t + k - left] (zero outside), L = left + right + 1."""
    L = left_frames + right_frames + 1
    B, T, Fdim = x.shape
    out = torch.zeros(B, T, Fdim, L, dtype=x.dtype)
    for k in range(L):
        off = k - left_frames
        lo, hi = max(0, -off), min(T, T - off)
        if hi > lo:
            out[:, lo:hi, :, k] = x[:, lo + off:hi + off, :]
    return out.reshape(B, T, Fdim * L)


def fbank(wav, deltas_on=False, context=False, sample_rate=16000, f_min=0,
          f_max=None, n_fft=400, n_mels=40, filter_shape="triangular",
          left_frames=5, right_frames=5, win_length=25, hop_length=10):
    """lobes/features.py:82-147 (Fbank.forward)."""
    if f_max is None:
        f_max = sample_rate / 2
    s = stft(wav, sample_rate, win_length, hop_length, n_fft)
    mag = spectral_magnitude(s)
    fb = filterbank(mag, n_mels=n_mels, filter_shape=filter_shape, f_min=f_min,
                    f_max=f_max, n_fft=n_fft, sample_rate=sample_rate)
    if deltas_on:
        d1 = deltas(fb)
        d2 = deltas(d1)
        fb = torch.cat([fb, d1, d2], dim=2)
    if context:
        fb = context_window(fb, left_frames, right_frames)
    return fb


def mfcc(wav, deltas_on=True, context=True, sample_rate=16000, f_min=0,
         f_max=None, n_fft=400, n_mels=23, n_mfcc=20, filter_shape="triangular",
         left_frames=5, right_frames=5, win_length=25, hop_length=10):
    """lobes/features.py:212-281 (MFCC.forward)."""
    if f_max is None:
        f_max = sample_rate / 2
    s = stft(wav, sample_rate, win_length, hop_length, n_fft)
    mag = spectral_magnitude(s)
    fb = filterbank(mag, n_mels=n_mels, filter_shape=filter_shape, f_min=f_min,
                    f_max=f_max, n_fft=n_fft, sample_rate=sample_rate)
    m = dct(fb, n_mfcc)
    if deltas_on:
        d1 = deltas(m)
        d2 = deltas(d1)
        m = torch.cat([m, d1, d2], dim=2)
    if context:
        m = context_window(m, left_frames, right_frames)
    return m


class InputNormalization:
    """CPU restatement of speechbrain/processing/features.py:940-1231
    (InputNormalization): per-utterance mean / unbiased std over the first
    round(len * T) frames (:1017-1024, :1120-1145), then sentence / batch /
    global / speaker normalisation with the reference's moving averages
    (:1026-1117).  Stateful like the reference (count, glob_*, spk_dict_*)."""

    def __init__(self, mean_norm=True, std_norm=True, norm_type="global", avg_factor=None, update_until_epoch=3):
        self.mean_norm, self.std_norm, self.norm_type = mean_norm, std_norm, norm_type
        self.avg_factor, self.update_until_epoch = avg_factor, update_until_epoch
        self.glob_mean = torch.tensor([0])
        self.glob_std = torch.tensor([0])
        self.spk_mean, self.spk_std, self.spk_count = {}, {}, {}
        self.count = 0
        self.eps = 1e-10
        self.training = True

    def _stats(self, x):
        mean = torch.mean(x, dim=0) if self.mean_norm else torch.tensor([0.0])
        std = torch.std(x, dim=0) if self.std_norm else torch.tensor([1.0])
        return mean, torch.max(std, self.eps * torch.ones_like(std))

    def __call__(self, x, lengths, spk_ids=torch.tensor([]), epoch=0):
        means, stds = [], []
        for b in range(x.shape[0]):
            n = int(torch.round(lengths[b] * x.shape[1]).int())
            m, s = self._stats(x[b, 0:n, ...])
            means.append(m)
            stds.append(s)
            if self.norm_type == "sentence":
                x[b] = (x[b] - m) / s
            if self.norm_type == "speaker":
                k = int(spk_ids[b][0])
                if self.training:
                    if k not in self.spk_mean:
                        self.spk_mean[k], self.spk_std[k], self.spk_count[k] = m, s, 1
                    else:
                        self.spk_count[k] += 1
                        w = 1 / self.spk_count[k] if self.avg_factor is None else self.avg_factor
                        self.spk_mean[k] = (1 - w) * self.spk_mean[k] + w * m
                        self.spk_std[k] = (1 - w) * self.spk_std[k] + w * s
                    sm, ss = self.spk_mean[k], self.spk_std[k]
                else:
                    sm, ss = (self.spk_mean[k], self.spk_std[k]) if k in self.spk_mean else (m, s)
                x[b] = (x[b] - sm) / ss
        if self.norm_type in ("batch", "global"):
            cm = torch.mean(torch.stack(means), dim=0)
            cs = torch.mean(torch.stack(stds), dim=0)
            if self.norm_type == "batch":
                x = (x - cm) / cs
            else:
                if self.training:
                    if self.count == 0:
                        self.glob_mean, self.glob_std = cm, cs
                    elif epoch < self.update_until_epoch:
                        w = 1 / (self.count + 1) if self.avg_factor is None else self.avg_factor
                        self.glob_mean = (1 - w) * self.glob_mean + w * cm
                        self.glob_std = (1 - w) * self.glob_std + w * cs
                    self.count += 1
                x = (x - self.glob_mean) / self.glob_std
        return x
