"""Drop-in for speechbrain.lobes.features (Fbank, MFCC) on HIP kernels.

Fbank on a mono (B,S) waveform with frozen filters is ONE fused kernel
(frame → window → FFT → |X|² → mel → dB, plus per-utterance max) followed by
the top_db clamp; with deltas the [x | Δ | ΔΔ] concat is one stencil kernel
that also applies the top_db floor as it loads (no clamp pass).
Module structure and state_dict keys match speechbrain/lobes/features.py:22-281.
"""
import torch

from .. import ops
from ..processing.features import DCT, STFT, ContextWindow, Deltas, Filterbank, spectral_magnitude

__all__ = ["Fbank", "MFCC"]


def _fused_fbank(stft_mod, fb_mod, wav):
    """STFT+spectral_magnitude+Filterbank in one launch (+ top_db clamp)."""
    w, tw1, tw2 = stft_mod._tables(wav.device)
    st, ln, of, mw = fb_mod.csr_tables(wav.device)
    log_mel, mult, off, amin, top_db = fb_mod._db_args()
    return ops.fbank(wav, w, tw1, tw2, st, ln, of, mw, stft_mod.n_fft, stft_mod.hop_length,
                     stft_mod.center, ops.PAD_MODES[stft_mod.pad_mode], fb_mod.n_mels, log_mel,
                     mult, off, amin, top_db)


def _can_fuse(stft_mod, fb_mod, wav):
    return (wav.dim() == 2 and fb_mod.freeze and not stft_mod.normalized_stft and stft_mod.onesided
            and fb_mod.power_spectrogram == 2 and not (fb_mod.param_rand_factor != 0 and fb_mod.training))


class Fbank(torch.nn.Module):
    """lobes/features.py:22-147."""

    def __init__(self, deltas=False, context=False, requires_grad=False, sample_rate=16000, f_min=0,
                 f_max=None, n_fft=400, n_mels=40, filter_shape="triangular", param_change_factor=1.0,
                 param_rand_factor=0.0, left_frames=5, right_frames=5, win_length=25, hop_length=10):
        super().__init__()
        self.deltas = deltas
        self.context = context
        self.requires_grad = requires_grad
        if f_max is None:
            f_max = sample_rate / 2
        self.compute_STFT = STFT(sample_rate=sample_rate, n_fft=n_fft, win_length=win_length,
                                 hop_length=hop_length)
        self.compute_fbanks = Filterbank(sample_rate=sample_rate, n_fft=n_fft, n_mels=n_mels, f_min=f_min,
                                         f_max=f_max, freeze=not requires_grad, filter_shape=filter_shape,
                                         param_change_factor=param_change_factor,
                                         param_rand_factor=param_rand_factor)
        self.compute_deltas = Deltas(input_size=n_mels)
        self.context_window = ContextWindow(left_frames=left_frames, right_frames=right_frames)

    def forward_deferred(self, wav):
        """forward() with the top_db floor left to the consumer: returns
        (features before the floor, (slot maxima (B, nslot), top_db)) when
        the fused spectrum kernel applies (log-mel, no deltas / context), else
        (forward(wav), None).  ConvolutionFrontEnd.run(..., topdb=...) applies
        the floor as it loads the rows (lobes/features.py:130-147 with
        processing/features.py:691-712, one pass over the features fewer)."""
        fb = self.compute_fbanks
        if (_can_fuse(self.compute_STFT, fb, wav) and fb.log_mel and fb.top_db is not None and not self.deltas
                and not self.context):
            return self._deferred(wav)
        return self.forward(wav), None

    def _deferred(self, wav):
        st, fb = self.compute_STFT, self.compute_fbanks
        w, tw1, tw2 = st._tables(wav.device)
        s0, ln, of, mw = fb.csr_tables(wav.device)
        _, mult, off, amin, top_db = fb._db_args()
        feats, slot_max = ops.fbank_deferred(wav, w, tw1, tw2, s0, ln, of, mw, st.n_fft, st.hop_length, st.center,
                                             ops.PAD_MODES[st.pad_mode], fb.n_mels, mult, off, amin)
        return feats, (slot_max, float(top_db))

    def forward(self, wav):
        """Returns the FBANK features of a batch of waveforms."""
        fb = self.compute_fbanks
        if (self.deltas and _can_fuse(self.compute_STFT, fb, wav) and fb.log_mel and fb.top_db is not None
                and fb.n_mels % 4 == 0):
            # the top_db floor applied by the concat deltas kernel as it loads
            # the rows (one pass over the features fewer)
            feats, (slot_max, top_db) = self._deferred(wav)
            fbanks = ops.deltas_floor(feats, 2 * self.compute_deltas.n + 1, slot_max, top_db)
            return self.context_window(fbanks) if self.context else fbanks
        if _can_fuse(self.compute_STFT, fb, wav):
            fbanks = _fused_fbank(self.compute_STFT, self.compute_fbanks, wav)
        else:
            fbanks = self.compute_fbanks(spectral_magnitude(self.compute_STFT(wav)))
        if self.deltas:
            if fbanks.dim() == 3:
                fbanks = ops.deltas(fbanks, 2 * self.compute_deltas.n + 1, True)
            else:
                d1 = self.compute_deltas(fbanks)
                d2 = self.compute_deltas(d1)
                fbanks = torch.cat([fbanks, d1, d2], dim=2)
        if self.context:
            fbanks = self.context_window(fbanks)
        return fbanks


class MFCC(torch.nn.Module):
    """lobes/features.py:150-281."""

    def __init__(self, deltas=True, context=True, requires_grad=False, sample_rate=16000, f_min=0,
                 f_max=None, n_fft=400, n_mels=23, n_mfcc=20, filter_shape="triangular",
                 param_change_factor=1.0, param_rand_factor=0.0, left_frames=5, right_frames=5,
                 win_length=25, hop_length=10):
        super().__init__()
        self.deltas = deltas
        self.context = context
        self.requires_grad = requires_grad
        if f_max is None:
            f_max = sample_rate / 2
        self.compute_STFT = STFT(sample_rate=sample_rate, n_fft=n_fft, win_length=win_length,
                                 hop_length=hop_length)
        self.compute_fbanks = Filterbank(sample_rate=sample_rate, n_fft=n_fft, n_mels=n_mels, f_min=f_min,
                                         f_max=f_max, freeze=not requires_grad, filter_shape=filter_shape,
                                         param_change_factor=param_change_factor,
                                         param_rand_factor=param_rand_factor)
        self.compute_dct = DCT(input_size=n_mels, n_out=n_mfcc)
        self.compute_deltas = Deltas(input_size=n_mfcc)
        self.context_window = ContextWindow(left_frames=left_frames, right_frames=right_frames)

    def forward(self, wav):
        """Returns the MFCCs of a batch of waveforms."""
        if _can_fuse(self.compute_STFT, self.compute_fbanks, wav):
            fbanks = _fused_fbank(self.compute_STFT, self.compute_fbanks, wav)
        else:
            fbanks = self.compute_fbanks(spectral_magnitude(self.compute_STFT(wav)))
        mfccs = self.compute_dct(fbanks)
        if self.deltas:
            if mfccs.dim() == 3:
                mfccs = ops.deltas(mfccs, 2 * self.compute_deltas.n + 1, True)
            else:
                d1 = self.compute_deltas(mfccs)
                d2 = self.compute_deltas(d1)
                mfccs = torch.cat([mfccs, d1, d2], dim=2)
        if self.context:
            mfccs = self.context_window(mfccs)
        return mfccs
