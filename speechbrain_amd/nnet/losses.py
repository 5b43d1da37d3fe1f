"""Drop-in for speechbrain.nnet.losses.transducer_loss (losses.py:27-85).

use_torchaudio=False: the SpeechBrain Numba semantics (time-normalised loss,
un-normalised gradients), pinned by the reference's known-answer test.
use_torchaudio=True: torchaudio.functional.rnnt_loss semantics (-log P,
mean over the batch, standard gradients) computed by the same HIP kernels
— torchaudio is not a dependency; this mode's parity is unpinned by the
reference's tests.
"""
import torch

from .loss.transducer_loss import TransducerLogits


def transducer_loss(logits, targets, input_lens, target_lens, blank_index, reduction="mean", use_torchaudio=True):
    input_lens = (input_lens * logits.shape[1]).round().int()
    target_lens = (target_lens * targets.shape[1]).round().int()
    if use_torchaudio:
        return TransducerLogits.apply(logits, targets, input_lens, target_lens, blank_index, reduction, 1)
    return TransducerLogits.apply(logits, targets, input_lens, target_lens, blank_index, reduction, 0)
