"""speechbrain_amd — MI355X-native (gfx950) drop-in for SpeechBrain's speech
front-end + Conformer encoder + RNN-T loss hot path.

Import paths mirror the reference (Sinica-SLAM/speechbrain 0.5.13):
    speechbrain_amd.processing.features   STFT, spectral_magnitude, Filterbank, DCT, Deltas, ContextWindow
    speechbrain_amd.lobes.features        Fbank, MFCC
    speechbrain_amd.lobes.augment         SpecAugment
    speechbrain_amd.lobes.models.convolution            ConvolutionFrontEnd, ConvBlock
    speechbrain_amd.lobes.models.transformer.Conformer  ConformerEncoder, ConformerEncoderLayer, ConvolutionModule
    speechbrain_amd.lobes.models.transformer.TransformerASR  TransformerASR (encode path)
    speechbrain_amd.lobes.models.transformer.Transformer  TransformerEncoder, TransformerEncoderLayer, PositionalEncoding
    speechbrain_amd.lobes.models.wav2vec  W2VLatentExtractor, EncoderWrapper (config 5)
    speechbrain_amd.nnet.attention        RelPosEncXL, RelPosMHAXL, PositionalwiseFeedForward, MultiheadAttention
    speechbrain_amd.nnet.loss.transducer_loss  Transducer, TransducerLoss
    speechbrain_amd.nnet.losses           transducer_loss
All compute runs in hand-written HIP kernels (libsbk.so, C ABI in include/sbk.h).
"""
import torch  # noqa: F401  (must load before libsbk.so: shared HIP runtime)

__version__ = "0.2.0"


def mxfp8(enabled=True):
    """Context manager: config-5 GEMMs on MXFP8 operands (see _enc.mxfp8)."""
    from ._enc import mxfp8 as _mx
    return _mx(enabled)
