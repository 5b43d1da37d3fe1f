"""speechbrain_amd — MI355X-native (gfx950) drop-in for SpeechBrain's speech
front-end + Conformer encoder + RNN-T loss hot path.

Import paths mirror the reference (Sinica-SLAM/speechbrain 0.5.13):
    speechbrain_amd.processing.features   STFT, spectral_magnitude, Filterbank, DCT, Deltas, ContextWindow
    speechbrain_amd.lobes.features        Fbank, MFCC
    speechbrain_amd.lobes.augment         SpecAugment
    speechbrain_amd.lobes.models.convolution            ConvolutionFrontEnd, ConvBlock
    speechbrain_amd.lobes.models.transformer.Conformer  ConformerEncoder, ConformerEncoderLayer, ConvolutionModule
    speechbrain_amd.lobes.models.transformer.TransformerASR  TransformerASR (encode path)
    speechbrain_amd.nnet.attention        RelPosEncXL, RelPosMHAXL, PositionalwiseFeedForward
    speechbrain_amd.nnet.loss.transducer_loss  Transducer, TransducerLoss
    speechbrain_amd.nnet.losses           transducer_loss
All compute runs in hand-written HIP kernels (libsbk.so, C ABI in include/sbk.h).
"""
import torch  # noqa: F401  (must load before libsbk.so: shared HIP runtime)

__version__ = "0.1.0"
