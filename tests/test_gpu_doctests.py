"""Every SURVEY §4 doctest example (plus the other drop-in modules' own
doctests) executed on the HIP drop-ins at the doctest's shapes
(tests/golden/doctest_cases.py, each case citing its reference lines): the
output shape must equal the one the doctest prints, and the first batch
element must equal the reference's output on the same inputs and detinit
weights (tests/golden/doctests.npz) within |a - b| <= 1e-4 * max(1, |b|).
The TransformerASR doctest also runs in training mode (its dropout 0.1, as
the doctest itself does) for the shape."""
from types import SimpleNamespace

import numpy as np
import pytest
import torch

from conftest import assert_close
from detinit import det_state
from doctest_cases import cases

pytestmark = pytest.mark.gpu

CASES = cases()


def _ns():
    from speechbrain_amd.processing import features as PF
    from speechbrain_amd.lobes import features as LFe
    from speechbrain_amd.lobes.augment import SpecAugment
    from speechbrain_amd.lobes.models.transformer import Conformer as RC, Transformer as RT, TransformerASR as RA
    from speechbrain_amd.lobes.models import convolution as RCV, wav2vec as RW
    from speechbrain_amd.nnet import attention as RAT, CNN as RCNN, linear as RL, normalization as RN
    from speechbrain_amd.nnet import activations as RACT
    from speechbrain_amd.nnet.transducer import transducer_joint as RJ
    return SimpleNamespace(
        STFT=PF.STFT, spectral_magnitude=PF.spectral_magnitude, Filterbank=PF.Filterbank, DCT=PF.DCT,
        Deltas=PF.Deltas, ContextWindow=PF.ContextWindow, InputNormalization=PF.InputNormalization,
        Fbank=LFe.Fbank, MFCC=LFe.MFCC, SpecAugment=SpecAugment, ConvolutionFrontEnd=RCV.ConvolutionFrontEnd,
        ConvBlock=RCV.ConvBlock, Conv2d=RCNN.Conv2d, Linear=RL.Linear, LayerNorm=RN.LayerNorm, Swish=RACT.Swish,
        RelPosMHAXL=RAT.RelPosMHAXL, MultiheadAttention=RAT.MultiheadAttention,
        PositionalwiseFeedForward=RAT.PositionalwiseFeedForward, ConvolutionModule=RC.ConvolutionModule,
        ConformerEncoderLayer=RC.ConformerEncoderLayer, ConformerEncoder=RC.ConformerEncoder,
        PositionalEncoding=RT.PositionalEncoding, TransformerEncoderLayer=RT.TransformerEncoderLayer,
        TransformerEncoder=RT.TransformerEncoder, TransformerDecoderLayer=RT.TransformerDecoderLayer,
        TransformerDecoder=RT.TransformerDecoder, NormalizedEmbedding=RT.NormalizedEmbedding,
        TransformerASR=RA.TransformerASR, EncoderWrapper=RA.EncoderWrapper, GELU=torch.nn.GELU,
        Transducer_joint=RJ.Transducer_joint, W2VLatentExtractor=RW.W2VLatentExtractor,
        W2VEncoderWrapper=RW.EncoderWrapper)


@pytest.mark.parametrize("case", CASES, ids=[c.name for c in CASES])
def test_doctest_example(golden, dev, case):
    g = golden("doctests")
    ns = _ns()
    m = case.build(ns) if case.build is not None else None
    if m is not None:
        if case.det:
            m.load_state_dict(det_state(m, case.seed), strict=True)
        m = m.to(dev).train(not case.eval_mode)
    xs = case.make_inputs(torch, dev)
    torch.manual_seed(case.seed)
    with torch.no_grad():
        y = case.call(ns, m, *xs)
    assert tuple(y.shape) == case.shape, f"{case.name} ({case.cite}): {tuple(y.shape)} != {case.shape}"
    assert tuple(g[case.name + ".shape"]) == case.shape
    assert_close(case.keep(y), g[case.name + ".out"], name=f"{case.name} ({case.cite})")


def test_transformer_asr_doctest_train_mode(dev):
    """TransformerASR.py:75-85 verbatim in spirit: default (training) mode,
    dropout 0.1, gradients enabled."""
    from speechbrain_amd.lobes.models.transformer.TransformerASR import TransformerASR, EncoderWrapper
    src = torch.rand([8, 120, 512], device=dev)
    tgt = torch.randint(0, 720, [8, 120], device=dev)
    net = TransformerASR(720, 512, 512, 8, 1, 1, 1024, activation=torch.nn.GELU).to(dev)
    enc_out, dec_out = net.forward(src, tgt)
    assert enc_out.shape == torch.Size([8, 120, 512])
    assert dec_out.shape == torch.Size([8, 120, 512])
    (enc_out.sum() + dec_out.sum()).backward()
    assert all(p.grad is not None for p in net.encoder.parameters())
    enc = EncoderWrapper(net)(src)
    assert enc.shape == torch.Size([8, 120, 512])
    assert np.isfinite(enc.detach().cpu().numpy()).all()
