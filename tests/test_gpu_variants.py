"""TransformerASR / encoder constructor variants on the HIP drop-ins, against
the reference's own outputs (tests/golden/variants.npz, made by
tests/golden/gen_golden.py from tests/golden/variant_cases.py):

  doc    the reference's TransformerASR doctest constructor
         (TransformerASR.py:77-79: transformer encoder, regularMHA,
         fixed_abs_sine, post-norm, GELU, d_model 512)
  tyaml  recipes/LibriSpeech/ASR/transformer/hparams/transformer.yaml:122-150
         (its 3-block CNN, pre-norm GELU transformer, regularMHA) at d 64
  trel   transformer encoder + RelPosMHAXL (Transformer.py:307-310), post-norm
         ReLU, causal=True
  trels  ... pre-norm with a Swish FFN
  cmha   Conformer with regularMHA (Conformer.py:173-180) + absolute sine table
  cmhac  ... causal
Each: weights loaded with load_state_dict(strict=True), forward (with and
without wav_len), encode, decode, and the gradients of sum(R * encode) w.r.t.
the encoder-side parameters and the input; plus ConformerEncoder(regularMHA)
called directly with a bool src_mask and a key padding mask.
fp32 tolerance |a - b| <= 1e-4 * max(1, |b|); gradients within 1e-4 of the
tensor's largest reference gradient."""
import numpy as np
import pytest
import torch

from conftest import assert_close
from detinit import det_state
from variant_cases import VARIANTS

pytestmark = pytest.mark.gpu


def assert_grad(a, b, rtol=1e-4, name=""):
    a = a.detach().float().cpu()
    b = torch.as_tensor(b).float()
    assert a.shape == b.shape, f"{name}: shape {tuple(a.shape)} != {tuple(b.shape)}"
    scale = max(b.abs().max().item(), 1e-12)
    err = (a - b).abs().max().item()
    assert err <= rtol * scale, f"{name}: max err {err:.3e} vs scale {scale:.3e}"


def _model(ctor, seed):
    from speechbrain_amd.lobes.models.transformer.TransformerASR import TransformerASR
    from speechbrain_amd.nnet.activations import Swish
    kw = dict(ctor)
    act = kw.pop("act", None)
    if act is not None:
        kw["activation"] = {"gelu": torch.nn.GELU, "relu": torch.nn.ReLU, "swish": Swish}[act]
    m = TransformerASR(**kw)
    m.load_state_dict(det_state(m, seed), strict=True)
    return m


def _cnn(seed):
    from speechbrain_amd.lobes.models.convolution import ConvolutionFrontEnd
    cnn = ConvolutionFrontEnd(input_shape=(8, 10, 80), num_blocks=3, num_layers_per_block=1,
                              out_channels=(64, 64, 64), kernel_sizes=(5, 5, 1), strides=(2, 2, 1),
                              residuals=(False, False, True))
    cnn.load_state_dict(det_state(cnn, seed), strict=True)
    return cnn


@pytest.mark.parametrize("tag", list(VARIANTS))
def test_transformer_asr_variant(golden, dev, tag):
    g = golden("variants")
    i = list(VARIANTS).index(tag)
    c = VARIANTS[tag]
    model = _model(c["ctor"], 50 + i).to(dev).eval()
    cnn = _cnn(150 + i).to(dev).eval() if c.get("cnn") else None
    x = torch.from_numpy(g[f"{tag}.x"]).to(dev)
    tgt = torch.from_numpy(g[f"{tag}.tgt"]).to(dev)
    wl = torch.from_numpy(g[f"{tag}.wav_len"]).to(dev)
    with torch.no_grad():
        src = cnn(x) if cnn is not None else x
        e1, d1 = model(src, tgt, wl)
        assert_close(e1, g[f"{tag}.fwd_enc"], name=f"{tag} forward encoder_out")
        assert_close(d1, g[f"{tag}.fwd_dec"], name=f"{tag} forward decoder_out")
        e0, d0 = model(src, tgt)
        assert_close(e0, g[f"{tag}.fwd0_enc"], name=f"{tag} forward (no wav_len) encoder_out")
        assert_close(d0, g[f"{tag}.fwd0_dec"], name=f"{tag} forward (no wav_len) decoder_out")
        enc = model.encode(src, wl)
        assert_close(enc, g[f"{tag}.enc"], name=f"{tag} encode")
        assert_close(model.encode(src), g[f"{tag}.enc0"], name=f"{tag} encode (no wav_len)")
        pred, att = model.decode(tgt, torch.from_numpy(g[f"{tag}.enc"]).to(dev),
                                 torch.from_numpy(g[f"{tag}.enc_len"]).to(dev))
        assert_close(pred, g[f"{tag}.dec_pred"], name=f"{tag} decode prediction")
        assert_close(att, g[f"{tag}.dec_att"], name=f"{tag} decode attention")
    if not c["grads"]:
        return
    xg = x.clone().requires_grad_(True)
    y = model.encode(cnn(xg) if cnn is not None else xg, wl)
    R = torch.from_numpy(np.asarray(_R(tuple(y.shape), 400 + i))).to(dev)
    (y * R).sum().backward()
    assert_grad(xg.grad, g[f"{tag}.grad_x"], name=f"{tag} dx")
    n = 0
    for k, p in model.named_parameters():
        key = f"{tag}.grad.{k}"
        if key in g.files:
            assert_grad(p.grad, g[key], name=f"{tag} d{k}")
            n += 1
    assert n > 0


def _R(shape, seed):
    from detinit import det_input
    return det_input(shape, seed)


def test_conformer_encoder_regular_mha_masks(golden, dev):
    """ConformerEncoder(attention_type="regularMHA") with src_mask + key padding:
    output, per-layer attention maps, gradients (Conformer.py:118-383)."""
    from speechbrain_amd.lobes.models.transformer.Conformer import ConformerEncoder
    g = golden("variants")
    enc = ConformerEncoder(2, 64, 128, 4, kernel_size=7, attention_type="regularMHA")
    enc.load_state_dict(det_state(enc, 90), strict=True)
    enc = enc.to(dev).eval()
    x = torch.from_numpy(g["cenc.x"]).to(dev).requires_grad_(True)
    kpm = torch.from_numpy(g["cenc.kpm"]).to(dev)
    am = torch.from_numpy(g["cenc.am"]).to(dev)
    y, attns = enc(x, src_mask=am, src_key_padding_mask=kpm)
    assert_close(y, g["cenc.y"], name="y")
    for j, a in enumerate(attns):
        assert_close(a, g[f"cenc.attn{j}"], name=f"attn{j}")
    R = torch.from_numpy(_R(tuple(y.shape), 92)).to(dev)
    (y * R).sum().backward()
    assert_grad(x.grad, g["cenc.grad_x"], name="dx")
    for k, p in enc.named_parameters():
        assert_grad(p.grad, g[f"cenc.grad.{k}"], name=f"d{k}")


def test_positional_encoding_none_raises(dev):
    """TransformerASR(positional_encoding=None, attention_type="regularMHA"):
    the reference leaves the positional term unset and fails in encode()
    (TransformerASR.py:304-315, UnboundLocalError); the drop-in raises too."""
    from speechbrain_amd.lobes.models.transformer.TransformerASR import TransformerASR
    m = TransformerASR(10, 16, d_model=32, nhead=4, num_encoder_layers=1, num_decoder_layers=1, d_ffn=64,
                       positional_encoding=None).to(dev).eval()
    with pytest.raises((ValueError, UnboundLocalError)):
        with torch.no_grad():
            m.encode(torch.rand(2, 5, 16, device=dev))


def test_transformer_encoder_float_padding_mask(dev):
    """An additive float key padding mask through TransformerEncoder in eval /
    no_grad takes the module path (0 / -inf adds), equal to the bool mask."""
    from speechbrain_amd.lobes.models.transformer.Transformer import TransformerEncoder
    enc = TransformerEncoder(2, 4, 128, d_model=64, normalize_before=True, activation=torch.nn.GELU)
    enc.load_state_dict(det_state(enc, 7), strict=True)
    enc = enc.to(dev).eval()
    x = torch.from_numpy(_R((3, 13, 64), 8)).to(dev)
    kb = torch.arange(13, device=dev)[None, :] >= torch.tensor([13, 9, 5], device=dev)[:, None]
    kf = torch.zeros(3, 13, device=dev).masked_fill(kb, float("-inf"))
    with torch.no_grad():
        yb, _ = enc(x, src_key_padding_mask=kb)
        yf, _ = enc(x, src_key_padding_mask=kf)
    assert torch.isfinite(yf).all()
    assert_close(yf, yb.cpu().numpy(), name="float mask vs bool mask")


@pytest.mark.parametrize("grad", [False, True])
def test_conformer_encoder_wide_heads_vs_oracle(dev, grad):
    """RelPosMHAXL heads wider than the fused kernels take (d_model 384, 2
    heads: dh 192) run the per-module layer with the xattn core; checked
    against the oracle restatement (oracle/conformer.py), forward and, with
    grad, every gradient."""
    import oracle.conformer as OC
    from speechbrain_amd.lobes.models.transformer.Conformer import ConformerEncoder
    enc = ConformerEncoder(num_layers=1, d_model=384, d_ffn=256, nhead=2, kernel_size=7)
    assert enc.layers[0].module_layer
    sd = det_state(enc, 11)
    enc.load_state_dict(sd, strict=True)
    enc = enc.to(dev).eval()
    T = 19
    src = torch.from_numpy(_R((2, T, 384), 12))
    pe = torch.from_numpy(_R((1, 2 * T - 1, 384), 13))
    kpm = torch.arange(T)[None, :] >= torch.tensor([T, 11])[:, None]
    sdo = {k: v.clone().requires_grad_(grad) for k, v in sd.items()}
    xr = src.clone().requires_grad_(grad)
    with torch.set_grad_enabled(grad):
        ref, _ = OC.conformer_encoder(xr, pe, sdo, "", 1, 2, kernel_size=7, key_padding_mask=kpm)
        xd = src.to(dev).requires_grad_(grad)
        y, _ = enc(xd, src_key_padding_mask=kpm.to(dev), pos_embs=pe.to(dev))
    assert_close(y, ref.detach(), name="wide-head encoder")
    if grad:
        R = torch.from_numpy(_R(tuple(ref.shape), 14))
        (ref * R).sum().backward()
        (y * R.to(dev)).sum().backward()
        assert_grad(xd.grad, xr.grad, name="dsrc")
        for k, p in enc.named_parameters():
            assert_grad(p.grad, sdo[k].grad, name=k)
