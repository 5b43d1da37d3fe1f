"""Drop-in coverage beyond the recipe configuration, on the HIP kernels,
against outputs of the reference itself (tests/golden/dropin.npz, made by
tests/golden/gen_golden.py) and the oracle:

  * ConvolutionFrontEnd(input_shape) with every default — 3 residual blocks
    x 5 layers, (128, 256, 512) channels, strides (1, 2, 2)
    (lobes/models/convolution.py:12-175) — forward;
  * a residual, 2-layer, kernel-5 front-end: forward and every gradient;
  * RelPosMHAXL attn_mask (attention.py:598-611): bool causal (T, T) and
    float additive (B*H, T, T), and vbias=True (:576-579);
  * ConformerEncoder with a src_mask vs the oracle;
  * SpecAugment time_warp_mode="bilinear" (augment.py:134-148).
fp32 tolerance as everywhere: |a - b| <= 1e-4 * max(1, |b|); gradients within
1e-4 of the tensor's largest reference gradient."""
import numpy as np
import pytest
import torch

from conftest import assert_close
import oracle.conformer as OC

pytestmark = pytest.mark.gpu


def assert_grad(a, b, rtol=1e-4, name=""):
    a = a.detach().float().cpu()
    b = torch.as_tensor(b).float()
    assert a.shape == b.shape, f"{name}: shape {tuple(a.shape)} != {tuple(b.shape)}"
    scale = max(b.abs().max().item(), 1e-12)
    err = (a - b).abs().max().item()
    assert err <= rtol * scale, f"{name}: max err {err:.3e} vs scale {scale:.3e}"


def test_default_frontend_forward(golden, dev):
    from speechbrain_amd.lobes.models.convolution import ConvolutionFrontEnd
    g = golden("dropin")
    torch.manual_seed(0)
    fe = ConvolutionFrontEnd(input_shape=(8, 30, 10)).to(dev).eval()
    with torch.no_grad():
        y = fe(torch.from_numpy(g["fe_def_x"]).to(dev))
    assert tuple(y.shape) == (8, 8, 3, 512)
    assert_close(y, g["fe_def_y"], name="default ConvolutionFrontEnd")


def _fe2(g, dev):
    from speechbrain_amd.lobes.models.convolution import ConvolutionFrontEnd
    fe = ConvolutionFrontEnd(input_shape=(3, 37, 20), num_blocks=2, num_layers_per_block=2, out_channels=(8, 16),
                             kernel_sizes=(3, 5), strides=(1, 2), residuals=(True, True), dropout=0.1)
    fe.load_state_dict({k[4:]: torch.from_numpy(g[k]) for k in g.files if k.startswith("fe2.")}, strict=True)
    return fe.to(dev)


def test_residual_frontend_forward_backward(golden, dev):
    g = golden("dropin")
    fe = _fe2(g, dev).eval()
    with torch.no_grad():
        assert_close(fe(torch.from_numpy(g["fe2_x"]).to(dev)), g["fe2_y"], name="fe2 no-grad")
    x = torch.from_numpy(g["fe2_x"]).to(dev).requires_grad_(True)
    y = fe(x)
    assert_close(y, g["fe2_y"], name="fe2")
    (y * torch.from_numpy(g["fe2_R"]).to(dev)).sum().backward()
    assert_grad(x.grad, g["fe2_grad_x"], name="dx")
    n = 0
    for k, p in fe.named_parameters():
        assert_grad(p.grad, g["fe2_grad." + k], name=k)
        n += 1
    assert n == sum(1 for k in g.files if k.startswith("fe2_grad."))


def test_residual_frontend_train_dropout(golden, dev):
    """Training mode: per-layer and block dropouts draw; same seed, same
    output; eval equals the reference."""
    g = golden("dropin")
    fe = _fe2(g, dev).train()
    x = torch.from_numpy(g["fe2_x"]).to(dev)
    torch.manual_seed(4)
    y1 = fe(x)
    torch.manual_seed(4)
    y2 = fe(x)
    y3 = fe(x)
    assert torch.equal(y1, y2) and not torch.equal(y1, y3) and torch.isfinite(y1).all()


def _mha(g, prefix, dev, **kw):
    from speechbrain_amd.nnet.attention import RelPosMHAXL
    m = RelPosMHAXL(embed_dim=64, num_heads=4, **kw)
    m.load_state_dict({k[len(prefix):]: torch.from_numpy(g[k]) for k in g.files if k.startswith(prefix)}, strict=True)
    return m.to(dev).eval()


@pytest.mark.parametrize("tag", ["causal", "float"])
def test_relposmha_attn_mask(golden, dev, tag):
    g = golden("dropin")
    mha = _mha(g, "mha.", dev)
    q = torch.from_numpy(g["mha_q"]).to(dev)
    pe = torch.from_numpy(g["mha_pe"]).to(dev)
    kpm = torch.from_numpy(g["mha_kpm"]).to(dev)
    T = q.shape[1]
    am = (torch.triu(torch.ones(T, T, dtype=torch.bool), diagonal=1) if tag == "causal"
          else torch.from_numpy(g["mha_fmask"])).to(dev)
    with torch.no_grad():
        out, attn = mha(q, q, q, pe, key_padding_mask=kpm, attn_mask=am)
    assert_close(out, g[f"mha_{tag}_out"], name=f"{tag} out")
    assert_close(attn, g[f"mha_{tag}_attn"], name=f"{tag} attn")
    # training path (probabilities kept, backward kernels): same forward
    mha.train()
    qd = q.clone().requires_grad_(True)
    out_t, attn_t = mha(qd, qd, qd, pe, key_padding_mask=kpm, attn_mask=am)
    assert_close(out_t, g[f"mha_{tag}_out"], name=f"{tag} train out")
    out_t.sum().backward()
    assert torch.isfinite(qd.grad).all()
    if tag == "causal":
        assert (attn_t.detach().cpu()[..., torch.triu(torch.ones(T, T, dtype=torch.bool), 1)] == 0).all()


def test_relposmha_vbias(golden, dev):
    g = golden("dropin")
    mha = _mha(g, "mhv.", dev, vbias=True)
    q = torch.from_numpy(g["mha_q"]).to(dev)
    pe = torch.from_numpy(g["mha_pe"]).to(dev)
    kpm = torch.from_numpy(g["mha_kpm"]).to(dev)
    with torch.no_grad():
        out, attn = mha(q, q, q, pe, key_padding_mask=kpm)
    assert_close(out, g["mhv_out"], name="vbias out")
    assert_close(attn, g["mhv_attn"], name="vbias attn")
    mha.train()
    out_t, _ = mha(q, q, q, pe, key_padding_mask=kpm)
    assert_close(out_t, g["mhv_out"], name="vbias train out")
    out_t.sum().backward()
    # d(sum out)/d(value bias) = sum over rows of the attention-weighted out_proj input gradient
    assert mha.value_bias_weight.grad is not None and torch.isfinite(mha.value_bias_weight.grad).all()
    assert mha.value_bias_weight.grad.abs().sum() > 0


@pytest.mark.parametrize("train", [False, True])
def test_conformer_encoder_src_mask_vs_oracle(golden, dev, train):
    """ConformerEncoder(src_mask = causal) — inference and training paths —
    vs the oracle (Conformer.py:343-383 with the mask passed to every
    layer's attention)."""
    from speechbrain_amd.lobes.models.transformer.Conformer import ConformerEncoder
    gc = golden("conformer")
    enc = ConformerEncoder(num_layers=2, d_model=64, d_ffn=128, nhead=4, kernel_size=31)
    sd = {k[4:]: torch.from_numpy(gc[k]) for k in gc.files if k.startswith("enc.")}
    enc.load_state_dict(sd, strict=True)
    enc = enc.to(dev).train(train)
    src = torch.from_numpy(gc["enc_src"])
    kpm = torch.from_numpy(gc["enc_kpm"])
    pe = torch.from_numpy(gc["enc_pos"])
    T = src.shape[1]
    causal = torch.triu(torch.ones(T, T, dtype=torch.bool), diagonal=1)
    for m in enc.modules():
        if isinstance(m, torch.nn.Dropout):
            m.p = 0.0
    sdo = {k: v.clone().requires_grad_(True) for k, v in sd.items()}
    xr = src.clone().requires_grad_(True)
    ref, _ = OC.conformer_encoder(xr, pe, sdo, "", 2, 4, key_padding_mask=kpm, attn_mask=causal)
    xd = src.to(dev).requires_grad_(train)
    with torch.set_grad_enabled(train):  # no grad: the fused inference kernels (per-layer path)
        y, attn = enc(xd, src_mask=causal.to(dev), src_key_padding_mask=kpm.to(dev), pos_embs=pe.to(dev))
    assert_close(y, ref.detach(), name="encoder with src_mask")
    assert (attn[0].detach().cpu()[..., causal] == 0).all()
    if train:
        R = torch.randn(ref.shape, generator=torch.Generator().manual_seed(3))
        (ref * R).sum().backward()
        (y * R.to(dev)).sum().backward()
        assert_grad(xd.grad, xr.grad, name="dsrc")
        for k, p in enc.named_parameters():
            assert_grad(p.grad, sdo[k].grad, name=k)


def test_specaugment_bilinear_warp(golden, dev):
    from speechbrain_amd.lobes.augment import SpecAugment
    g = golden("dropin")
    aug = SpecAugment(time_warp=True, time_warp_mode="bilinear", freq_mask=False, time_mask=False)
    feats = torch.from_numpy(g["warp_feats"])
    for s in range(3):
        torch.manual_seed(s)
        assert_close(aug(feats.clone().to(dev)), g[f"warp_bilinear_s{s}"], rtol=1e-5, name=f"bilinear s{s}")
    with pytest.raises(ValueError):
        SpecAugment(time_warp=True, time_warp_mode="nearest")
