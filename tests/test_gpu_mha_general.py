"""MultiheadAttention beyond inference self-attention (attention.py:642-778):
cross-attention with S != L, attn_mask (bool / byte / additive, 2-D and
(B*H, L, S)), pos_embs, float key padding, kdim / vdim, gradients — and the
TransformerEncoder(Layer) with src_mask / pos_embs / gradients
(Transformer.py:343-376, 448-486).  The reference's MultiheadAttention is
torch.nn.MultiheadAttention called on (L, B, E) tensors (attention.py:749-
778); it and the layer's composition run here on the CPU in fp32 with the
drop-in's weights as the oracle."""
import copy

import pytest
import torch
import torch.nn as nn

pytestmark = pytest.mark.gpu


def _ref_mha(att, q, k, v, attn_mask=None, kpm=None, pos_embs=None):
    if pos_embs is not None:  # attention.py:756-761, in place
        if attn_mask is not None:
            attn_mask += pos_embs
        else:
            attn_mask = pos_embs
    o, w = att(q.permute(1, 0, 2), k.permute(1, 0, 2), v.permute(1, 0, 2), attn_mask=attn_mask, key_padding_mask=kpm,
               need_weights=True)
    return o.permute(1, 0, 2), w


def _close(a, b, tol, what):
    sc = max(1.0, float(b.abs().max()))
    err = float((a.detach().float().cpu() - b.detach().float()).abs().max())
    assert err <= tol * sc, (what, err)


CASES = {
    "cross_bool_masks": dict(L=7, S=11, kpm="bool", am="bool2"),
    "self_float3d_pos": dict(L=9, S=9, am="float3", pos=True, self_attn=True),
    "cross_float_kpm": dict(L=5, S=13, kpm="float", am="float2"),
    "byte_mask": dict(L=6, S=8, am="byte2", kpm="bool"),
    "kdim_vdim": dict(L=7, S=10, kdim=20, vdim=24),
    # several 16-row query blocks and 64-key chunks, 128-dim heads (the
    # query-blocked xattn kernels' loop structure and their dh bound)
    "cross_multi_chunk": dict(L=37, S=150, E=256, H=2, kpm="bool", am="float2"),
    "self_multi_chunk": dict(L=70, S=70, E=64, H=4, am="bool2", self_attn=True),
}


@pytest.mark.parametrize("name", list(CASES))
def test_mha_general_vs_torch(dev, name):
    from speechbrain_amd.nnet.attention import MultiheadAttention
    c = CASES[name]
    B, E, H, L, S = 2, c.get("E", 32), c.get("H", 4), c["L"], c["S"]
    torch.manual_seed(len(name))
    mha = MultiheadAttention(nhead=H, d_model=E, kdim=c.get("kdim"), vdim=c.get("vdim")).eval()
    att = copy.deepcopy(mha.att)  # the CPU reference keeps its own parameters (and grads)
    q = torch.randn(B, L, E)
    k = q if c.get("self_attn") else torch.randn(B, S, c.get("kdim") or E)
    v = q if c.get("self_attn") else torch.randn(B, S, c.get("vdim") or E)
    am = None
    if c.get("am") == "bool2":
        am = torch.rand(L, S) < 0.2
        am[:, 0] = False
    elif c.get("am") == "byte2":
        am = (torch.rand(L, S) < 0.2).to(torch.uint8)
        am[:, 0] = 0
    elif c.get("am") == "float2":
        am = torch.randn(L, S)
    elif c.get("am") == "float3":
        am = torch.randn(B * H, L, S)
    kpm = None
    if c.get("kpm") == "bool":
        kpm = torch.zeros(B, S, dtype=torch.bool)
        kpm[1, -3:] = True
        kpm[0, S // 2:] = S > 64  # a padded tail longer than a key chunk
    elif c.get("kpm") == "float":
        kpm = torch.randn(B, S)
    pos = torch.randn(L, S) if c.get("pos") else None
    qr, kr, vr = (t.clone().requires_grad_(True) for t in (q, k, v))
    if c.get("self_attn"):
        kr = vr = qr
    ref_am = am.bool() if am is not None and am.dtype == torch.uint8 else am
    ro, rw = _ref_mha(att, qr, kr, vr, None if ref_am is None else ref_am.clone(), kpm, pos)
    mha = mha.to(dev)
    qd = q.to(dev).requires_grad_(True)
    kd = qd if c.get("self_attn") else k.to(dev).requires_grad_(True)
    vd = qd if c.get("self_attn") else v.to(dev).requires_grad_(True)
    o, w = mha(qd, kd, vd, attn_mask=None if am is None else am.to(dev),
               key_padding_mask=None if kpm is None else kpm.to(dev), pos_embs=None if pos is None else pos.to(dev))
    _close(o, ro, 1e-5, "out")
    _close(w, rw, 1e-5, "weights")
    g = torch.randn_like(ro)
    ro.backward(g)
    o.backward(g.to(dev))
    _close(qd.grad, qr.grad, 2e-5, "dq")
    if not c.get("self_attn"):
        _close(kd.grad, kr.grad, 2e-5, "dk")
        _close(vd.grad, vr.grad, 2e-5, "dv")
    wname = "in_proj_weight" if att._qkv_same_embed_dim else "q_proj_weight"
    _close(getattr(mha.att, wname).grad, getattr(att, wname).grad, 5e-5, "d" + wname)
    _close(mha.att.out_proj.weight.grad, att.out_proj.weight.grad, 5e-5, "dout_proj")


def _ref_layer(layer, src, src_mask, kpm, pos):
    """Transformer.py:343-376 with torch modules holding the layer's weights."""
    pre = layer.normalize_before
    n1, n2 = layer.norm1.norm, layer.norm2.norm
    src1 = n1(src) if pre else src
    out, attn = _ref_mha(layer.self_att.att, src1, src1, src1, src_mask, kpm, pos)
    src = src + out
    if not pre:
        src = n1(src)
    src1 = n2(src) if pre else src
    f = layer.pos_ffn.ffn
    out = src + f[3](f[1](f[0](src1)))
    if not pre:
        out = n2(out)
    return out, attn


@pytest.mark.parametrize("pre", [True, False])
def test_transformer_encoder_masks_and_grads(dev, pre):
    from speechbrain_amd.lobes.models.transformer.Transformer import TransformerEncoder
    torch.manual_seed(3)
    B, T, d = 2, 12, 32
    enc = TransformerEncoder(num_layers=2, nhead=4, d_ffn=64, d_model=d, activation=nn.GELU, normalize_before=pre)
    enc.eval()
    x = torch.randn(B, T, d)
    # causal, additive: the reference adds pos_embs into it in place, once per
    # layer (attention.py:756-761), which the drop-in reproduces
    src_mask = torch.zeros(T, T).masked_fill(torch.triu(torch.ones(T, T, dtype=torch.bool), diagonal=1), -1e4)
    kpm = torch.zeros(B, T, dtype=torch.bool)
    kpm[1, -4:] = True
    pos = 0.1 * torch.randn(T, T)
    ref_enc = copy.deepcopy(enc)
    xr = x.clone().requires_grad_(True)
    out = xr
    ref_mask = src_mask.clone()
    for layer in ref_enc.layers:
        out, _ = _ref_layer(layer, out, ref_mask, kpm, pos)
    ref = ref_enc.norm.norm(out)
    enc = enc.to(dev)
    xd = x.to(dev).requires_grad_(True)
    y, attns = enc(xd, src_mask=src_mask.clone().to(dev), src_key_padding_mask=kpm.to(dev), pos_embs=pos.to(dev))
    assert len(attns) == 2 and attns[0].shape == (B, T, T)
    _close(y, ref, 2e-5, "encoder out")
    g = torch.randn_like(ref)
    ref.backward(g)
    y.backward(g.to(dev))
    _close(xd.grad, xr.grad, 5e-5, "dx")


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_nopos_core_dropout_vs_autograd(dev, dtype):
    """The no-position xattn core (the MultiheadAttention general path) in
    training with attention dropout, over several query blocks and key chunks:
    the returned weights are the kept probabilities / (1 - p), out = attn · V,
    and dq / dk / dv equal autograd of that composition under the same keep
    mask (recovered from the weights).  fp32 1e-5 of the largest value; bf16
    operands: the fp32 reference is fed the same rounded operands."""
    from speechbrain_amd import _autograd as A
    from speechbrain_amd import _enc
    torch.manual_seed(9)
    B, H, dh, Lq, Lk, p = 2, 2, 64, 37, 150, 0.25
    q = torch.randn(B * Lq, H * dh, device=dev).to(dtype).requires_grad_(True)
    k = torch.randn(B * Lk, H * dh, device=dev).to(dtype).requires_grad_(True)
    v = torch.randn(B * Lk, H * dh, device=dev).to(dtype).requires_grad_(True)
    kpm = torch.zeros(B, Lk, dtype=torch.uint8, device=dev)
    kpm[1, 100:] = 1
    am = torch.randn(Lq, Lk, device=dev)
    scale = dh ** -0.5
    o, attn = A.RelPosCrossAttnFn.apply(q, k, v, None, None, None, kpm, _enc.attn_mask_arg(am, B, Lq, H, dev, Lk=Lk),
                                        B, Lq, Lk, H, dh, scale, False, p)
    R = torch.randn_like(o.float())
    (o.float() * R).sum().backward()
    q2, k2, v2 = (t.detach().float().cpu().double().requires_grad_(True) for t in (q, k, v))
    qh = q2.view(B, Lq, H, dh).transpose(1, 2)
    kh = k2.view(B, Lk, H, dh).transpose(1, 2)
    vh = v2.view(B, Lk, H, dh).transpose(1, 2)
    sc = qh @ kh.transpose(-1, -2) * scale + am.cpu().double()
    sc = sc.masked_fill(kpm.cpu().bool()[:, None, None, :], float("-inf"))
    P = sc.softmax(-1)
    keep = (attn.detach().cpu() != 0).double()
    Pd = P * keep / (1 - p)
    tol = 1e-5 if dtype == torch.float32 else 1e-4
    _close(attn, Pd, tol, "dropped weights")
    o2 = (Pd @ vh).transpose(1, 2).reshape(B * Lq, H * dh)
    otol = 1e-5 if dtype == torch.float32 else 1e-2  # bf16 output rounding
    _close(o, o2, otol, "out")
    (o2 * R.cpu().double()).sum().backward()
    _close(q.grad, q2.grad, 2e-5 if dtype == torch.float32 else 2e-2, "dq")
    _close(k.grad, k2.grad, 2e-5 if dtype == torch.float32 else 2e-2, "dk")
    _close(v.grad, v2.grad, 2e-5 if dtype == torch.float32 else 2e-2, "dv")
