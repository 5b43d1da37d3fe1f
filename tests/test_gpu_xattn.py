"""RelPosMHAXL with query != key/value and q_len != k_len on the GPU
(csrc/xattn.hip through the drop-in module) against reference-generated
fixtures (tests/golden/xattn.npz, gen_golden.gen_xattn): the 16 combinations
of the reference's own tests/unittests/test_attention.py:4-27 plus causal
(mask_pos_future), key padding, bool / float attn_mask and key != value
cases — outputs, attention maps and every gradient at 1e-4."""
import math

import pytest
import torch

from conftest import assert_close
import oracle.conformer as OC

pytestmark = pytest.mark.gpu


def _case(g, t, dev):
    E, H, vbias, ql, kl, same_kv, mpf, has_kpm, am_kind = (int(x) for x in g[f"{t}.meta"])
    from speechbrain_amd.nnet.attention import RelPosMHAXL
    m = RelPosMHAXL(E, num_heads=H, vbias=bool(vbias), mask_pos_future=bool(mpf))
    pre = f"{t}.sd."
    m.load_state_dict({k[len(pre):]: torch.from_numpy(g[k]) for k in g.files if k.startswith(pre)}, strict=True)
    m = m.to(dev)
    q = torch.from_numpy(g[f"{t}.q"]).to(dev).requires_grad_(True)
    k = torch.from_numpy(g[f"{t}.k"]).to(dev).requires_grad_(True)
    v = k if same_kv else torch.from_numpy(g[f"{t}.v"]).to(dev).requires_grad_(True)
    kpm = torch.from_numpy(g[f"{t}.kpm"]).to(dev) if has_kpm else None
    am = torch.from_numpy(g[f"{t}.am"]).to(dev) if am_kind else None
    return m, q, k, v, torch.from_numpy(g[f"{t}.pe"]).to(dev), kpm, am, bool(same_kv)


def test_relpos_cross_attention_vs_reference(golden, dev):
    g = golden("xattn")
    for t in g["cases"]:
        m, q, k, v, pe, kpm, am, same_kv = _case(g, t, dev)
        o, a = m(q, k, v, pos_embs=pe, key_padding_mask=kpm, attn_mask=am)
        assert_close(o, g[f"{t}.out"], name=f"{t} out")
        assert_close(a, g[f"{t}.attn"], name=f"{t} attn")
        (o * torch.from_numpy(g[f"{t}.R"]).to(dev)).sum().backward()
        assert_close(q.grad, g[f"{t}.grad_q"], name=f"{t} grad_q")
        assert_close(k.grad, g[f"{t}.grad_k"], name=f"{t} grad_k")
        if not same_kv:
            assert_close(v.grad, g[f"{t}.grad_v"], name=f"{t} grad_v")
        for name, p in m.named_parameters():
            assert_close(p.grad, g[f"{t}.grad.{name}"], name=f"{t} grad {name}")


def test_reference_unit_test_runs(dev):
    """tests/unittests/test_attention.py:4-27 verbatim in behaviour: every
    combination constructs and runs (grad mode, random inputs)."""
    from speechbrain_amd.nnet.attention import RelPosMHAXL
    for kl in (12, 10):
        for ql in (10, 12):
            for b in (True, False):
                for h in (4, None):
                    relpos = RelPosMHAXL(4, num_heads=2, vbias=b, vdim=h).to(dev)
                    q = torch.rand((2, ql, 4), device=dev)
                    k = torch.rand((2, kl, 4), device=dev)
                    pos_embs = torch.rand((1, 2 * kl - 1, 4), device=dev)
                    o, a = relpos(q, k, k, pos_embs=pos_embs)
                    assert o.shape == (2, ql, 4) and a.shape == (2, 2, ql, kl)
                    assert torch.isfinite(o).all()


def test_relpos_cross_attention_bf16_and_no_grad(golden, dev):
    """bf16 autocast (bf16 operands, fp32 softmax) and the no-grad call:
    within the bf16 rounding of the fixture (case c1: 4 heads of 16)."""
    g = golden("xattn")
    m, q, k, v, pe, kpm, am, _ = _case(g, "c1", dev)
    with torch.no_grad():
        o32, a32 = m(q, k, v, pos_embs=pe, key_padding_mask=kpm, attn_mask=am)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            o16, a16 = m(q, k, v, pos_embs=pe, key_padding_mask=kpm, attn_mask=am)
    assert_close(o32, g["c1.out"], name="no-grad out")
    assert_close(a32, g["c1.attn"], name="no-grad attn")
    assert float((o16.float().cpu() - torch.from_numpy(g["c1.out"])).abs().max()) < 3e-2
    assert float((a16.float().cpu() - torch.from_numpy(g["c1.attn"])).abs().max()) < 1e-2


def test_relpos_cross_attention_dropout(dev):
    """Training mode with attention dropout: the returned weights are the
    dropped probabilities, out = out_proj(attn · V), and the gradients equal
    autograd of the oracle restatement under the same keep mask."""
    from speechbrain_amd.nnet.attention import RelPosMHAXL
    torch.manual_seed(5)
    E, H, Lq, Lk, B, p = 32, 2, 13, 9, 2, 0.3
    m = RelPosMHAXL(E, num_heads=H, dropout=p, vbias=True, mask_pos_future=True).to(dev).train()
    with torch.no_grad():
        m.value_bias_weight.normal_()
    q = torch.randn(B, Lq, E, device=dev, requires_grad=True)
    k = torch.randn(B, Lk, E, device=dev, requires_grad=True)
    pe = torch.randn(1, 2 * Lk - 1, E, device=dev)
    o, attn = m(q, k, k, pos_embs=pe)
    R = torch.randn_like(o)
    (o * R).sum().backward()
    # oracle with the same keep mask (recovered from the dropped weights)
    sd = {kk: vv.detach().cpu().double().requires_grad_(True) for kk, vv in m.state_dict().items()}
    q2 = q.detach().cpu().double().requires_grad_(True)
    k2 = k.detach().cpu().double().requires_grad_(True)
    _, P = OC.rel_pos_mha_cross(q2, k2, k2, pe.cpu().double(), sd, "", H, True, True)
    keep = (attn.detach().cpu() != 0).double()
    Pd = P * keep / (1 - p)
    assert_close(attn, Pd, name="dropped weights")
    dh = E // H
    wq, wk, wv = sd["in_proj_weight"].chunk(3, dim=0)
    vv = (torch.nn.functional.linear(k2, wv) + sd["value_bias_weight"]).view(B, Lk, H, dh).transpose(1, 2)
    ctx = (Pd @ vv).transpose(1, 2).reshape(B, Lq, E)
    o2 = torch.nn.functional.linear(ctx, sd["out_proj.weight"], sd["out_proj.bias"])
    assert_close(o, o2, name="out")
    (o2 * R.cpu().double()).sum().backward()
    assert_close(q.grad, q2.grad, name="grad q")
    assert_close(k.grad, k2.grad, name="grad k")
    for name, prm in m.named_parameters():
        assert_close(prm.grad, sd[name].grad, name=f"grad {name}")
