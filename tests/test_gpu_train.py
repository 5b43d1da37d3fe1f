"""Training path: backward kernels of
csrc/backward.hip and the differentiable module chain (_autograd) vs the
reference's own autograd (tests/golden/train.npz) and vs torch autograd of
the same op on CPU.

Tolerances: fp32 gradients within 1e-4 of the largest reference gradient of
the tensor (|a-b| <= 1e-4 * max|b|) — the backward sums differ from the
reference's only in fp32 summation order.  bf16 (autocast) gradients are
bounded per tensor by a derived tolerance: the same oracle run under
torch.autocast("cpu", bfloat16) (every matmul / conv operand rounded to
bf16 — what a bf16 MFMA implementation cannot avoid) deviates from the fp32
oracle by e_emu (normwise, per tensor); the HIP bf16 gradient must stay
within 1.0 x e_emu of the fp32 oracle."""
import math

import numpy as np
import pytest
import torch
import torch.nn.functional as F

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


def nrel(a, b):
    """normwise relative error ||a - b|| / ||b|| (float64)."""
    a, b = a.detach().double().flatten().cpu(), b.detach().double().flatten().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-300)).item()


def check_emu_bound(rows, factor=1.0):
    """rows: (name, e_hip, e_emu); every HIP bf16 error within factor x the
    bf16-operand oracle's (the worst ratios printed)."""
    for name, eh, ee in sorted(rows, key=lambda r: -r[1] / max(r[2], 1e-30))[:8]:
        print(f"{name}: HIP bf16 {eh:.3e}  bf16-operand oracle {ee:.3e}  ratio {eh / max(ee, 1e-30):.2f}")
    bad = [(n, eh, ee) for n, eh, ee in rows if not eh <= factor * ee]
    assert not bad, f"{len(bad)} gradients beyond {factor} x e_emu: {bad[:4]}"


def cosine(a, b):
    a, b = a.detach().float().flatten().cpu(), b.detach().float().flatten().cpu()
    return (a @ b / (a.norm() * b.norm() + 1e-30)).item()


# ----------------------------------------------------------------- kernels
def test_dropout_add(dev):
    from speechbrain_amd import _autograd as A
    x = torch.randn(2000, 513, device=dev)
    x[x == 0] = 1.0  # randn yields exact zeros (~2^-24 per value): they would read as dropped
    res = torch.randn(2000, 513, device=dev)
    y0 = A.drop_add(x, res, 0.5, None, 0.0, 0)
    assert_close(y0, res + 0.5 * x, rtol=1e-6, name="p=0")
    y = A.drop_add(x, None, 1.0, None, 0.1, 1234)
    kept = y != 0
    frac = 1 - kept.float().mean().item()
    assert abs(frac - 0.1) < 0.005, frac
    assert_close(y[kept], x[kept] / 0.9, rtol=1e-6, name="scale")
    # same seed -> same mask (the backward regenerates it); different seed -> different mask
    y2 = A.drop_add(torch.ones_like(x), None, 1.0, None, 0.1, 1234)
    assert torch.equal(y2 != 0, kept)
    y3 = A.drop_add(torch.ones_like(x), None, 1.0, None, 0.1, 99)
    assert not torch.equal(y3 != 0, kept)
    mask = (torch.arange(2000, device=dev) % 3 == 0).to(torch.uint8)
    y4 = A.drop_add(x, res, 2.0, mask, 0.0, 0, torch.bfloat16)
    ref = res + 2 * x
    ref[mask.bool()] = res[mask.bool()]
    assert_close(y4.float(), ref, rtol=1e-2, name="rowmask bf16")


def test_dropout_add_vec4_matches_scalar(dev):
    """The 4-wide kernel (aligned, cols % 4 == 0) keeps the same per-element
    mask and values as the per-element kernel (forced by a misaligned view)."""
    from speechbrain_amd import _autograd as A
    base = torch.randn(2000 * 512 + 1, device=dev)
    res = torch.randn(2000, 512, device=dev)
    mask = (torch.arange(2000, device=dev) % 5 == 0).to(torch.uint8)
    xa = base[:-1].view(2000, 512).clone()          # aligned -> dropout_add4
    xs = base[1:].view(2000, 512)                   # 4-byte offset -> per-element kernel
    xs.copy_(xa)
    for dt in (torch.float32, torch.bfloat16):
        ya = A.drop_add(xa, res, 0.7, mask, 0.15, 4321, dt)
        ys = A.drop_add(xs, res, 0.7, mask, 0.15, 4321, dt)
        assert torch.equal(ya, ys), dt


def test_rowsum_batched(dev):
    from speechbrain_amd import _autograd as A
    g = torch.Generator().manual_seed(5)
    x = torch.randn(4, 3001, 72, generator=g)
    # fp32 sums in a different order: bound by 1e-6 of sum |x| (float64 reference)
    tol = 1e-6 * x.abs().sum(1).max().item()
    out = A.rowsum_batched(x.to(dev))
    assert (out.cpu().double() - x.double().sum(1)).abs().max().item() <= tol
    xb = x.to(torch.bfloat16)
    assert (A.rowsum_batched(xb.to(dev)).cpu().double() - xb.double().sum(1)).abs().max().item() <= tol
    assert (A.rowsum(x[0].to(dev)).cpu().double() - x[0].double().sum(0)).abs().max().item() <= tol


def test_dropout_autograd(dev):
    from speechbrain_amd import _autograd as A
    torch.manual_seed(0)
    x = torch.randn(300, 64, device=dev, requires_grad=True)
    res = torch.randn(300, 64, device=dev, requires_grad=True)
    y = A.DropAddFn.apply(x, res, 0.5, None, 0.2, torch.float32)
    g = torch.randn_like(y)
    y.backward(g)
    keep = ((y - res).detach() != 0)
    assert_close(x.grad, torch.where(keep, g * 0.5 / 0.8, torch.zeros_like(g)), rtol=1e-6, name="dx")
    assert_close(res.grad, g, rtol=0, name="dres")


@pytest.mark.parametrize("D", [64, 256, 640, 2560])
@pytest.mark.parametrize("dy_bf16", [False, True])
def test_layernorm_bwd(dev, D, dy_bf16):
    from speechbrain_amd import _autograd as A
    g = torch.Generator().manual_seed(D)
    M = 1003
    x = torch.randn(M, D, generator=g) * 2 + 0.3
    ln = torch.nn.LayerNorm(D)
    with torch.no_grad():
        ln.weight.copy_(1 + 0.2 * torch.randn(D, generator=g))
        ln.bias.copy_(0.1 * torch.randn(D, generator=g))
    dy = torch.randn(M, D, generator=g)
    if dy_bf16:
        dy = dy.to(torch.bfloat16).float()
    xr = x.clone().requires_grad_(True)
    F.layer_norm(xr, (D,), ln.weight, ln.bias, 1e-5).backward(dy)
    lnd = torch.nn.LayerNorm(D).to(dev)
    lnd.load_state_dict(ln.state_dict())
    xd = x.to(dev).requires_grad_(True)
    y = A.layer_norm(xd, lnd)
    assert_close(y, F.layer_norm(x, (D,), ln.weight, ln.bias, 1e-5).detach(), rtol=1e-5, name="fwd")
    y.backward(dy.to(dev).to(torch.bfloat16) if dy_bf16 else dy.to(dev))
    assert_grad(xd.grad, xr.grad, name="dx")
    assert_grad(lnd.weight.grad, ln.weight.grad, name="dgamma")
    assert_grad(lnd.bias.grad, ln.bias.grad, name="dbeta")


@pytest.mark.parametrize("D", [10240, 16384])  # the default 80-mel front-end's (F·C) rows; the kernels' limit
@pytest.mark.parametrize("with_dres", [False, True])
def test_layernorm_wide_rows(dev, D, with_dres):
    """Workgroup-per-row LayerNorm kernels (D > 2560: ln_fwd_row_kernel /
    ln_bwd_row_kernel) through the C ABI, incl. the residual-gradient input
    dres (dx = LN backward + dres, ConvBlockFn's use), against torch autograd."""
    from speechbrain_amd._lib import lib, ptr, stream_of
    g = torch.Generator().manual_seed(D + with_dres)
    M = 37
    x = torch.randn(M, D, generator=g) * 2 + 0.3
    w = 1 + 0.2 * torch.randn(D, generator=g)
    b = 0.1 * torch.randn(D, generator=g)
    dy = torch.randn(M, D, generator=g)
    dres = torch.randn(M, D, generator=g)
    xr, wr, br = (t.clone().requires_grad_(True) for t in (x, w, b))
    yr = F.layer_norm(xr, (D,), wr, br, 1e-5)
    yr.backward(dy)
    xd, wd, bd, dyd, dresd = (t.to(dev) for t in (x, w, b, dy, dres))
    y = torch.empty(M, D, device=dev)
    L = lib()
    assert L.sbk_layernorm_wide(ptr(xd), M, D, ptr(wd), ptr(bd), 1e-5, ptr(y), 0, stream_of(xd)) == 0
    assert_close(y, yr.detach(), rtol=1e-5, name="fwd")
    nblk = int(L.sbk_layernorm_bwd_blocks(M))
    part = torch.empty(nblk * 2 * D, device=dev)
    dx = torch.empty(M, D, device=dev)
    assert L.sbk_layernorm_bwd(ptr(xd), ptr(dyd), 0, M, D, ptr(wd), 1e-5, ptr(dresd) if with_dres else None, ptr(dx),
                               ptr(part), stream_of(xd)) == 0
    gb = part.view(nblk, 2 * D).sum(0)
    assert_grad(dx, xr.grad + (dres if with_dres else 0), name="dx")
    assert_grad(gb[:D], wr.grad, name="dgamma")
    assert_grad(gb[D:], br.grad, name="dbeta")


@pytest.mark.parametrize("cols", [96, 98])  # 4-wide kernels / per-element kernels (GLU halves 49)
@pytest.mark.parametrize("name", ["swish", "glu", "leaky_relu"])
def test_act_bwd(dev, name, cols):
    from speechbrain_amd import _autograd as A
    g = torch.Generator().manual_seed(3)
    x = torch.randn(777, cols, generator=g) * 3
    xr = x.clone().requires_grad_(True)
    ref = {"swish": lambda t: t * torch.sigmoid(t), "glu": lambda t: F.glu(t, dim=-1),
           "leaky_relu": lambda t: F.leaky_relu(t, 0.01)}[name](xr)
    dy = torch.randn(ref.shape, generator=g)
    ref.backward(dy)
    xd = x.to(dev).requires_grad_(True)
    y = A.act(xd, name, 0.01)
    assert_close(y, ref.detach(), rtol=1e-5, name="fwd")
    y.backward(dy.to(dev))
    assert_grad(xd.grad, xr.grad, rtol=1e-5, name="dx")


@pytest.mark.parametrize("K,causal", [(31, False), (7, True), (3, False)])
def test_dwconv_fwd_bwd(dev, K, causal):
    from speechbrain_amd import _autograd as A
    g = torch.Generator().manual_seed(K)
    B, T, C = 3, 77, 64
    x = torch.randn(B, T, C, generator=g)
    w = torch.randn(C, 1, K, generator=g) / math.sqrt(K)
    b = torch.randn(C, generator=g)
    xr, wr, br = (t.clone().requires_grad_(True) for t in (x, w, b))
    pad = K - 1 if causal else (K - 1) // 2
    ref = F.conv1d(xr.transpose(1, 2), wr, br, padding=pad, groups=C)
    if causal:
        ref = ref[..., :-pad]
    ref = ref.transpose(1, 2)
    dy = torch.randn(ref.shape, generator=g)
    ref.backward(dy)
    xd, wd, bd = (t.to(dev).requires_grad_(True) for t in (x, w, b))
    y = A.DwConvFn.apply(xd.reshape(B * T, C), wd, bd, B, T, causal)
    assert_close(y.view(B, T, C), ref.detach(), rtol=1e-5, name="fwd")
    y.backward(dy.to(dev).reshape(B * T, C))
    assert_grad(xd.grad, xr.grad, name="dx")
    assert_grad(wd.grad, wr.grad, name="dw")
    assert_grad(bd.grad, br.grad, name="db")


@pytest.mark.parametrize("Ti,Fi,Ci,Co", [(101, 80, 1, 64), (51, 40, 64, 32), (3, 3, 8, 16), (8, 5, 16, 16)])
def test_conv_block_fn_vs_oracle(dev, Ti, Fi, Ci, Co):
    """im2col (reflect pad) + MFMA GEMM + (freq x chan) LayerNorm + LeakyReLU
    and its backward (col2im) vs autograd of the oracle ConvBlock."""
    from speechbrain_amd import _autograd as A
    g = torch.Generator().manual_seed(Ti * Ci)
    B = 2
    x = torch.randn(B, Ti, Fi, Ci, generator=g)
    w = torch.randn(Co, Ci, 3, 3, generator=g) / math.sqrt(9 * Ci)
    b = 0.1 * torch.randn(Co, generator=g)
    To, Fo = (Ti - 1) // 2 + 1, (Fi - 1) // 2 + 1
    lw = 1 + 0.1 * torch.randn(Fo, Co, generator=g)
    lb = 0.1 * torch.randn(Fo, Co, generator=g)
    leaves = [t.clone().requires_grad_(True) for t in (x, w, b, lw, lb)]
    sd = {"conv_0.conv.weight": leaves[1], "conv_0.conv.bias": leaves[2], "norm_0.norm.weight": leaves[3],
          "norm_0.norm.bias": leaves[4]}
    ref = OC.conv_block(leaves[0], sd, "")
    dy = torch.randn(ref.shape, generator=g)
    ref.backward(dy)
    dl = [t.to(dev).requires_grad_(True) for t in (x, w, b, lw, lb)]
    y = A.ConvBlockFn.apply(dl[0], dl[1], dl[2], dl[3], dl[4], 1e-5, 0.01, torch.float32, torch.float32,
                            (3, 3, 2, 2))
    assert_close(y, ref.detach(), rtol=1e-4, name="fwd")
    y.backward(dy.to(dev))
    for n, a, r in zip(("dx", "dw", "db", "dln_w", "dln_b"), dl, leaves):
        assert_grad(a.grad, r.grad, name=n)


@pytest.mark.parametrize("T,lens,d", [(37, [37, 30, 21], 64), (97, [97, 60, 5], 64), (51, [51, 40], 144)])
def test_relpos_attention_bwd_vs_oracle(dev, T, lens, d):
    """fp32 attention backward on the exact-f32 MFMA GEMMs (sbk_gemm_batched,
    sbk_gemm_tn_f32) over padded rows: T not a multiple of 8, and head size 36
    (d = 144) padded to 40."""
    from speechbrain_amd.nnet.attention import RelPosEncXL, RelPosMHAXL
    torch.manual_seed(T)
    H = 4
    mha = RelPosMHAXL(embed_dim=d, num_heads=H)
    B = len(lens)
    x = torch.randn(B, T, d)
    pe = RelPosEncXL(d)(x)
    kpm = torch.arange(T)[None] >= torch.tensor(lens)[:, None]
    sd = {k: v.clone().requires_grad_(True) for k, v in mha.state_dict().items()}
    xr = x.clone().requires_grad_(True)
    ref, ref_attn = OC.rel_pos_mha(xr, pe, sd, "", H, kpm)
    dy = torch.randn(ref.shape)
    ref.backward(dy)
    mha = mha.to(dev).train()
    xd = x.to(dev).requires_grad_(True)
    out, attn = mha(xd, xd, xd, pe.to(dev), key_padding_mask=kpm.to(dev))
    assert_close(out, ref.detach(), name="fwd")
    assert_close(attn, ref_attn.detach(), name="attn")
    out.backward(dy.to(dev))
    assert_grad(xd.grad, xr.grad, name="dx")
    for k, p in mha.named_parameters():
        assert_grad(p.grad, sd[k].grad, name=k)


def _oracle_mha_grads(x, pe, sd0, H, kpm, dy, bf16):
    sd = {k: v.clone().requires_grad_(True) for k, v in sd0.items()}
    xr = x.clone().requires_grad_(True)
    with torch.autocast("cpu", dtype=torch.bfloat16, enabled=bf16):
        out, _ = OC.rel_pos_mha(xr, pe, sd, "", H, kpm)
    out.float().backward(dy)
    return out.detach().float(), {"dx": xr.grad, **{k: v.grad for k, v in sd.items()}}


@pytest.mark.parametrize("T,lens,d", [(37, [37, 30, 21], 64), (376, [376, 300], 256), (377, [377, 290], 256),
                                      (121, [121, 99], 144)])
def test_relpos_attention_bwd_bf16_vs_oracle(dev, T, lens, d):
    """bf16 autocast attention forward + backward (own kernels: the fused
    attention kernel, sbk_gemm_batched / sbk_gemm_tn over rows padded to a
    multiple of 8, the softmax / rel_shift backward) against the fp32 oracle
    with the derived bound: per gradient, error <= 1.0 x that of the oracle run
    on bf16 operands.  T = 37, 377, 121 are not multiples of 8; d = 144 has
    head size 36 (padded to 40)."""
    from speechbrain_amd.nnet.attention import RelPosEncXL, RelPosMHAXL
    torch.manual_seed(T + d)
    H = 4
    mha = RelPosMHAXL(embed_dim=d, num_heads=H)
    B = len(lens)
    x = torch.randn(B, T, d)
    pe = RelPosEncXL(d)(x)
    kpm = torch.arange(T)[None] >= torch.tensor(lens)[:, None]
    dy = torch.randn(B, T, d)
    sd0 = {k: v.clone() for k, v in mha.state_dict().items()}
    ref_out, ref = _oracle_mha_grads(x, pe, sd0, H, kpm, dy, False)
    emu_out, emu = _oracle_mha_grads(x, pe, sd0, H, kpm, dy, True)
    mha = mha.to(dev).train()
    xd = x.to(dev).requires_grad_(True)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        out, _ = mha(xd, xd, xd, pe.to(dev), key_padding_mask=kpm.to(dev))
    out.float().backward(dy.to(dev))
    hip = {"dx": xd.grad, **{k: p.grad for k, p in mha.named_parameters()}}
    rows = [("out", nrel(out, ref_out), nrel(emu_out, ref_out))]
    rows += [(k, nrel(hip[k], ref[k]), nrel(emu[k], ref[k])) for k in ref if ref[k] is not None]
    assert len(rows) == 8  # out, dx and the six parameters
    check_emu_bound(rows)


def _core_ref(qkv, pk, pbu, pbv, kpm, B, T, H, dh, scale, D):
    """RelPosMHAXL core (attention.py:581-633) in float64 with a given
    dropout scale D (B, H, T, T) on the probabilities."""
    q5 = qkv.view(B, T, H, 3, dh)
    q, k, v = q5[:, :, :, 0], q5[:, :, :, 1], q5[:, :, :, 2]
    u, vb = pbu.reshape(H, dh), pbv.reshape(H, dh)
    ac = torch.einsum("bihd,bjhd->bhij", q + u, k)
    bd = torch.einsum("bihd,whd->bhiw", q + vb, pk.view(2 * T - 1, H, dh))
    bd = OC.rel_shift(bd)
    score = ((ac + bd) * scale).masked_fill(kpm.view(B, 1, 1, T), -float("inf"))
    attn = torch.softmax(score, -1) * D
    return torch.einsum("bhij,bjhd->bihd", attn, v).reshape(B * T, H * dh), attn


@pytest.mark.parametrize("T", [45, 64])
def test_relpos_attention_dropout_fwd_bwd(dev, T):
    """Attention dropout (attention.py:626) on the HIP path: the forward's
    drop(P)·V (sbk_attn_probs_pad + sbk_gemm_batched writing the head-merged
    layout) and the backward's regenerated mask (sbk_relpos_softmax_bwd_pad),
    fp32, against float64 autograd of the same algebra with the kernel's own
    mask (read off the returned weights: kept = nonzero, scale 1/(1-p))."""
    from speechbrain_amd import _autograd as A
    B, H, dh, p = 2, 4, 16, 0.2
    d = H * dh
    g = torch.Generator().manual_seed(T)
    qkv = torch.randn(B * T, 3 * d, generator=g)
    pk = torch.randn(2 * T - 1, d, generator=g)
    pbu, pbv = 0.3 * torch.randn(dh, H, generator=g), 0.3 * torch.randn(dh, H, generator=g)
    kpm = torch.arange(T)[None] >= torch.tensor([T, T - 9])[:, None]
    scale = 1 / math.sqrt(d)
    leaves = [t.to(dev).requires_grad_(True) for t in (qkv, pk, pbu, pbv)]
    torch.manual_seed(3)
    o, attn = A.RelPosAttentionFn.apply(*leaves, kpm.to(dev).to(torch.uint8), B, T, H, dh, scale, p, None)
    do = torch.randn(o.shape, generator=g)
    o.backward(do.to(dev))
    attn = attn.cpu().double()
    kept = attn != 0
    frac = 1 - kept[..., : T - 9].double().mean().item()
    assert abs(frac - p) < 0.03, frac
    D = kept.double() / (1 - p)
    rl = [t.double().requires_grad_(True) for t in (qkv, pk, pbu, pbv)]
    ro, rattn = _core_ref(*rl, kpm, B, T, H, dh, scale, D)
    assert_close(attn, rattn.detach(), rtol=1e-5, name="attn")
    assert_close(o, ro.detach(), rtol=1e-4, name="o")
    ro.backward(do.double())
    for n, a, r in zip(("dqkv", "dpk", "dpbu", "dpbv"), leaves, rl):
        assert_grad(a.grad, r.grad, name=n)
    # same seed, bf16: the same mask
    torch.manual_seed(3)
    _, attn_b = A.RelPosAttentionFn.apply(qkv.to(dev).bfloat16(), pk.to(dev).bfloat16(), pbu.to(dev), pbv.to(dev),
                                          kpm.to(dev).to(torch.uint8), B, T, H, dh, scale, p, None)
    assert torch.equal(attn_b.cpu() != 0, attn != 0)


@pytest.mark.parametrize("act", [0, 3, 5, 6])
@pytest.mark.parametrize("J", [130, 131, 1024])
@pytest.mark.parametrize("z_bf16", [False, True])
def test_joint_fwd_bwd(dev, act, J, z_bf16):
    """Vector (J % 4 == 0 / J % 2 == 0) and scalar paths; 37 frames = two
    16-frame runs + a ragged one; bf16 z / dz: the reference is fed the same
    bf16-rounded dz and compared at bf16 resolution for z."""
    from speechbrain_amd import _autograd as A
    g = torch.Generator().manual_seed(act + J)
    B, T, U1 = 2, 37, 5
    tn = torch.randn(B, T, J, generator=g)
    pn = torch.randn(B, U1, J, generator=g)
    tr, pr = tn.clone().requires_grad_(True), pn.clone().requires_grad_(True)
    z = tr.unsqueeze(2) + pr.unsqueeze(1)
    z = {0: lambda t: t, 3: lambda t: F.leaky_relu(t, 0.01), 5: torch.tanh, 6: F.relu}[act](z)
    dz = torch.randn(z.shape, generator=g)
    zdt = torch.bfloat16 if z_bf16 else torch.float32
    dz = dz.to(zdt).float()
    z.backward(dz)
    td, pd = tn.to(dev).requires_grad_(True), pn.to(dev).requires_grad_(True)
    y = A.JointFn.apply(td, pd, act, 0.01, zdt)
    assert y.dtype == zdt
    assert_close(y.float(), z.detach(), rtol=1e-5 if not z_bf16 else 8e-3, name="fwd")
    y.backward(dz.to(dev).to(zdt))
    assert_grad(td.grad, tr.grad, rtol=1e-5, name="dtn")
    assert_grad(pd.grad, pr.grad, rtol=1e-5, name="dpn")


# ------------------------------------------------------------- whole encoder
def _modules(golden, dev, dropout=0.0):
    from speechbrain_amd.lobes.models.convolution import ConvolutionFrontEnd
    from speechbrain_amd.lobes.models.transformer.TransformerASR import TransformerASR
    g = golden("conformer")
    cnn = ConvolutionFrontEnd(input_shape=(8, 10, 80), num_blocks=2, num_layers_per_block=1, out_channels=(64, 32),
                              kernel_sizes=(3, 3), strides=(2, 2), residuals=(False, False), dropout=dropout)
    tr = TransformerASR(tgt_vocab=10, input_size=640, d_model=64, nhead=4, num_encoder_layers=2,
                        num_decoder_layers=0, d_ffn=128, dropout=dropout, encoder_module="conformer",
                        attention_type="RelPosMHAXL", normalize_before=True, causal=False)
    for pre, m in (("cnn.", cnn), ("tr.", tr)):
        m.load_state_dict({k[len(pre):]: torch.from_numpy(g[k]) for k in g.files if k.startswith(pre)}, strict=True)
    return cnn.to(dev).train(), tr.to(dev).train(), g


def test_encoder_grads_vs_reference(golden, dev):
    """fp32 training path: every parameter gradient and the feature gradient
    of sum(R * encode(cnn(feats))) vs the reference's autograd (train.npz)."""
    cnn, tr, g = _modules(golden, dev)
    gt = golden("train")
    feats = torch.from_numpy(g["feats"]).to(dev).requires_grad_(True)
    y = tr.encode(cnn(feats), torch.from_numpy(g["wav_len"]).to(dev))
    assert_close(y, gt["y"], name="y")
    (y * torch.from_numpy(gt["R"]).to(dev)).sum().backward()
    assert_grad(feats.grad, gt["grad_feats"], name="feats")
    n = 0
    for pre, m in (("cnn.", cnn), ("tr.", tr)):
        for k, p in m.named_parameters():
            key = "grad." + pre + k
            if key in gt.files:
                assert p.grad is not None, key
                assert_grad(p.grad, gt[key], name=key)
                n += 1
            else:
                assert p.grad is None or not p.grad.any(), key
    assert n == sum(1 for k in gt.files if k.startswith("grad."))


def _oracle_encoder_grads(feats, wav_len, cnn, tr, R, layers, heads, bf16):
    """Autograd of the oracle's ConvolutionFrontEnd + TransformerASR.encode
    (fp32, or under torch.autocast("cpu", bfloat16)) on the modules'
    weights: {parameter name: gradient}."""
    import os
    torch.set_num_threads(max(1, min(16, os.cpu_count() or 1)))
    sd_c = {k: v.detach().cpu().clone().requires_grad_(True) for k, v in cnn.state_dict().items()}
    sd_t = {k: v.detach().cpu().clone().requires_grad_(v.is_floating_point()) for k, v in tr.state_dict().items()}
    with torch.autocast("cpu", dtype=torch.bfloat16, enabled=bf16):
        yr = OC.transformer_asr_encode(OC.conv_frontend(feats.detach().cpu(), sd_c), sd_t, "", layers, heads,
                                       wav_len.cpu())
    (yr.float() * R).sum().backward()
    out = {"cnn." + k: v.grad for k, v in sd_c.items() if v.grad is not None}
    out.update({"tr." + k: v.grad for k, v in sd_t.items() if v.requires_grad and v.grad is not None})
    return out


def _emu_rows(cnn, tr, ref, emu):
    rows = []
    for pre, m in (("cnn.", cnn), ("tr.", tr)):
        for k, p in m.named_parameters():
            if pre + k not in ref:
                continue
            assert p.grad is not None, f"{k}: no gradient on the HIP path"
            rows.append((pre + k, nrel(p.grad, ref[pre + k]), nrel(emu[pre + k], ref[pre + k])))
    return rows


def test_encoder_grads_bf16_autocast(golden, dev):
    """bf16 operands (autocast): every parameter gradient of sum(R * encode(
    cnn(feats))) within 1.0 x the bf16-operand oracle's deviation from the
    fp32 oracle (which matches the reference's autograd, train.npz, to 1e-5).
    The model is small (d = 64, 2 layers), so a single projection R gives a
    noisy per-tensor error: errors are pooled over three projections (the
    fixture's R and two seeded ones), sqrt(sum ||a - b||^2 / sum ||b||^2),
    for the HIP path and the emulation alike."""
    cnn, tr, g = _modules(golden, dev)
    gt = golden("train")
    feats = torch.from_numpy(g["feats"])
    wl = torch.from_numpy(g["wav_len"])
    Rs = [torch.from_numpy(gt["R"])]
    Rs += [torch.randn(Rs[0].shape, generator=torch.Generator().manual_seed(s)) for s in (1, 2)]
    acc = {}
    for i, R in enumerate(Rs):
        for m in (cnn, tr):
            m.zero_grad(set_to_none=True)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            y = tr.encode(cnn(feats.to(dev)), wl.to(dev))
        assert y.dtype == torch.float32
        (y * R.to(dev)).sum().backward()
        ref = _oracle_encoder_grads(feats, wl, cnn, tr, R, 2, 4, False)
        if i == 0:
            assert sorted("grad." + k for k in ref) == sorted(k for k in gt.files if k.startswith("grad."))
            for key, v in ref.items():  # the oracle is the reference's autograd
                assert_grad(v, gt["grad." + key], rtol=1e-4, name=key)
        emu = _oracle_encoder_grads(feats, wl, cnn, tr, R, 2, 4, True)
        for pre, m in (("cnn.", cnn), ("tr.", tr)):
            for k, p in m.named_parameters():
                if pre + k not in ref:
                    continue
                assert p.grad is not None, f"{k}: no gradient on the HIP path"
                r = ref[pre + k].double()
                a = acc.setdefault(pre + k, [0.0, 0.0, 0.0])
                a[0] += (p.grad.detach().cpu().double() - r).norm().item() ** 2
                a[1] += (emu[pre + k].double() - r).norm().item() ** 2
                a[2] += r.norm().item() ** 2
    rows = [(k, (a[0] / a[2]) ** 0.5, (a[1] / a[2]) ** 0.5) for k, a in acc.items()]
    assert len(rows) == sum(1 for k in gt.files if k.startswith("grad."))
    check_emu_bound(rows)


def test_encoder_train_dropout(golden, dev):
    """Training mode with dropout 0.1 (recipe value): stochastic, finite, and
    identical for identical seeds; eval mode is deterministic and dropout-free."""
    cnn, tr, g = _modules(golden, dev, dropout=0.1)
    feats = torch.from_numpy(g["feats"]).to(dev)
    wl = torch.from_numpy(g["wav_len"]).to(dev)
    torch.manual_seed(5)
    y1 = tr.encode(cnn(feats), wl)
    y1.sum().backward()
    torch.manual_seed(5)
    y2 = tr.encode(cnn(feats), wl)
    y3 = tr.encode(cnn(feats), wl)
    assert torch.isfinite(y1).all()
    assert torch.equal(y1, y2)
    assert not torch.equal(y1, y3)
    assert all(torch.isfinite(p.grad).all() for p in tr.parameters() if p.grad is not None)
    cnn.eval()
    tr.eval()
    with torch.no_grad():
        ye = tr.encode(cnn(feats), wl)
    assert_close(ye, golden("train")["y"], name="eval")


@pytest.mark.parametrize("bf16", [False, True])
def test_full_size_encoder_grads_vs_oracle(dev, bf16):
    """Config-4 encoder at full size (ConvolutionFrontEnd(64, 32) + 12-layer
    Conformer, d = 256, 2 x 15 s, one utterance at 80 % length, dropout off):
    every parameter gradient of the HIP training path against autograd of the
    fp32 oracle on the same weights and features (TransformerASR.py:279-316,
    Conformer.py:157-383 backward).  fp32: relative L2 error <= 2e-3 per tensor
    (measured on MI355X: <= 1.5e-4 for every encoder parameter, <= 8.7e-4 for
    the ConvBlock parameters, whose gradients sum ~60k cancelling
    position terms per weight) — every contraction on the exact-f32 MFMA
    kernels (sbk_gemm, sbk_gemm_tn_f32, sbk_gemm_batched), no library GEMM;
    bf16 autocast: per tensor within 1.0 x the deviation of the oracle run
    on bf16 operands (check_emu_bound)."""
    from speechbrain_amd.lobes.features import Fbank
    from speechbrain_amd.lobes.models.convolution import ConvolutionFrontEnd
    from speechbrain_amd.lobes.models.transformer.TransformerASR import TransformerASR
    torch.manual_seed(0)
    cnn = ConvolutionFrontEnd(input_shape=(8, 10, 80), num_blocks=2, num_layers_per_block=1, out_channels=(64, 32),
                              kernel_sizes=(3, 3), strides=(2, 2), residuals=(False, False)).to(dev).train()
    tr = TransformerASR(tgt_vocab=100, input_size=640, d_model=256, nhead=4, num_encoder_layers=12,
                        num_decoder_layers=0, d_ffn=1024, dropout=0.0, encoder_module="conformer",
                        attention_type="RelPosMHAXL", normalize_before=True, causal=False).to(dev).train()
    for mod in list(cnn.modules()) + list(tr.modules()):
        if isinstance(mod, torch.nn.Dropout):
            mod.p = 0.0
    g = torch.Generator().manual_seed(11)
    wav = 0.1 * torch.randn(2, 240000, generator=g)
    lens = torch.tensor([1.0, 0.8])
    feats = Fbank(n_mels=80)(wav.to(dev)).detach()
    with torch.autocast("cuda", dtype=torch.bfloat16, enabled=bf16):
        y = tr.encode(cnn(feats), lens.to(dev))
    R = torch.randn(y.shape, generator=torch.Generator().manual_seed(7))
    (y.float() * R.to(dev)).sum().backward()
    ref = _oracle_encoder_grads(feats, lens, cnn, tr, R, 12, 4, False)
    if bf16:
        emu = _oracle_encoder_grads(feats, lens, cnn, tr, R, 12, 4, True)
        rows = _emu_rows(cnn, tr, ref, emu)
        assert len(rows) > 12 * 20
        check_emu_bound(rows)
        return
    rows = []
    for pre, mod in (("cnn.", cnn), ("tr.", tr)):
        for k, p in mod.named_parameters():
            ref_g = ref.get(pre + k)
            if ref_g is None:
                continue
            assert p.grad is not None, f"{k}: no gradient on the HIP path"
            a, b = p.grad.detach().float().cpu(), ref_g.float()
            rel = (a - b).abs().max().item() / max(b.abs().max().item(), 1e-12)
            rows.append((k, rel, nrel(a, b)))
    assert len(rows) > 12 * 20
    for k, rel, l2 in sorted(rows, key=lambda r: -r[2])[:8]:
        print(f"{k}: max-norm rel {rel:.2e}, l2 rel {l2:.2e}")
    worst = max(rows, key=lambda r: r[2])
    assert worst[2] <= 2e-3, f"{worst[0]}: fp32 gradient l2 rel error {worst[2]:.2e}"
