"""HIP encoder kernels (GEMM, LayerNorm, rel-pos attention, conv module,
conv front-end) and the drop-in modules vs the golden fixtures / CPU oracle.
fp32 path: within 1e-4 of the reference; bf16 path: sanity bounds."""
import math
import os

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from conftest import assert_close
import oracle.conformer as OC
import oracle.features as OF

pytestmark = pytest.mark.gpu


def _sub(g, prefix):
    return {k[len(prefix):]: torch.from_numpy(g[k]) for k in g.files if k.startswith(prefix)}


# ----------------------------------------------------------------------------- kernels
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("M,N,K", [(12032, 768, 256), (1000, 256, 1024), (77, 96, 40), (12032, 256, 640),
                                   (300, 144, 144)])
def test_gemm_vs_torch(dev, dtype, M, N, K):
    from speechbrain_amd import _enc
    g = torch.Generator().manual_seed(M + N + K)
    a = torch.randn(M, K, generator=g)
    w = torch.randn(N, K, generator=g) / math.sqrt(K)
    bias = torch.randn(N, generator=g)
    res = torch.randn(M, N, generator=g)
    ad, wd = a.to(dev, dtype), w.to(dev, dtype)
    ref_a, ref_w = ad.float().cpu(), wd.float().cpu()  # same rounded operands
    ref = ref_a @ ref_w.t()
    tol = 2e-5 if dtype == torch.float32 else 2e-3
    out = _enc.gemm(ad, wd)
    assert_close(out, ref, rtol=tol, name="plain")
    out = _enc.gemm(ad, wd, bias=bias.to(dev), act="swish", res=res.to(dev), alpha=0.5)
    r2 = res + 0.5 * F.silu(ref + bias)
    assert_close(out, r2, rtol=tol, name="swish+res")
    mask = (torch.arange(M) % 7 == 3).to(torch.uint8)
    out = _enc.gemm(ad, wd, bias=bias.to(dev), act="gelu", rowmask=mask.to(dev), out_dtype=dtype)
    r3 = F.gelu(ref + bias)
    r3[mask.bool()] = 0
    assert_close(out.float(), r3, rtol=tol if dtype == torch.float32 else 1e-2, name="gelu+mask")


@pytest.mark.parametrize("tile", [11, 12, 13, 18, 19, 20, 21, 22])
@pytest.mark.parametrize("M,N,K", [(12032, 768, 256), (1000, 320, 1024), (77, 64, 192), (12032, 512, 640), (300, 96, 200)])
def test_gemm_ring_tiles_vs_torch(dev, tile, M, N, K):
    """LDS-DMA ring GEMM (bf16) at every tile shape, incl. ragged M and N, with
    the fused epilogues (bias + Swish + residual, GLU pairs)."""
    from speechbrain_amd import _enc
    g = torch.Generator().manual_seed(M + N + K + tile)
    a = torch.randn(M, K, generator=g)
    w = torch.randn(N, K, generator=g) / math.sqrt(K)
    bias = torch.randn(N, generator=g)
    res = torch.randn(M, N, generator=g)
    ad, wd = a.to(dev, torch.bfloat16), w.to(dev, torch.bfloat16)
    ref = ad.float().cpu() @ wd.float().cpu().t()
    if K % 64 and tile in (11, 12, 13):
        pytest.skip("LDS-DMA ring needs K % 64 == 0")
    out = _enc.gemm(ad, wd, tile=tile)
    assert_close(out, ref, rtol=2e-3, name="plain")
    out = _enc.gemm(ad, wd, bias=bias.to(dev), act="swish", res=res.to(dev), alpha=0.5, tile=tile)
    assert_close(out, res + 0.5 * F.silu(ref + bias), rtol=2e-3, name="swish+res")
    if N % 32 == 0:
        gl = _enc.gemm(ad, wd, bias=bias.to(dev), act="glu", tile=tile)
        v = (ref + bias).view(M, N // 32, 2, 16)
        assert_close(gl, (v[:, :, 0] * torch.sigmoid(v[:, :, 1])).reshape(M, N // 2), rtol=2e-3, name="glu")


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("tile", [0, 1, 2])
@pytest.mark.parametrize("M,K", [(12032, 256), (77, 256), (300, 128), (33, 64)])
def test_gemm_ln_vs_torch(dev, dtype, tile, M, K):
    """Output projection + residual + row LayerNorm in one launch (sbk_gemm_ln):
    out = res + (a @ w.T + bias) with masked rows, u = LN(out).  fp32 within
    1e-4 (2e-5 GEMM, LN in fp32); bf16 operands: 2e-3 on out, 2e-2 on bf16 u."""
    from speechbrain_amd import _enc
    if dtype == torch.float32 and tile:
        pytest.skip("fp32 has one tile")
    N = 256
    g = torch.Generator().manual_seed(M + K + tile)
    a = torch.randn(M, K, generator=g)
    w = torch.randn(N, K, generator=g) / math.sqrt(K)
    bias = torch.randn(N, generator=g)
    res = torch.randn(M, N, generator=g)
    lw, lb = 1 + 0.1 * torch.randn(N, generator=g), 0.1 * torch.randn(N, generator=g)
    mask = (torch.arange(M) % 5 == 2).to(torch.uint8)
    ad, wd = a.to(dev, dtype), w.to(dev, dtype)
    ref = ad.float().cpu() @ wd.float().cpu().t() + bias
    ref[mask.bool()] = 0
    ref = ref + res
    uref = F.layer_norm(ref, (N,), lw, lb, 1e-5)
    out, u = _enc.gemm_ln(ad, wd, (lw.to(dev), lb.to(dev), 1e-5), bias=bias.to(dev), res=res.to(dev),
                          rowmask=mask.to(dev), u_dtype=dtype, tile=tile)
    f32 = dtype == torch.float32
    assert_close(out, ref, rtol=2e-5 if f32 else 2e-3, name="out")
    assert_close(u.float(), uref, rtol=1e-4 if f32 else 2e-2, name="u")


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_gemm_glu_permutation(dev, dtype):
    from speechbrain_amd.lobes.models.transformer.Conformer import ConvolutionModule
    from speechbrain_amd import _enc
    torch.manual_seed(0)
    d = 128
    cm = ConvolutionModule(d, 7).to(dev)
    w1p, b1p, _ = cm.kernel_weights(dtype)
    u = torch.randn(333, d).to(dev)
    ud = u.to(dtype)
    g = _enc.gemm(ud, w1p, bias=b1p, act="glu", out_dtype=torch.float32)
    w1 = cm.bottleneck[0].weight.detach().reshape(2 * d, d).float()
    ref = F.glu(ud.float() @ w1.to(dtype).float().t() + cm.bottleneck[0].bias.detach(), dim=-1)
    assert_close(g, ref, rtol=2e-5 if dtype == torch.float32 else 3e-3, name="glu")


def test_layernorm_chain(dev):
    from speechbrain_amd import _enc
    x = torch.randn(1000, 256) * 3 + 1
    w1, b1, w2, b2 = (torch.randn(256) for _ in range(4))
    y1, y2 = _enc.layernorm(x.to(dev), w1.to(dev), b1.to(dev), 1e-5, torch.float32, w2.to(dev), b2.to(dev), 1e-6,
                            torch.float32)
    r1 = F.layer_norm(x, (256,), w1, b1, 1e-5)
    assert_close(y1, r1, rtol=1e-5)
    assert_close(y2, F.layer_norm(r1, (256,), w2, b2, 1e-6), rtol=1e-5)


@pytest.mark.parametrize("D,H,M", [(256, 1024, 1000), (256, 2048, 333), (256, 512, 48), (256, 1024, 12032)])
def test_fused_ffn_vs_unfused(dev, D, H, M):
    """sbk_ffn (LN → Linear → Swish → Linear → 0.5·residual → norm2 → next LN,
    one kernel) vs the same chain through the separate HIP kernels, both bf16
    operands / fp32 accumulation.  Rounding points are identical; only the
    fp32 summation order of the LayerNorm statistics and MFMA K-chunks differ,
    which can flip single bf16 roundings: tolerance 2e-2 of LayerNorm-scale
    values (|a-b| <= 2e-2 * max(1, |b|))."""
    from speechbrain_amd import _enc
    from speechbrain_amd.nnet.attention import PositionalwiseFeedForward
    from speechbrain_amd.nnet.activations import Swish
    torch.manual_seed(0)
    ffn = PositionalwiseFeedForward(H, input_size=D, activation=Swish).to(dev).eval()
    x = (torch.randn(M, D) * 2 + 0.5).to(dev)
    lns = [(torch.randn(D, device=dev) * 0.5 + 1, torch.randn(D, device=dev) * 0.1, 1e-5) for _ in range(3)]
    bf = torch.bfloat16
    with torch.no_grad():
        out, u = ffn.run_fused(x, lns[0], 0.5, post_ln=lns[1], next_ln=lns[2])
        u0, _ = _enc.layernorm(x, *lns[0], out1_dtype=bf)
        z = ffn.run(u0, bf, residual=x, alpha=0.5)
        ref, uref = _enc.layernorm(z, *lns[1], out1_dtype=torch.float32, w2=lns[2][0], b2=lns[2][1],
                                   eps2=lns[2][2], out2_dtype=bf)
        # no post/next LN (the op returns a new tensor; `out=` is ignored)
        x2 = x.clone()
        out2, none = ffn.run_fused(x2, lns[0], 0.5, out=x2)
    assert none is None and torch.equal(x2, x)
    assert_close(out, ref, rtol=2e-2, name="ffn out")
    assert_close(u.float(), uref.float(), rtol=2e-2, name="ffn next-LN")
    assert_close(out2, z, rtol=2e-2, name="ffn no post-LN")


@pytest.mark.parametrize("H,M,NP", [(1024, 12032, 768), (1024, 1000, 768), (512, 48, 256), (2048, 333, 512),
                                    (1024, 500, 1024)])
def test_fused_ffn_proj_vs_unfused(dev, H, M, NP):
    """sbk_ffn_proj (the FFN block + next-LN + the MHSA in_proj, one kernel)
    vs sbk_ffn's u output through the separate sbk_gemm: the same rounding
    points (u rounded to bf16, the projection accumulated in fp32 and rounded
    once), so only summation order differs: 2e-2 as the FFN test.  Ragged M
    exercises the partial last workgroup (its stores and counted waits)."""
    from speechbrain_amd import _enc
    from speechbrain_amd.nnet.attention import PositionalwiseFeedForward
    from speechbrain_amd.nnet.activations import Swish
    torch.manual_seed(1)
    D = 256
    ffn = PositionalwiseFeedForward(H, input_size=D, activation=Swish).to(dev).eval()
    x = (torch.randn(M, D) * 2 + 0.5).to(dev)
    lns = [(torch.randn(D, device=dev) * 0.5 + 1, torch.randn(D, device=dev) * 0.1, 1e-5) for _ in range(2)]
    wp = _enc.cast_bf16((torch.randn(NP, D) / 16).to(dev))
    with torch.no_grad():
        out, y = ffn.run_fused_proj(x, lns[0], 0.5, lns[1], wp)
        ref, u = ffn.run_fused(x, lns[0], 0.5, next_ln=lns[1])
        yref = _enc.gemm(u, wp, out_dtype=torch.bfloat16)
    assert y.shape == (M, NP) and y.dtype == torch.bfloat16
    assert torch.equal(out, ref), "out must not depend on the projection tail"
    assert_close(y.float(), yref.float(), rtol=2e-2, name="ffn_proj y")


@pytest.mark.parametrize("T,F", [(1501, 80), (101, 80), (7, 40)])
def test_fused_frontend_vs_blockwise(dev, T, F):
    """sbk_conv_frontend2 (both ConvBlocks in one kernel, bf16 compute) vs the
    two per-block kernels at the same rounding points, within 2e-2 (a
    different fp32 summation order in block 1's LayerNorm can flip a bf16
    rounding of the intermediate).  The fp32 path runs the per-block kernels."""
    from speechbrain_amd.lobes.models.convolution import ConvolutionFrontEnd
    torch.manual_seed(0)
    cnn = ConvolutionFrontEnd(input_shape=(8, 10, F), num_blocks=2, num_layers_per_block=1, out_channels=(64, 32),
                              kernel_sizes=(3, 3), strides=(2, 2), residuals=(False, False)).to(dev).eval()
    x = torch.randn(3, T, F, device=dev)
    b1, b2 = cnn.convblock_0, cnn.convblock_1
    with torch.no_grad():
        y = cnn.run(x, torch.float32)
        ref = b2.run(b1.run(x, torch.float32), torch.float32)
        assert y.shape == ref.shape
        assert_close(y, ref, rtol=0, name="frontend fp32")
        with torch.autocast("cuda", dtype=torch.bfloat16):
            y16 = cnn.run(x, torch.bfloat16)
            r16 = b2.run(b1.run(x, torch.bfloat16), torch.bfloat16)
    assert_close(y16.float(), r16.float(), rtol=2e-2, name="frontend bf16")


@pytest.mark.parametrize("B,S", [(11, 240000), (32, 240000), (16, 224000)])
def test_fused_frontend_tile_runs(dev, B, S):
    """The persistent front-end kernel at batch sizes where a workgroup walks
    a run of several tiles (B = 32: 1504 tiles on <= 256 workgroups; B = 11:
    517, runs of 2-3 crossing utterance boundaries; B = 16 at 14 s: 351
    output rows per utterance, so every utterance ends in a 7-row tile inside
    a run): the carried block-1 row,
    the staged next-tile rows and the per-utterance top_db floor.  The floor
    binds in every utterance (a near-silent stretch far below max - 80 dB;
    one utterance 20 dB louder, so the floors differ): applying it on load
    must equal running on the clamped features, bit for bit.  Against the
    fp32 oracle (oracle/conformer.py conv_frontend) the error is bounded by
    the oracle's own deviation under CPU bf16 autocast (every conv operand
    rounded to bf16, as the reference runs under autocast), as in
    test_gpu_bench_parity.py."""
    import oracle.conformer as OC
    from speechbrain_amd import ops
    from speechbrain_amd.lobes.features import Fbank
    from speechbrain_amd.lobes.models.convolution import ConvolutionFrontEnd
    g = torch.Generator().manual_seed(B)
    wav = 0.1 * torch.randn(B, S, generator=g)
    wav[:, 40000:56000] *= 1e-6
    wav[B // 2, :] *= 10.0
    wav = wav.to(dev)
    fb = Fbank(n_mels=80).to(dev)
    raw, topdb = fb.forward_deferred(wav)
    clamped = ops.topdb_clamp(raw, *topdb)
    assert (raw < clamped).any()
    torch.manual_seed(1)
    cnn = ConvolutionFrontEnd(input_shape=(8, 10, 80), num_blocks=2, num_layers_per_block=1, out_channels=(64, 32),
                              kernel_sizes=(3, 3), strides=(2, 2), residuals=(False, False)).to(dev).eval()
    with torch.no_grad(), torch.autocast("cuda", dtype=torch.bfloat16):
        y = cnn.run(raw, torch.bfloat16, topdb=topdb)
        y2 = cnn.run(clamped, torch.bfloat16)
    assert torch.equal(y, y2), "the floor on load must equal the clamped input"
    sd = {k: v.cpu() for k, v in cnn.state_dict().items()}
    xin = clamped.float().cpu()
    torch.set_num_threads(max(1, min(16, os.cpu_count() or 1)))
    with torch.no_grad():
        ref = OC.conv_frontend(xin, sd)
        with torch.autocast("cpu", dtype=torch.bfloat16):
            emu = OC.conv_frontend(xin, sd).float()
    out = y.float().cpu()
    assert out.shape == ref.shape
    e_hip, e_emu = (out - ref).abs(), (emu - ref).abs()
    print(f"\nfrontend B={B}: HIP vs fp32 oracle max {e_hip.max():.4e} mean {e_hip.mean():.4e}; "
          f"bf16-operand oracle max {e_emu.max():.4e} mean {e_emu.mean():.4e}")
    assert float(e_hip.max()) <= float(e_emu.max())
    assert float(e_hip.mean()) <= float(e_emu.mean())


# ----------------------------------------------------------------------------- modules vs golden
def test_conv_frontend_vs_golden(golden, dev):
    from speechbrain_amd.lobes.models.convolution import ConvolutionFrontEnd
    g = golden("conformer")
    cnn = ConvolutionFrontEnd(input_shape=(8, 10, 80), num_blocks=2, num_layers_per_block=1, out_channels=(64, 32),
                              kernel_sizes=(3, 3), strides=(2, 2), residuals=(False, False))
    cnn.load_state_dict(_sub(g, "cnn."), strict=True)
    cnn = cnn.to(dev).eval()
    with torch.no_grad():
        out = cnn(torch.from_numpy(g["feats"]).to(dev))
    assert_close(out, g["cnn_out"], name="cnn")


def _tr(g, dev):
    from speechbrain_amd.lobes.models.transformer.TransformerASR import TransformerASR
    tr = TransformerASR(tgt_vocab=10, input_size=640, d_model=64, nhead=4, num_encoder_layers=2,
                        num_decoder_layers=0, d_ffn=128, dropout=0.0, encoder_module="conformer",
                        attention_type="RelPosMHAXL", normalize_before=True, causal=False)
    tr.load_state_dict(_sub(g, "tr."), strict=True)
    return tr.to(dev).eval()


def test_transformer_asr_encode_vs_golden(golden, dev):
    g = golden("conformer")
    tr = _tr(g, dev)
    src = torch.from_numpy(g["cnn_out"]).to(dev)
    with torch.no_grad():
        assert_close(tr.encode(src, torch.from_numpy(g["wav_len"]).to(dev)), g["enc_out"], name="enc")
        assert_close(tr.encode(src), g["enc_out_nolen"], name="enc_nolen")


def test_conformer_encoder_vs_golden(golden, dev):
    from speechbrain_amd.lobes.models.transformer.Conformer import ConformerEncoder
    g = golden("conformer")
    enc = ConformerEncoder(num_layers=2, d_model=64, d_ffn=128, nhead=4, kernel_size=31)
    enc.load_state_dict(_sub(g, "enc."), strict=True)
    enc = enc.to(dev).eval()
    src = torch.from_numpy(g["enc_src"]).to(dev)
    kpm = torch.from_numpy(g["enc_kpm"]).to(dev)
    pe = torch.from_numpy(g["enc_pos"]).to(dev)
    with torch.no_grad():
        y, attn = enc(src, src_key_padding_mask=kpm, pos_embs=pe)
    assert_close(y, g["enc_y"], name="y")
    assert_close(attn[0], g["enc_attn0"], name="attn0")
    assert_close(attn[1], g["enc_attn1"], name="attn1")
    encc = ConformerEncoder(num_layers=1, d_model=64, d_ffn=96, nhead=2, kernel_size=7, causal=True)
    encc.load_state_dict(_sub(g, "encc."), strict=True)
    encc = encc.to(dev).eval()
    with torch.no_grad():
        yc, _ = encc(src, pos_embs=pe)
    assert_close(yc, g["encc_y"], name="causal")


def test_relpos_mha_module_vs_oracle(dev):
    """Standalone RelPosMHAXL (d=256, H=4) vs the oracle at a ragged length."""
    from speechbrain_amd.nnet.attention import RelPosEncXL, RelPosMHAXL
    torch.manual_seed(0)
    mha = RelPosMHAXL(embed_dim=256, num_heads=4).eval()
    sd = {k: v.clone() for k, v in mha.state_dict().items()}
    x = torch.randn(3, 97, 256)
    pe = RelPosEncXL(256)(x)
    kpm = torch.arange(97)[None] >= torch.tensor([97, 60, 5])[:, None]
    ref, ref_attn = OC.rel_pos_mha(x, pe, sd, "", 4, kpm)
    mha = mha.to(dev)
    with torch.no_grad():
        out, attn = mha(x.to(dev), x.to(dev), x.to(dev), pe.to(dev), key_padding_mask=kpm.to(dev))
    assert_close(out, ref, name="mha")
    assert_close(attn, ref_attn, name="attn")


def _relpos_ref(qkv, pk, pbu, pbv, kpm, B, T, H, dh, scale):
    """fp32 torch evaluation of attention.py:566-631 on the kernel's operand
    layout: qkv (B*T, 3d) head-interleaved [h][q|k|v][dh], pk (2T-1, d)."""
    x = qkv.float().view(B, T, H, 3, dh)
    q, k, v = x[:, :, :, 0], x[:, :, :, 1], x[:, :, :, 2]
    p = pk.float().reshape(2 * T - 1, H, dh)
    ac = torch.einsum("bihd,bjhd->bhij", q + pbu.view(H, dh), k)
    bd_full = torch.einsum("bihd,rhd->bhir", q + pbv.view(H, dh), p)
    i = torch.arange(T, device=qkv.device)[:, None]
    j = torch.arange(T, device=qkv.device)[None]
    bd = bd_full[:, :, i, T - 1 - i + j]  # rel_shift in closed form
    s = ((ac + bd) * scale).masked_fill(kpm[:, None, None, :], float("-inf"))
    return torch.einsum("bhij,bjhd->bihd", s.softmax(-1), v).reshape(B * T, H * dh)


@pytest.mark.parametrize("T,lens,strided", [(37, [37, 30, 21], False), (97, [97, 60, 5], True),
                                            (376, [376, 376, 200, 1], True), (640, [640, 640], False),
                                            (256, None, True), (2200, [2200, 2100], False)])
def test_relpos_attention_bf16_vs_torch(dev, T, lens, strided):
    """The encoder's attention path (bf16, dh = 64, no probabilities: the
    LDS-DMA kernel) vs an fp32 torch evaluation on the same bf16 operands:
    ragged key-padding masks incl. a 1-key utterance, and the strided p_k slice
    the encoder passes (one stacked linear_pos GEMM); T = 2200 puts padded keys in
    chunks 32-34 (the high word of the kernel's chunk bitmap).  P is rounded to bf16 for
    the P·V MFMA, so outputs (~N(0,1) averages) agree to 2e-2."""
    from speechbrain_amd import _enc
    g = torch.Generator().manual_seed(T)
    no_mask = lens is None  # no key-padding mask at all (kpm = null)
    lens = [T, T] if no_mask else lens
    B, H, dh = len(lens), 4, 64
    d = H * dh
    qkv = torch.randn(B * T, 3 * d, generator=g).to(torch.bfloat16).to(dev)
    pk_all = torch.randn(2 * T - 1, 3 * d, generator=g).to(torch.bfloat16).to(dev)
    pk = pk_all[:, d:2 * d] if strided else pk_all[:, :d].contiguous()
    pbu = (0.1 * torch.randn(d, generator=g)).to(dev)
    pbv = (0.1 * torch.randn(d, generator=g)).to(dev)
    kpm = (torch.arange(T)[None] >= torch.tensor(lens)[:, None]).to(dev)
    scale = 1.0 / math.sqrt(d)
    out, _ = _enc.relpos_attention(qkv, pk, pbu, pbv, None if no_mask else kpm.to(torch.uint8).contiguous(),
                                   B, T, H, dh, scale)
    ref = _relpos_ref(qkv, pk, pbu, pbv, kpm, B, T, H, dh, scale)
    assert out.dtype == torch.bfloat16
    assert_close(out, ref, rtol=2e-2, name="attn_bf16")


def test_encoder_bf16_autocast_close(golden, dev):
    g = golden("conformer")
    tr = _tr(g, dev)
    src = torch.from_numpy(g["cnn_out"]).to(dev)
    with torch.no_grad(), torch.autocast("cuda", dtype=torch.bfloat16):
        y = tr.encode(src, torch.from_numpy(g["wav_len"]).to(dev))
    ref = torch.from_numpy(g["enc_out"])
    err = (y.float().cpu() - ref).abs().max().item()
    assert y.dtype == torch.float32 and err < 0.1, err  # LayerNorm-scale outputs, bf16 operands


def _c3_modules(d_model, dev):
    """BASELINE config 3: ConvolutionFrontEnd + 12-layer Conformer (conformer_small.yaml shapes)."""
    from speechbrain_amd.lobes.models.convolution import ConvolutionFrontEnd
    from speechbrain_amd.lobes.models.transformer.TransformerASR import TransformerASR
    torch.manual_seed(0)
    cnn = ConvolutionFrontEnd(input_shape=(8, 10, 80), num_blocks=2, num_layers_per_block=1, out_channels=(64, 32),
                              kernel_sizes=(3, 3), strides=(2, 2), residuals=(False, False))
    tr = TransformerASR(tgt_vocab=5000, input_size=640, d_model=d_model, nhead=4, num_encoder_layers=12,
                        num_decoder_layers=0, d_ffn=1024, dropout=0.1, encoder_module="conformer",
                        attention_type="RelPosMHAXL", normalize_before=True, causal=False)
    return cnn.to(dev).eval(), tr.to(dev).eval()


@pytest.mark.parametrize("d_model", [256, 144])
def test_full_size_encoder_vs_oracle(dev, d_model):
    """Fbank → CNN → 12-layer encoder at 15 s, fp32 path vs the CPU oracle on
    2 utterances (rows are independent, so this checks the full-size kernels)."""
    from speechbrain_amd.lobes.features import Fbank
    cnn, tr = _c3_modules(d_model, dev)
    g = torch.Generator().manual_seed(0)
    wav = 0.1 * torch.randn(2, 240000, generator=g)
    with torch.no_grad():
        feats = Fbank(n_mels=80)(wav.to(dev))
        y = tr.encode(cnn(feats), torch.ones(2, device=dev))
    sd_cnn = {k: v.cpu() for k, v in cnn.state_dict().items()}
    sd_tr = {k: v.cpu() for k, v in tr.state_dict().items()}
    ref = OC.fbank_to_encoder(wav, sd_cnn, sd_tr, 12, 4, wav_len=torch.ones(2))
    assert y.shape == (2, 376, d_model)
    assert_close(y, ref, rtol=1e-4, name="full")


def test_full_size_encoder_bf16_vs_fp32(dev):
    """d=256 encoder at 15 s under bf16 autocast (fused FFN kernels, bf16
    GEMM/attention) vs the fp32 path: LayerNorm-scale outputs within 0.1."""
    cnn, tr = _c3_modules(256, dev)
    g = torch.Generator().manual_seed(1)
    feats = torch.randn(4, 1501, 80, generator=g).to(dev)
    with torch.no_grad():
        src = cnn(feats)
        y32 = tr.encode(src, torch.ones(4, device=dev))
        with torch.autocast("cuda", dtype=torch.bfloat16):
            y16 = tr.encode(src, torch.ones(4, device=dev))
    err = (y16.float() - y32).abs()
    assert y16.dtype == torch.float32 and torch.isfinite(y16).all()
    assert err.max().item() < 0.1 and err.mean().item() < 0.01, (err.max().item(), err.mean().item())


def test_length_mask_vs_reference_formula(dev):
    """sbk_length_mask == (arange(T) > floor(wav_len * T)) (TransformerASR.py:295-301),
    bit-exact, incl. lengths whose product lands exactly on an integer."""
    from speechbrain_amd import _enc
    g = torch.Generator().manual_seed(5)
    for T in (1, 7, 376, 1000):
        rel = torch.cat([torch.rand(13, generator=g), torch.tensor([1.0, 0.5, 0.25, 0.0, 0.8, 1 / 3])])
        ref = (torch.arange(T)[None, :].to(torch.float32) > torch.floor(rel * T)[:, None]).to(torch.uint8)
        out = _enc.length_mask(rel.to(dev), T).cpu()
        assert torch.equal(out, ref), T


@pytest.mark.parametrize("B,T,K,causal,masked", [(32, 376, 31, False, True), (3, 37, 31, False, True),
                                                 (2, 50, 7, True, False), (4, 97, 15, False, True),
                                                 (1, 5, 31, False, False)])
def test_fused_conv_module_vs_chain(dev, B, T, K, causal, masked):
    """sbk_conv_module (LN -> GLU GEMM -> dwconv -> LN -> Swish -> GEMM -> mask ->
    residual in one launch, halo frames recomputed per 48-frame block) vs the
    four-launch chain at the same bf16 rounding points: within 2e-2 of
    LayerNorm-scale values (fp32 summation order can flip single bf16
    roundings of the intermediates); and vs the fp32 oracle within 0.1."""
    from speechbrain_amd.lobes.models.transformer.Conformer import ConvolutionModule
    from speechbrain_amd import _enc
    torch.manual_seed(K + T)
    cm = ConvolutionModule(256, K, causal=causal).to(dev).eval()
    with torch.no_grad():
        for p in cm.parameters():
            p.add_(0.05 * torch.randn_like(p))
    x = (torch.randn(B * T, 256) * 2 + 0.3).to(dev)
    kpm = None
    if masked:
        lens = torch.randint(1, T + 1, (B,))
        lens[0] = T
        kpm = (torch.arange(T)[None] >= lens[:, None]).to(torch.uint8).reshape(-1).to(dev)
    assert cm.fusable(torch.bfloat16, 256)
    with torch.no_grad():
        y = cm.run_fused(x, B, T, kpm)
        ref = cm.run(x, B, T, torch.bfloat16, kpm, residual=x)
    assert_close(y, ref, rtol=2e-2, name="fused vs chain")
    sd = {k: v.cpu() for k, v in cm.state_dict().items()}
    pm = kpm.cpu().bool().view(B, T, 1) if kpm is not None else None
    r32 = x.cpu().view(B, T, 256) + OC.conv_module(x.cpu().view(B, T, 256), sd, "", K, causal, pm)
    err = (y.cpu().view(B, T, 256) - r32).abs().max().item()
    assert err < 0.1, err


@pytest.mark.parametrize("B,T,K,causal,masked", [(32, 376, 31, False, True), (3, 37, 31, False, True),
                                                 (2, 50, 7, True, False), (1, 5, 31, False, False)])
def test_conv_module_with_out_proj(dev, B, T, K, causal, masked):
    """sbk_conv_module_pre (the MHSA output projection + residual computed in
    the conv module's prologue, x_att = x + o Wo^T + bo never written apart
    from the launch's own rows) vs sbk_gemm(o, Wo, bo, res=x) followed by
    sbk_conv_module: x_att is the same fp32 product in a different summation
    order, so the LN0 bf16 rounding can flip — 2e-2 as the other fused
    module tests."""
    from speechbrain_amd.lobes.models.transformer.Conformer import ConvolutionModule
    from speechbrain_amd import _enc
    torch.manual_seed(K + T + 1)
    cm = ConvolutionModule(256, K, causal=causal).to(dev).eval()
    with torch.no_grad():
        for p in cm.parameters():
            p.add_(0.05 * torch.randn_like(p))
    x = (torch.randn(B * T, 256) * 2 + 0.3).to(dev)
    o = torch.randn(B * T, 256, device=dev).to(torch.bfloat16)
    wo = _enc.cast_bf16(torch.randn(256, 256, device=dev) / 16)
    bo = torch.randn(256, device=dev) * 0.1
    kpm = None
    if masked:
        lens = torch.randint(1, T + 1, (B,))
        lens[0] = T
        kpm = (torch.arange(T)[None] >= lens[:, None]).to(torch.uint8).reshape(-1).to(dev)
    with torch.no_grad():
        y = cm.run_fused(x, B, T, kpm, pre=(o, wo, bo))
        xa = _enc.gemm(o, wo, bias=bo, res=x)
        ref = cm.run_fused(xa, B, T, kpm)
    assert_close(y, ref, rtol=2e-2, name="conv module with out_proj")


@pytest.mark.parametrize("H,M", [(1024, 12032), (1024, 1000), (512, 48)])
def test_ffn_chain_vs_two_launches(dev, H, M):
    """sbk_ffn_chain (FFN2 + norm2 of layer i, then FFN1 + norm1 + in_proj of
    layer i+1, the intermediate rows kept on chip) vs sbk_ffn (with norm2)
    followed by sbk_ffn_proj: the same rounding points, so only summation
    order differs (2e-2 as the other fused-FFN tests)."""
    from speechbrain_amd import _enc
    from speechbrain_amd.nnet.attention import PositionalwiseFeedForward
    from speechbrain_amd.nnet.activations import Swish
    torch.manual_seed(2)
    D = 256
    fa = PositionalwiseFeedForward(H, input_size=D, activation=Swish).to(dev).eval()
    fb = PositionalwiseFeedForward(H, input_size=D, activation=Swish).to(dev).eval()
    x = (torch.randn(M, D) * 2 + 0.5).to(dev)
    lns = [(torch.randn(D, device=dev) * 0.5 + 1, torch.randn(D, device=dev) * 0.1, 1e-5) for _ in range(4)]
    wp = _enc.cast_bf16((torch.randn(768, D) / 16).to(dev))
    with torch.no_grad():
        out, y = _enc.ffn_chain(x, fa.chain_block(lns[0], 0.5, post_ln=lns[1]), fb.chain_block(lns[2], 0.5),
                                "swish", 0.0, lns[3], wp)
        mid, _ = fa.run_fused(x, lns[0], 0.5, post_ln=lns[1])
        ref, yref = fb.run_fused_proj(mid, lns[2], 0.5, lns[3], wp)
    assert_close(out, ref, rtol=2e-2, name="chain out")
    assert_close(y.float(), yref.float(), rtol=2e-2, name="chain projection")


def test_encoder_chain_vs_per_layer(dev):
    """The chained stack (3 launches per layer) vs the per-layer fused path
    on a config-3 encoder at full size: bf16 rounding points are the same
    up to summation order, so 2e-2 of LayerNorm-scale values."""
    from speechbrain_amd.lobes.models.transformer import Conformer as C
    from speechbrain_amd.lobes.models.transformer.TransformerASR import TransformerASR
    torch.manual_seed(0)
    tr = TransformerASR(tgt_vocab=10, input_size=640, d_model=256, nhead=4, num_encoder_layers=12,
                        num_decoder_layers=0, d_ffn=1024, dropout=0.0, encoder_module="conformer",
                        attention_type="RelPosMHAXL", normalize_before=True, causal=False).to(dev).eval()
    src = torch.randn(4, 376, 640, device=dev)
    lens = torch.tensor([1.0, 0.8, 0.6, 1.0], device=dev)
    with torch.no_grad(), torch.autocast("cuda", dtype=torch.bfloat16):
        y_chain = tr.encode(src, lens)
        C.USE_LAYER_CHAIN = False
        try:
            y_ref = tr.encode(src, lens)
        finally:
            C.USE_LAYER_CHAIN = True
    assert_close(y_chain, y_ref, rtol=2e-2, name="chain vs per-layer")


def test_ffn_weight_image_layout(dev):
    """sbk_ffn_image: the fused FFN kernels' weight stream — 32-KB tiles in
    stream order (per block and 256-unit hidden chunk: D/64 tiles of W1, 4 of
    W2; then D/64 per 256 projection columns), each row's 16-B chunks in the
    ring's swizzled order j' -> j' ^ ((row >> 1) & 7) — bit-exact against the
    same layout built with torch indexing."""
    from speechbrain_amd import _enc
    g = torch.Generator().manual_seed(3)
    D, H, NP = 256, 512, 768
    ws = [torch.randn(*shp, generator=g).to(torch.bfloat16).to(dev)
          for shp in ((H, D), (D, H), (H, D), (D, H), (NP, D))]
    perm = torch.tensor([[jp ^ ((r >> 1) & 7) for jp in range(8)] for r in range(256)])

    def tile(mat, r0, k0):
        t = mat[r0:r0 + 256, k0:k0 + 64].cpu().reshape(256, 8, 8)
        return torch.gather(t, 1, perm[:, :, None].expand(256, 8, 8)).reshape(-1)

    def blocks(w1, w2):
        out = []
        for c in range(H // 256):
            out += [tile(w1, c * 256, r * 64) for r in range(D // 64)]
            out += [tile(w2, 0, c * 256 + r * 64) for r in range(4)]
        return out

    proj = [tile(ws[4], nc * 256, r * 64) for nc in range(NP // 256) for r in range(D // 64)]
    single = _enc.ffn_image(ws[0], ws[1])
    assert torch.equal(single.cpu(), torch.cat(blocks(ws[0], ws[1])))
    chain = _enc.ffn_image(*ws)
    assert torch.equal(chain.cpu(), torch.cat(blocks(ws[0], ws[1]) + blocks(ws[2], ws[3]) + proj))
    assert _enc.ffn_image(*ws) is chain  # cached while no weight changes
    ws[4].add_(1)  # an in-place update (new version) rebuilds it
    assert _enc.ffn_image(*ws) is not chain
