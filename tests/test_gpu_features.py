"""HIP feature kernels vs the golden fixtures and the CPU oracle (parity)."""
import numpy as np
import pytest
import torch

from conftest import assert_close
import oracle.features as OF

pytestmark = pytest.mark.gpu


def _mods():
    from speechbrain_amd.processing import features as F
    from speechbrain_amd.lobes import features as LF
    return F, LF


def test_stft_vs_golden(golden, dev):
    F, _ = _mods()
    g = golden("features")
    x, x3 = torch.from_numpy(g["x"]).to(dev), torch.from_numpy(g["x3"]).to(dev)
    st = F.STFT(sample_rate=16000)
    s = st(x)
    assert_close(s, g["stft"], name="stft")
    assert_close(st(x3), g["stft3"], name="stft3")
    stb = F.STFT(sample_rate=16000, win_length=20, hop_length=5, n_fft=512, pad_mode="reflect")
    assert_close(stb(x), g["stft_b"], name="stft_b")
    assert_close(F.spectral_magnitude(s), g["mag_p1"], name="mag")
    assert_close(F.spectral_magnitude(s, power=0.5), g["mag_p05"], name="mag05")
    assert_close(F.spectral_magnitude(s, power=1, log=True), g["mag_log"], rtol=2e-4, name="maglog")
    # fused STFT→power equals the two-step path
    assert_close(st.power_spectrum(x), g["mag_p1"], name="fused power")


@pytest.mark.parametrize("n_fft,hop,center,pad", [(400, 160, True, "constant"), (512, 128, True, "reflect"),
                                                    (256, 100, False, "constant"), (480, 160, True, "replicate"),
                                                    (384, 96, True, "circular")])
def test_stft_geometries_vs_oracle(dev, n_fft, hop, center, pad):
    F, _ = _mods()
    g = torch.Generator().manual_seed(n_fft)
    x = 0.3 * torch.randn(3, 4001, generator=g)
    ms_win, ms_hop = n_fft / 16.0, hop / 16.0
    st = F.STFT(16000, win_length=ms_win, hop_length=ms_hop, n_fft=n_fft, center=center, pad_mode=pad)
    ref = OF.stft(x, 16000, ms_win, ms_hop, n_fft, center=center, pad_mode=pad, compute_dtype=torch.float64)
    out = st(x.to(dev))
    scale = float(ref.abs().max())
    assert_close(out / scale, ref / scale, rtol=2e-6, name=f"stft{n_fft}")
    st2 = F.STFT(16000, win_length=ms_win, hop_length=ms_hop, n_fft=n_fft, center=center, pad_mode=pad,
                 onesided=False, normalized_stft=True)
    ref2 = OF.stft(x, 16000, ms_win, ms_hop, n_fft, normalized=True, center=center, pad_mode=pad, onesided=False,
                   compute_dtype=torch.float64)
    s2 = float(ref2.abs().max())
    assert_close(st2(x.to(dev)) / s2, ref2 / s2, rtol=2e-6, name="twosided")


@pytest.mark.parametrize("shape", ["triangular", "rectangular", "gaussian"])
def test_filterbank_vs_golden(golden, dev, shape):
    F, _ = _mods()
    g = golden("features")
    mag = torch.from_numpy(g["mag_p1"]).to(dev)
    assert_close(F.Filterbank(n_mels=40, filter_shape=shape)(mag), g[f"fb_{shape}"], name=shape)


def test_filterbank_variants_vs_golden(golden, dev):
    F, _ = _mods()
    g = golden("features")
    mag = torch.from_numpy(g["mag_p1"]).to(dev)
    assert_close(F.Filterbank(n_mels=23, log_mel=False)(mag), g["fb_lin"], name="lin")
    assert_close(F.Filterbank(n_mels=80)(mag), g["fb_80"], name="80")
    assert_close(F.Filterbank(n_mels=40, f_min=100, f_max=7000)(mag), g["fb_fmin_fmax"], name="fminmax")
    x3 = torch.from_numpy(g["x3"]).to(dev)
    st = F.STFT(sample_rate=16000)
    assert_close(F.Filterbank(n_mels=40)(F.spectral_magnitude(st(x3))), g["fb_multi"], name="multi")
    assert_close(F.Filterbank(n_mels=40, freeze=False)(mag), g["fb_learn"], name="learnable fwd")


def test_filterbank_reference_unit_checks(dev):
    """tests/unittests/test_features.py:60-88 on the HIP path."""
    F, _ = _mods()
    fb = F.Filterbank()
    z = fb(torch.zeros(10, 101, 201, device=dev))
    assert torch.equal(z, torch.full_like(z, -100.0))
    i1 = torch.rand(1, 101, 201, device=dev) * 10
    i2 = torch.rand(1, 101, 201, device=dev)
    f1, f2, f3 = fb(i1), fb(i2), fb(torch.cat([i1, i2]))
    assert torch.sum(torch.abs(f1[0] - f3[0])) < 8e-5
    assert torch.sum(torch.abs(f2[0] - f3[1])) < 8e-5
    assert torch.jit.trace(fb, torch.ones(10, 101, 201, device=dev))


def test_dct_deltas_context_vs_golden(golden, dev):
    F, _ = _mods()
    g = golden("features")
    fb40 = torch.from_numpy(g["fb_triangular"]).to(dev)
    d = F.DCT(input_size=40)(fb40)
    assert_close(d, g["dct"], name="dct")
    assert_close(F.DCT(input_size=40, n_out=13, ortho_norm=False)(fb40), g["dct_noortho"], name="dct2")
    deltas = F.Deltas(input_size=20)
    d1 = deltas(d)
    assert_close(d1, g["delta1"], name="d1")
    assert_close(deltas(d1), g["delta2"], name="d2")
    assert_close(F.Deltas(input_size=20, window_length=7)(d), g["delta_w7"], name="d7")
    for lf, rf in ((5, 5), (0, 2), (3, 1), (0, 0)):
        assert_close(F.ContextWindow(lf, rf)(d), g[f"cw_{lf}_{rf}"], rtol=0, name=f"cw{lf}{rf}")


def test_deltas_context_reference_unit_checks(dev):
    """tests/unittests/test_features.py:4-39."""
    F, _ = _mods()
    inp = torch.ones(10, 101, 20, device=dev)
    d = F.Deltas(input_size=20)
    assert torch.sum(d(inp) == 0) == inp.numel()
    assert torch.jit.trace(d, inp)
    cw = F.ContextWindow(left_frames=1, right_frames=1)
    out = cw(torch.tensor([1.0, 2, 3], device=dev).view(1, 3, 1))
    assert torch.equal(out, torch.tensor([[[0.0, 1, 2], [1, 2, 3], [2, 3, 0]]], device=dev))
    inp = torch.rand(2, 10, 5, device=dev)
    assert torch.equal(F.ContextWindow(0, 0)(inp), inp)
    assert torch.jit.trace(F.ContextWindow(0, 0), inp)


def test_multichannel_deltas_context(dev):
    F, _ = _mods()
    x = torch.randn(2, 30, 6, 3)
    d = F.Deltas(input_size=6)(x.to(dev))
    ref = OF.deltas(x)
    assert_close(d, ref, name="deltas4d")


@pytest.mark.parametrize("n_mels", [80, 40])
def test_fbank_wavs_vs_golden(golden, dev, n_mels):
    _, LF = _mods()
    g = golden("fbank_wavs")
    fb = LF.Fbank(n_mels=n_mels)
    for i in range(3):
        w = torch.from_numpy(g[f"pcm{i}"].astype(np.float32) / 32768.0)[None].to(dev)
        assert_close(fb(w), g[f"fbank{n_mels}_single{i}"], name=f"wav{i}")
    L = max(len(g[f"pcm{i}"]) for i in range(3))
    batch = torch.zeros(3, L)
    for i in range(3):
        p = g[f"pcm{i}"]
        batch[i, :len(p)] = torch.from_numpy(p.astype(np.float32) / 32768.0)
    assert_close(fb(batch.to(dev)), g[f"fbank{n_mels}_batch"], name="batch")


def test_mfcc_fbank_composites_vs_golden(golden, dev):
    _, LF = _mods()
    g = golden("features")
    x = torch.from_numpy(g["x"]).to(dev)
    assert_close(LF.MFCC()(x), g["mfcc"], name="mfcc")
    fb = LF.Fbank(n_mels=40, deltas=True, context=True, left_frames=2, right_frames=2)
    assert_close(fb(x), g["fbank_dc"], name="fbdc")
    # state_dict key names match the reference (Fbank has buffer compute_deltas.kernel)
    assert list(fb.state_dict()) == ["compute_deltas.kernel"]


def test_fbank_full_size_properties(dev):
    """BASELINE config 2 size (32 x 15 s): compare against the oracle on a
    subset of utterances, and check batch-invariance on the full batch."""
    _, LF = _mods()
    g = torch.Generator().manual_seed(0)
    wav = 0.1 * torch.randn(32, 240000, generator=g)
    fb = LF.Fbank(n_mels=80)
    out = fb(wav.to(dev))
    assert out.shape == (32, 1501, 80)
    ref = OF.fbank(wav[:2], n_mels=80)
    assert_close(out[:2], ref, name="full")
    one = fb(wav[5:6].to(dev))
    assert torch.equal(one[0], out[5])  # per-utterance top_db: batch-invariant, bit-exact


def _rel_max(a, b):
    a = a.detach().double().cpu() if isinstance(a, torch.Tensor) else torch.as_tensor(a).double()
    b = torch.as_tensor(b).double()
    return float((a - b).abs().max() / b.abs().max().clamp(min=1e-30))


def test_learnable_filterbank_backward_vs_golden(golden, dev):
    """Filterbank(freeze=False) trains: y.sum().backward() gives the reference's
    own autograd gradients of f_central / band (features.py:476-482; golden
    fb_learn_grad_fc / fb_learn_grad_band), via the HIP dB/top_db backward,
    the dense matᵀ product and the chunked matrix-gradient reduction."""
    F, _ = _mods()
    g = golden("features")
    mag = torch.from_numpy(g["mag_p1"]).to(dev)
    fb = F.Filterbank(n_mels=40, freeze=False).to(dev)
    y = fb(mag)
    assert_close(y, g["fb_learn"], name="fwd")
    y.sum().backward()
    # tolerance: 1e-4 of the largest gradient (fp32 sums of 8,080 dB terms)
    assert _rel_max(fb.f_central.grad, g["fb_learn_grad_fc"]) < 1e-4
    assert _rel_max(fb.band.grad, g["fb_learn_grad_band"]) < 1e-4


def test_fbank_requires_grad_trains_filters(golden, dev):
    """Fbank(requires_grad=True) (lobes/features.py:108-112 → freeze=False): the
    same pipeline as the golden learnable filterbank, so the same gradients."""
    _, LF = _mods()
    g = golden("features")
    fb = LF.Fbank(n_mels=40, requires_grad=True).to(dev)
    y = fb(torch.from_numpy(g["x"]).to(dev))
    assert_close(y, g["fb_learn"], name="fwd")
    y.sum().backward()
    assert _rel_max(fb.compute_fbanks.f_central.grad, g["fb_learn_grad_fc"]) < 1e-4
    assert _rel_max(fb.compute_fbanks.band.grad, g["fb_learn_grad_band"]) < 1e-4


def test_filterbank_backward_vs_torch_autograd(dev):
    """dL/dspec and dL/dmat of the dense filterbank (random weights R, a
    spectrogram with silent frames so the top_db floor and the amin clamp are
    both active) against torch autograd of the reference's formula
    (features.py:551,701-711) in float64 on the CPU."""
    from speechbrain_amd import ops
    gen = torch.Generator().manual_seed(3)
    spec = torch.rand(3, 37, 201, generator=gen) ** 4
    spec[0, :5] = 0.0            # x < amin → clamp path, zero gradient
    spec[1] *= 1e-6
    spec[1, 10] = 1.0            # one loud frame → most of utterance 1 floored at max-80 dB
    mat = torch.rand(201, 40, generator=gen)
    R = torch.randn(3, 37, 40, generator=gen)
    sd, md = spec.to(dev).requires_grad_(), mat.to(dev).requires_grad_()
    y = ops.filterbank_dense(sd, md, True, 10.0, 0.0, 1e-10, 80.0)
    (y * R.to(dev)).sum().backward()
    s64, m64 = spec.double().requires_grad_(), mat.double().requires_grad_()
    x_db = 10.0 * torch.log10(torch.clamp(s64 @ m64, min=1e-10))
    ref = torch.max(x_db, (x_db.amax(dim=(-2, -1)) - 80.0).view(3, 1, 1))
    (ref * R.double()).sum().backward()
    assert float((y.detach().cpu().double() - ref.detach()).abs().max()) < 1e-3
    assert _rel_max(sd.grad, s64.grad) < 1e-4
    assert _rel_max(md.grad, m64.grad) < 1e-4


def test_dct_backward(dev):
    F, _ = _mods()
    gen = torch.Generator().manual_seed(4)
    x = torch.randn(2, 11, 23, generator=gen)
    R = torch.randn(2, 11, 20, generator=gen)
    d = F.DCT(input_size=23, n_out=20)
    xd = x.to(dev).requires_grad_()
    (d(xd) * R.to(dev)).sum().backward()
    assert _rel_max(xd.grad, R @ d.dct_mat.t()) < 1e-5


def test_fbank_deferred_topdb_into_frontend2(dev):
    """The bench step's fusion: Fbank.forward_deferred leaves the top_db floor
    (features.py:706-711) to the consumer; ops.topdb_clamp of it is
    bit-identical to Fbank.forward, and the fused front-end applying the
    floor on load is bit-identical to the front-end on the clamped features.
    The wave is scaled so that the floor clamps part of every utterance."""
    from speechbrain_amd import ops
    from speechbrain_amd.lobes.features import Fbank
    from speechbrain_amd.lobes.models.convolution import ConvolutionFrontEnd
    g = torch.Generator().manual_seed(8)
    wav = 0.1 * torch.randn(3, 48000, generator=g)
    wav[:, 16000:20000] *= 1e-6  # near-silence: far below max - 80 dB
    wav = wav.to(dev)
    fb = Fbank(n_mels=80).to(dev)
    ref = fb(wav)
    raw, topdb = fb.forward_deferred(wav)
    assert topdb is not None
    clamped = ops.topdb_clamp(raw, *topdb)
    assert torch.equal(clamped, ref)
    assert (raw < ref).any(), "the floor must bind somewhere for this test to mean anything"
    torch.manual_seed(0)
    cnn = ConvolutionFrontEnd(input_shape=(8, 10, 80), num_blocks=2, num_layers_per_block=1, out_channels=(64, 32),
                              kernel_sizes=(3, 3), strides=(2, 2), residuals=(False, False)).to(dev).eval()
    with torch.no_grad(), torch.autocast("cuda", dtype=torch.bfloat16):
        a = cnn.run(ref, torch.bfloat16)
        b = cnn.run(raw, torch.bfloat16, topdb=topdb)
    assert torch.equal(a, b)


@pytest.mark.parametrize("n_mels", [80, 42])
def test_fbank_deltas_floor_on_load(dev, n_mels):
    """Fbank(deltas=True): the concat deltas kernel applies the deferred
    top_db floor as it loads (sbk_deltas_floor) — bit-identical to the
    clamped fbank followed by the concat deltas; n_mels % 4 != 0 keeps the
    clamp pass (scalar kernel).  The floor binds in every utterance."""
    from speechbrain_amd import ops
    from speechbrain_amd.lobes.features import Fbank
    g = torch.Generator().manual_seed(9)
    wav = 0.1 * torch.randn(3, 48000, generator=g)
    wav[:, 16000:20000] *= 1e-6
    wav = wav.to(dev)
    plain = Fbank(n_mels=n_mels).to(dev)(wav)
    ref = ops.deltas(plain, 5, True)
    out = Fbank(n_mels=n_mels, deltas=True).to(dev)(wav)
    assert out.shape == (3, plain.shape[1], 3 * n_mels)
    assert torch.equal(out, ref)
    raw, _ = Fbank(n_mels=n_mels).to(dev).forward_deferred(wav)
    assert (raw < plain).any(), "the floor must bind somewhere for this test to mean anything"


@pytest.mark.parametrize("S,hop_ms,center,pad,power,log", [
    (16000, 10, True, "constant", 1, False),    # staged spans (hop 160), utterance ends on the map_pos path
    (3001, 10, True, "constant", 1, False),     # T = 19: a partial 8-frame wave, frames past T recomputed
    (1200, 10, True, "constant", 1, False),     # T = 8: one wave, every frame near an end
    (16000, 6.25, True, "reflect", 1, False),   # hop 100 (staged), reflect padding at the ends
    (16000, 10.125, True, "constant", 1, False),  # hop 162: spans not 16-B aligned -> unstaged path
    (16000, 10, False, "constant", 0.5, True),  # center=False, generic power + log magnitude
])
def test_register_fft_geometries_vs_oracle(dev, S, hop_ms, center, pad, power, log):
    """The n_fft = 400 power / Fbank path (spec_reg_kernel, features.hip): its
    LDS-DMA span staging, unstaged edge path, partial waves and generic
    power, against the float64 oracle (features.py:101-188, 327-356)."""
    F, _ = _mods()
    g = torch.Generator().manual_seed(S + int(100 * hop_ms))
    x = 0.2 * torch.randn(3, S, generator=g)
    st = F.STFT(16000, hop_length=hop_ms, center=center, pad_mode=pad)
    ref = OF.spectral_magnitude(OF.stft(x, 16000, 25, hop_ms, 400, center=center, pad_mode=pad,
                                        compute_dtype=torch.float64), power=power, log=log)
    out = st.power_spectrum(x.to(dev), power=power, log=log)
    assert out.shape == ref.shape
    if log:
        assert_close(out, ref, rtol=2e-4, name="log power")
    else:
        scale = float(ref.abs().max())
        assert_close(out / scale, ref / scale, rtol=2e-6, name="power")
    if center and pad == "constant" and power == 1:
        # the fused Fbank (mel + dB in the same kernel) at this geometry
        _, LF = _mods()
        fbk = LF.Fbank(n_mels=80, hop_length=hop_ms)(x.to(dev))
        assert_close(fbk, OF.fbank(x, n_mels=80, hop_length=hop_ms), name="fbank")


def test_fbank_misaligned_view(dev):
    """A contiguous waveform view at a 4-B storage offset (not 16-B aligned):
    the register-FFT kernel's LDS-DMA span staging needs a 16-B aligned base,
    so such a view must take the unstaged load path (features.hip span_of),
    with the same result as an aligned copy and the oracle."""
    _, LF = _mods()
    g = torch.Generator().manual_seed(11)
    flat = 0.2 * torch.randn(3 * 16000 + 1, generator=g)
    xd = flat.to(dev)[1:].view(3, 16000)
    assert xd.is_contiguous() and xd.data_ptr() % 16 == 4
    fb = LF.Fbank(n_mels=80)
    out = fb(xd)
    assert_close(out, OF.fbank(flat[1:].view(3, 16000), n_mels=80), name="fbank of a 4-B offset view")
    assert torch.equal(out, fb(xd.clone()))


@pytest.mark.parametrize("T", [1, 3, 5, 8, 9, 12, 17, 100, 1501])
@pytest.mark.parametrize("F", [4, 40, 80, 240])
def test_concat_deltas_edges_vs_oracle(dev, T, F):
    """The concat deltas (window 5) against the oracle's
    Δ / ΔΔ restatement (features.py:806-852) for T around the run length
    and the utterance edges; the top_db-floor form against clamp + deltas
    bit for bit."""
    import oracle.features as OF
    from speechbrain_amd import ops
    g = torch.Generator().manual_seed(T * 1000 + F)
    x = torch.randn(3, T, F, generator=g)
    out = ops.deltas(x.to(dev), 5, True)
    d1 = OF.deltas(x)
    d2 = OF.deltas(d1)
    ref = torch.cat([x, d1, d2], dim=-1)
    assert_close(out, ref, rtol=1e-5, name=f"deltas T={T} F={F}")
    slots = torch.randn(3, 7, generator=g).to(dev)
    top_db = 1.5
    floored = ops.deltas_floor(x.to(dev), 5, slots, top_db)
    fl = slots.max(dim=1).values - top_db
    ref2 = ops.deltas(torch.maximum(x.to(dev), fl[:, None, None]), 5, True)
    assert torch.equal(floored, ref2)
