"""Pin the CPU oracle against golden vectors produced by the real reference
(tests/golden/gen_golden.py) and the reference's own known-answer tests.
CPU only; no GPU, no libsbk.so."""
import numpy as np
import pytest
import torch

from conftest import assert_close
import oracle.augment as OA
import oracle.conformer as OC
import oracle.features as OF
import oracle.rnnt as OR


def test_stft_family(golden):
    g = golden("features")
    x, x3 = torch.from_numpy(g["x"]), torch.from_numpy(g["x3"])
    s = OF.stft(x)
    assert_close(s, g["stft"], name="stft")
    assert_close(OF.stft(x3), g["stft3"], name="stft3")
    assert_close(OF.stft(x, win_length=20, hop_length=5, n_fft=512, pad_mode="reflect"), g["stft_b"], name="stft_b")
    mag = OF.spectral_magnitude(s)
    assert_close(mag, g["mag_p1"], name="mag")
    assert_close(OF.spectral_magnitude(s, 0.5), g["mag_p05"], name="mag05")
    assert_close(OF.spectral_magnitude(s, 1, True), g["mag_log"], rtol=2e-4, name="maglog")


@pytest.mark.parametrize("shape", ["triangular", "rectangular", "gaussian"])
def test_filterbank_shapes(golden, shape):
    g = golden("features")
    mag = torch.from_numpy(g["mag_p1"])
    assert_close(OF.filterbank(mag, filter_shape=shape), g[f"fb_{shape}"], name=shape)


def test_filterbank_variants(golden):
    g = golden("features")
    mag = torch.from_numpy(g["mag_p1"])
    assert_close(OF.filterbank(mag, n_mels=23, log_mel=False), g["fb_lin"], name="lin")
    assert_close(OF.filterbank(mag, n_mels=80), g["fb_80"], name="80")
    assert_close(OF.filterbank(mag, f_min=100, f_max=7000), g["fb_fmin_fmax"], name="fminmax")
    x3 = torch.from_numpy(g["x3"])
    assert_close(OF.filterbank(OF.spectral_magnitude(OF.stft(x3))), g["fb_multi"], name="multi")


def test_filterbank_reference_unit_checks():
    """tests/unittests/test_features.py:60-88 restated on the oracle."""
    z = OF.filterbank(torch.zeros(10, 101, 201))
    assert torch.equal(z, torch.full_like(z, -100.0))
    assert torch.equal(OF.amplitude_to_db(torch.zeros(1, 1, 1)), torch.tensor([[[-100.0]]]))


def test_dct_deltas_context(golden):
    g = golden("features")
    fb40 = torch.from_numpy(g["fb_triangular"])
    d = OF.dct(fb40)
    assert_close(d, g["dct"], name="dct")
    assert_close(OF.dct(fb40, 13, False), g["dct_noortho"], name="dct2")
    d1 = OF.deltas(d)
    assert_close(d1, g["delta1"], name="d1")
    assert_close(OF.deltas(d1), g["delta2"], name="d2")
    assert_close(OF.deltas(d, 7), g["delta_w7"], name="d7")
    for lf, rf in ((5, 5), (0, 2), (3, 1), (0, 0)):
        assert_close(OF.context_window(d, lf, rf), g[f"cw_{lf}_{rf}"], name=f"cw{lf}{rf}")
    # tests/unittests/test_features.py:4-39
    assert torch.equal(OF.deltas(torch.ones(10, 101, 20)), torch.zeros(10, 101, 20))
    cw = OF.context_window(torch.tensor([1.0, 2, 3]).view(1, 3, 1), 1, 1)
    assert torch.equal(cw, torch.tensor([[[0.0, 1, 2], [1, 2, 3], [2, 3, 0]]]))


def test_mfcc_fbank_composites(golden):
    g = golden("features")
    x = torch.from_numpy(g["x"])
    assert_close(OF.mfcc(x), g["mfcc"], name="mfcc")
    assert_close(OF.fbank(x, True, True, n_mels=40, left_frames=2, right_frames=2), g["fbank_dc"], name="fbdc")


@pytest.mark.parametrize("n_mels", [80, 40])
def test_fbank_on_reference_wavs(golden, n_mels):
    g = golden("fbank_wavs")
    for i in range(3):
        w = torch.from_numpy(g[f"pcm{i}"].astype(np.float32) / 32768.0)[None]
        assert_close(OF.fbank(w, n_mels=n_mels), g[f"fbank{n_mels}_single{i}"], name=f"wav{i}")
    L = max(len(g[f"pcm{i}"]) for i in range(3))
    batch = torch.zeros(3, L)
    for i in range(3):
        p = g[f"pcm{i}"]
        batch[i, :len(p)] = torch.from_numpy(p.astype(np.float32) / 32768.0)
    assert_close(OF.fbank(batch, n_mels=n_mels), g[f"fbank{n_mels}_batch"], name="batch")


CFGS = {
    "recipe": dict(time_warp_on=True, time_warp_window=5, freq_mask=True, n_freq_mask=2, time_mask=True,
                   n_time_mask=2, replace_with_zero=False, freq_mask_width=30, time_mask_width=40),
    "default": dict(),
    "nowarp": dict(time_warp_on=False, freq_mask_width=(5, 15), time_mask_width=(10, 20), n_freq_mask=3,
                   n_time_mask=1),
}


@pytest.mark.parametrize("cfg", list(CFGS))
def test_specaugment(golden, cfg):
    g = golden("specaug")
    feats = torch.from_numpy(g["feats"])
    for s in range(4):
        torch.manual_seed(s)
        y = OA.spec_augment(feats.clone(), **CFGS[cfg])
        assert_close(y, g[f"{cfg}_s{s}"], rtol=1e-5, name=f"{cfg}{s}")
        # masked cells are exactly the fill value: indices are bit-exact
        ref = g[f"{cfg}_s{s}"]
        if cfg == "nowarp":
            assert np.array_equal(y.numpy(), ref)


def test_specaugment_draw_order(golden):
    """The oracle's randint sequence equals the one recorded from the reference."""
    g = golden("specaug")
    feats = torch.from_numpy(g["feats"])
    for s in range(4):
        draws = []
        real = torch.randint

        def rec(*a, **k):
            r = real(*a, **k)
            draws.append(r.reshape(-1).numpy().astype(np.int64))
            return r
        torch.randint = rec
        try:
            torch.manual_seed(s)
            OA.spec_augment(feats.clone(), **CFGS["recipe"])
        finally:
            torch.randint = real
        assert np.array_equal(np.concatenate(draws), g[f"recipe_s{s}_draws"])


def test_time_warp(golden):
    g = golden("specaug")
    feats = torch.from_numpy(g["feats"])
    for s in range(4):
        torch.manual_seed(100 + s)
        y = OA.spec_augment(feats.clone(), freq_mask=False, time_mask=False)
        assert_close(y, g[f"warp_s{s}"], rtol=1e-5, name=f"warp{s}")


def _sub(g, prefix):
    return {k[len(prefix):]: torch.from_numpy(g[k]) for k in g.files if k.startswith(prefix)}


def test_conformer_path(golden):
    g = golden("conformer")
    c = OC.conv_frontend(torch.from_numpy(g["feats"]), _sub(g, "cnn."))
    assert_close(c, g["cnn_out"], rtol=1e-5, name="cnn")
    tr = _sub(g, "tr.")
    cnn_out = torch.from_numpy(g["cnn_out"])
    assert_close(OC.transformer_asr_encode(cnn_out, tr, "", 2, 4, torch.from_numpy(g["wav_len"])),
                 g["enc_out"], rtol=1e-5, name="enc")
    assert_close(OC.transformer_asr_encode(cnn_out, tr, "", 2, 4), g["enc_out_nolen"], rtol=1e-5)


def test_conformer_encoder_direct(golden):
    g = golden("conformer")
    pe = OC.rel_pos_enc_xl(37, 64)
    assert_close(pe, g["enc_pos"], rtol=1e-6, name="pe")
    y, at = OC.conformer_encoder(torch.from_numpy(g["enc_src"]), pe, _sub(g, "enc."), "", 2, 4,
                                 key_padding_mask=torch.from_numpy(g["enc_kpm"]))
    assert_close(y, g["enc_y"], rtol=1e-5, name="y")
    assert_close(at[0], g["enc_attn0"], rtol=1e-5)
    assert_close(at[1], g["enc_attn1"], rtol=1e-5)
    yc, _ = OC.conformer_encoder(torch.from_numpy(g["enc_src"]), pe, _sub(g, "encc."), "", 1, 2,
                                 kernel_size=7, causal=True)
    assert_close(yc, g["encc_y"], rtol=1e-5, name="causal")
    assert_close(OC.rel_shift(torch.from_numpy(g["relshift_in"])), g["relshift_out"], rtol=0)


INORM_CASES = {"global": dict(norm_type="global"), "global_avg": dict(norm_type="global", avg_factor=0.1),
               "batch": dict(norm_type="batch"), "sentence": dict(norm_type="sentence"),
               "speaker": dict(norm_type="speaker"), "global_nostd": dict(norm_type="global", std_norm=False),
               "global_until1": dict(norm_type="global", update_until_epoch=1)}


@pytest.mark.parametrize("name", list(INORM_CASES))
def test_input_normalization_oracle(golden, name):
    """oracle.features.InputNormalization vs the reference run (inputnorm.npz):
    12 training batches over 3 epochs (running statistics) then eval."""
    g = golden("inputnorm")
    m = OF.InputNormalization(**INORM_CASES[name])
    for epoch in range(3):
        for i in range(4):
            y = m(torch.from_numpy(g[f"x{i}"]).clone(), torch.from_numpy(g[f"len{i}"]),
                  spk_ids=torch.from_numpy(g[f"spk{i}"]), epoch=epoch)
            if epoch != 1:
                assert_close(y, g[f"{name}_train_e{epoch}_b{i}"], rtol=1e-5, name=f"e{epoch} b{i}")
    if name.startswith("global"):
        assert m.count == int(g[f"{name}_count"])
        assert_close(m.glob_mean, g[f"{name}_glob_mean"], rtol=1e-6)
    m.training = False
    y = m(torch.from_numpy(g["x0"]).clone(), torch.from_numpy(g["len0"]), spk_ids=torch.from_numpy(g["spk0"]), epoch=5)
    assert_close(y, g[f"{name}_eval_b0"], rtol=1e-5, name="eval")


def test_conformer_grads_vs_reference(golden):
    """Oracle autograd (CPU restatement) vs the reference's own gradients
    (train.npz): pins the checker used by tests/test_gpu_train.py."""
    g = golden("conformer")
    gt = golden("train")
    sd_c = {k: v.clone().requires_grad_(True) for k, v in _sub(g, "cnn.").items()}
    sd_t = {k: v.clone().requires_grad_(True) for k, v in _sub(g, "tr.").items()}
    feats = torch.from_numpy(g["feats"]).clone().requires_grad_(True)
    y = OC.transformer_asr_encode(OC.conv_frontend(feats, sd_c), sd_t, "", 2, 4, torch.from_numpy(g["wav_len"]))
    assert_close(y, gt["y"], rtol=1e-5, name="y")
    (y * torch.from_numpy(gt["R"])).sum().backward()
    pairs = [("grad_feats", feats)] + [("grad.cnn." + k, v) for k, v in sd_c.items()] + \
        [("grad.tr." + k, v) for k, v in sd_t.items()]
    n = 0
    for key, t in pairs:
        if key in gt.files:
            ref = gt[key]
            err = np.abs(t.grad.numpy() - ref).max()
            assert err <= 1e-5 * max(np.abs(ref).max(), 1e-12), (key, err)
            n += 1
    assert n == len([k for k in gt.files if k.startswith("grad")])


KAT_LOGITS = np.array([[[[0.1, 0.6, 0.1, 0.1, 0.1], [0.1, 0.1, 0.6, 0.1, 0.1], [0.1, 0.1, 0.2, 0.8, 0.1]],
                        [[0.1, 0.6, 0.1, 0.1, 0.1], [0.1, 0.1, 0.2, 0.1, 0.1], [0.7, 0.1, 0.2, 0.1, 0.1]]]],
                      np.float32)


def test_rnnt_known_answer():
    """tests/unittests/test_losses.py:109-152: exact float equality."""
    lp = torch.from_numpy(KAT_LOGITS).log_softmax(-1).numpy()
    loss, _ = OR.transducer_loss(lp, np.array([[1, 2]]), np.array([1.0]), np.array([1.0]), 0)
    assert float(loss) == 2.247833251953125


def test_rnnt_brute_force():
    rng = np.random.default_rng(0)
    for _ in range(4):
        B, T, U, V = 3, 5, 3, 6
        lp = OR.log_softmax(rng.standard_normal((B, T, U + 1, V))).astype(np.float32)
        lab = rng.integers(1, V, (B, U))
        Tb, Ub = np.array([5, 4, 2]), np.array([3, 1, 2])
        loss, grads, alpha, beta = OR.transducer_forward(lp, lab, Tb, Ub, 0, "none", np.float64)
        for b in range(B):
            bf = OR.brute_force_nll(lp[b], lab[b], Tb[b], Ub[b], 0)
            assert abs(loss[b] * Tb[b] - bf) < 1e-9
            assert abs(beta[b, 0, 0] + bf) < 1e-9  # log P from β
        # gradient: finite differences of -log P wrt lp (float64)
        b = 0
        eps = 1e-6
        for (t, u, v) in [(0, 0, 0), (2, 1, int(lab[0][1])), (4, 3, 0), (1, 2, 0)]:
            lp2 = lp.astype(np.float64).copy()
            lp2[b, t, u, v] += eps
            l2, _, _, _ = OR.transducer_forward(lp2, lab, Tb, Ub, 0, "none", np.float64)
            fd = (l2[b] - loss[b]) * Tb[b] / eps
            assert abs(fd - grads[b, t, u, v]) < 1e-4


def _sub(g, prefix):
    return {k[len(prefix):]: torch.from_numpy(g[k]) for k in g.files if k.startswith(prefix)}


def test_wav2vec_latent_extractor(golden):
    """oracle/wav2vec.py vs the reference's W2VLatentExtractor (default
    kernels/strides at 64 channels, and a custom 3-layer stack)."""
    import oracle.wav2vec as OW
    g = golden("wav2vec")
    wav = torch.from_numpy(g["wav"])
    sd = _sub(g, "ext.")
    assert_close(OW.latent_extractor(wav, sd), g["latents"], rtol=1e-5, name="latents")
    assert_close(OW.latent_extractor(wav, sd, normalize_signal=False), g["latents_nonorm"], rtol=1e-5, name="nonorm")
    assert np.array_equal(OW.output_lengths([6000, 4500]).numpy(), g["out_lengths"])
    sd2 = _sub(g, "ext2.")
    assert_close(OW.latent_extractor(wav, sd2, kernels=(5, 3, 3), strides=(3, 2, 2)), g["latents2"], rtol=1e-5,
                 name="latents2")


def test_wav2vec_encoder_wrapper_and_transformer(golden):
    import oracle.wav2vec as OW
    g = golden("wav2vec")
    lat = torch.from_numpy(g["latents"])
    sd = _sub(g, "wrap.")
    y = OW.encoder_wrapper(lat, sd, "", 2, 4, wav_lens=torch.from_numpy(g["wav_lens"]))
    assert_close(y, g["embeddings"], rtol=1e-5, name="embeddings")
    assert_close(OW.encoder_wrapper(lat, sd, "", 2, 4), g["embeddings_nolen"], rtol=1e-5, name="nolen")
    assert_close(OW.positional_encoding(37, 64), g["posenc_64"], rtol=0, name="posenc")
    sd2 = _sub(g, "enc2.")
    y2, attn = OW.transformer_encoder(torch.from_numpy(g["enc2_src"]), sd2, "", 2, 2,
                                      key_padding_mask=torch.from_numpy(g["enc2_kpm"]))
    assert_close(y2, g["enc2_y"], rtol=1e-5, name="post-norm relu")
    for i, a in enumerate(attn):
        assert_close(a, g[f"enc2_attn{i}"], rtol=1e-5, name=f"attn{i}")
    sdm = _sub(g, "mha.")
    kv = torch.from_numpy(g["mha_kv"])
    o, w = OW.mha(torch.from_numpy(g["mha_q"]), kv, kv, sdm, "", 4, torch.from_numpy(g["mha_kpm"]))
    assert_close(o, g["mha_out"], rtol=1e-5, name="mha out")
    assert_close(w, g["mha_w"], rtol=1e-5, name="mha weights")


def _xattn_case(g, t):
    """Inputs of one xattn.npz case (gen_golden.gen_xattn) as torch tensors."""
    E, H, vbias, ql, kl, same_kv, mpf, has_kpm, am_kind = (int(x) for x in g[f"{t}.meta"])
    pre = f"{t}.sd."
    sd = {k[len(pre):]: torch.from_numpy(g[k]) for k in g.files if k.startswith(pre)}
    q, k = torch.from_numpy(g[f"{t}.q"]), torch.from_numpy(g[f"{t}.k"])
    v = k if same_kv else torch.from_numpy(g[f"{t}.v"])
    kpm = torch.from_numpy(g[f"{t}.kpm"]) if has_kpm else None
    am = torch.from_numpy(g[f"{t}.am"]) if am_kind else None
    return dict(E=E, H=H, vbias=bool(vbias), mpf=bool(mpf), sd=sd, q=q, k=k, v=v, same_kv=bool(same_kv),
                pe=torch.from_numpy(g[f"{t}.pe"]), kpm=kpm, am=am, R=torch.from_numpy(g[f"{t}.R"]))


def test_relpos_cross_attention_oracle(golden):
    """The cross-length RelPosMHAXL restatement (oracle.conformer.rel_pos_mha_cross)
    against the reference on test_attention.py's 16 combinations and the
    masked / causal / key != value cases, outputs, attention maps and
    gradients."""
    g = golden("xattn")
    for t in g["cases"]:
        c = _xattn_case(g, t)
        sd = {k: v.clone().requires_grad_(True) for k, v in c["sd"].items()}
        q, k = c["q"].clone().requires_grad_(True), c["k"].clone().requires_grad_(True)
        v = k if c["same_kv"] else c["v"].clone().requires_grad_(True)
        o, a = OC.rel_pos_mha_cross(q, k, v, c["pe"], sd, "", c["H"], c["vbias"], c["mpf"], c["kpm"], c["am"])
        assert_close(o, g[f"{t}.out"], rtol=1e-5, name=f"{t} out")
        assert_close(a, g[f"{t}.attn"], rtol=1e-5, name=f"{t} attn")
        (o * c["R"]).sum().backward()
        assert_close(q.grad, g[f"{t}.grad_q"], rtol=1e-5, name=f"{t} grad_q")
        assert_close(k.grad, g[f"{t}.grad_k"], rtol=1e-5, name=f"{t} grad_k")
        if not c["same_kv"]:
            assert_close(v.grad, g[f"{t}.grad_v"], rtol=1e-5, name=f"{t} grad_v")
        for name, p in sd.items():
            if f"{t}.grad.{name}" in g.files:
                assert_close(p.grad, g[f"{t}.grad.{name}"], rtol=1e-5, name=f"{t} grad {name}")
