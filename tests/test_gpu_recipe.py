"""Recipe-level drop-ins on the HIP kernels against outputs of the reference
itself (tests/golden/recipe.npz, made by tests/golden/gen_golden.py):

  * Fbank(n_mels=80) on all 12 tests/samples/ASR WAVs (lobes/features.py:82-147);
  * Filterbank(param_rand_factor=0.1) in training mode: the per-call
    torch.rand(2) jitter of central frequencies and bands drawn from the CPU
    generator in the reference's order (processing/features.py:525-532);
  * the standalone Conv2d (nnet/CNN.py:616-700): "same" reflect padding at
    stride 1 and (2, 1) with a non-square kernel, "valid", a 3-D input —
    outputs and every gradient;
  * TransformerASR with a 2-layer decoder: strict checkpoint load, encode()
    on HIP, forward() (encoder + decoder) and decode()
    (lobes/models/transformer/TransformerASR.py:87-300);
  * Brain.fit_batch (core.py:882-994): six reference steps with SGD, gradient
    accumulation 2, max_grad_norm 5.0 (clipping active: the gradient norm is
    far above 5) and a NaN loss on a stepping batch (skipped step,
    nonfinite_count 1) — the parameters after both optimizer steps that ran.

fp32 tolerance as everywhere: |a - b| <= 1e-4 * max(1, |b|); gradients within
1e-4 of the tensor's largest reference gradient; Brain parameters within 1e-4
of the largest parameter change the reference made (plus 2 fp32 ulp of the
parameter)."""
import numpy as np
import pytest
import torch

from conftest import assert_close

pytestmark = pytest.mark.gpu


def assert_grad(a, b, rtol=1e-4, name=""):
    a = a.detach().float().cpu()
    b = torch.as_tensor(b).float()
    assert a.shape == b.shape, f"{name}: shape {tuple(a.shape)} != {tuple(b.shape)}"
    scale = max(b.abs().max().item(), 1e-12)
    err = (a - b).abs().max().item()
    assert err <= rtol * scale, f"{name}: max err {err:.3e} vs scale {scale:.3e}"


def test_fbank_all_sample_wavs(golden, dev):
    from speechbrain_amd.lobes.features import Fbank
    g = golden("recipe")
    fb = Fbank(n_mels=80).to(dev).eval()
    names = [str(n) for n in g["wav_names"]]
    assert len(names) == 12
    with torch.no_grad():
        for n in names:
            wav = torch.from_numpy(g[f"pcm.{n}"].astype(np.float32) / 32768.0)[None].to(dev)
            assert_close(fb(wav), g[f"fbank80.{n}"], name=f"Fbank {n}")


def test_filterbank_param_rand_factor(golden, dev):
    from speechbrain_amd.processing.features import Filterbank
    g = golden("recipe")
    spec = torch.from_numpy(g["fbj_spec"]).to(dev)
    fb = Filterbank(n_mels=40, param_rand_factor=0.1).to(dev).train()
    with torch.no_grad():
        for sd in range(3):
            torch.manual_seed(sd)
            assert_close(fb(spec), g[f"fbj_train_s{sd}"], name=f"jittered Filterbank seed {sd}")
        fb.eval()
        assert_close(fb(spec), g["fbj_eval"], name="Filterbank eval (no jitter)")
    # the jitter really moved the filters (the fixture is not the eval output)
    assert np.abs(g["fbj_train_s0"] - g["fbj_eval"]).max() > 1e-2


CONVS = {
    "c33": dict(out_channels=5, kernel_size=(3, 3), input_shape=(2, 21, 13, 3)),
    "c53s21": dict(out_channels=6, kernel_size=(5, 3), stride=(2, 1), input_shape=(2, 19, 16, 4)),
    "cvalid": dict(out_channels=4, kernel_size=(3, 5), padding="valid", input_shape=(2, 17, 12, 2)),
    "c3d": dict(out_channels=3, kernel_size=(3, 3), input_shape=(2, 15, 11)),
}


@pytest.mark.parametrize("tag", list(CONVS))
def test_conv2d_standalone(golden, dev, tag):
    from speechbrain_amd.nnet.CNN import Conv2d
    g = golden("recipe")
    conv = Conv2d(**CONVS[tag])
    conv.load_state_dict({k[len(tag) + 1:]: torch.from_numpy(g[k]) for k in g.files if k.startswith(tag + ".")},
                         strict=True)
    conv = conv.to(dev)
    with torch.no_grad():
        assert_close(conv(torch.from_numpy(g[f"{tag}_x"]).to(dev)), g[f"{tag}_y"], name=f"{tag} no-grad")
    x = torch.from_numpy(g[f"{tag}_x"]).to(dev).requires_grad_(True)
    y = conv(x)
    assert_close(y, g[f"{tag}_y"], name=tag)
    (y * torch.from_numpy(g[f"{tag}_R"]).to(dev)).sum().backward()
    assert_grad(x.grad, g[f"{tag}_grad_x"], name=f"{tag} dx")
    for k, p in conv.named_parameters():
        assert_grad(p.grad, g[f"{tag}_grad.{k}"], name=f"{tag} d{k}")


def _asr(g):
    from speechbrain_amd.lobes.models.transformer.TransformerASR import TransformerASR
    asr = TransformerASR(tgt_vocab=31, input_size=40, d_model=64, nhead=4, num_encoder_layers=2,
                         num_decoder_layers=2, d_ffn=128, dropout=0.1, activation=torch.nn.GELU,
                         encoder_module="conformer", attention_type="RelPosMHAXL", normalize_before=True,
                         causal=False)
    sd = asr.state_dict()
    for k in sd:
        if "asr." + k in g.files:
            sd[k] = torch.from_numpy(g["asr." + k])
    asr.load_state_dict(sd, strict=True)
    return asr


def test_transformer_asr_with_decoder(golden, dev):
    g = golden("recipe")
    asr = _asr(g).to(dev).eval()
    src = torch.from_numpy(g["asr_src"]).to(dev)
    tgt = torch.from_numpy(g["asr_tgt"]).to(dev)
    wl = torch.from_numpy(g["asr_wav_len"]).to(dev)
    with torch.no_grad():
        assert_close(asr.encode(src, wl), g["asr_enc"], name="encode")
        enc_out, dec_out = asr(src, tgt, wl)
        assert_close(enc_out, g["asr_fwd_enc"], name="forward encoder_out")
        assert_close(dec_out, g["asr_fwd_dec"], name="forward decoder_out")
        pred, att = asr.decode(tgt, torch.from_numpy(g["asr_enc"]).to(dev),
                               torch.from_numpy(g["asr_enc_len"]).to(dev))
        assert_close(pred, g["asr_dec_pred"], name="decode prediction")
        assert_close(att, g["asr_dec_att"], name="decode attention")


def test_brain_step_matches_reference(golden, dev):
    """speechbrain_amd.core.Brain against six reference fit_batch calls."""
    import speechbrain_amd.core as C
    from speechbrain_amd.lobes.models.convolution import ConvolutionFrontEnd
    from speechbrain_amd.lobes.models.transformer.TransformerASR import TransformerASR
    g, g0 = golden("recipe"), golden("conformer")
    cnn = ConvolutionFrontEnd(input_shape=(8, 10, 80), num_blocks=2, num_layers_per_block=1, out_channels=(64, 32),
                              kernel_sizes=(3, 3), strides=(2, 2), residuals=(False, False), dropout=0.0)
    tr = TransformerASR(tgt_vocab=10, input_size=640, d_model=64, nhead=4, num_encoder_layers=2,
                        num_decoder_layers=0, d_ffn=128, dropout=0.0, encoder_module="conformer",
                        attention_type="RelPosMHAXL", normalize_before=True, causal=False)
    for pre, m in (("cnn.", cnn), ("tr.", tr)):
        m.load_state_dict({k[len(pre):]: torch.from_numpy(g0[k]) for k in g0.files if k.startswith(pre)})
    init = {f"{pre}{k}": p.detach().clone() for pre, m in (("cnn.", cnn), ("tr.", tr))
            for k, p in m.named_parameters()}

    class StepBrain(C.Brain):
        def compute_forward(self, batch, stage):
            feats, wl, _, _ = batch
            return self.modules.tr.encode(self.modules.cnn(feats), wl)

        def compute_objectives(self, y, batch, stage):
            _, _, tgt, bad = batch
            loss = 0.5 * ((y - tgt) ** 2).sum()
            return loss * float("nan") if bad else loss

    brain = StepBrain(modules={"cnn": cnn, "tr": tr}, opt_class=lambda ps: torch.optim.SGD(ps, lr=0.01),
                      run_opts={"device": str(dev), "grad_accumulation_factor": 2, "max_grad_norm": 5.0})
    brain.modules.train()
    wl = torch.from_numpy(g["brain_wav_len"]).to(dev)
    for i in range(6):
        batch = (torch.from_numpy(g[f"brain_feats{i}"]).to(dev), wl, torch.from_numpy(g[f"brain_tgt{i}"]).to(dev),
                 i == 3)
        loss = float(brain.fit_batch(batch))
        ref_loss = float(g[f"brain_loss{i}"])
        if i == 3:
            assert np.isnan(loss) and np.isnan(ref_loss)
        else:
            assert abs(loss - ref_loss) <= 1e-4 * abs(ref_loss), (i, loss, ref_loss)
        assert [brain.step, brain.optimizer_step, brain.nonfinite_count] == g[f"brain_state{i}"].tolist(), i
        psum = sum(float((p.detach().double() ** 2).sum()) for p in brain.modules.parameters())
        assert abs(psum - float(g[f"brain_psum{i}"])) <= 1e-5 * float(g[f"brain_psum{i}"]), (i, psum)
        if i in (1, 5):
            for pre, m in (("cnn.", cnn), ("tr.", tr)):
                for k, p in m.named_parameters():
                    ref = torch.from_numpy(g[f"brain_p{i}.{pre}{k}"])
                    step = (ref - init[pre + k].cpu()).abs().max().item()
                    err = (p.detach().cpu() - ref).abs().max().item()
                    # 1e-4 of the update the reference made, plus the fp32 rounding
                    # of the parameter itself (2 ulp of its largest element)
                    tol = 1e-4 * step + 2.4e-7 * ref.abs().max().item()
                    assert err <= tol, f"after batch {i}: {pre}{k} err {err:.3e} step {step:.3e}"
