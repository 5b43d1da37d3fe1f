"""Integration test in the style of the reference's
tests/integration/ASR_Transducer/example_asr_transducer_experiment.py:134-175
(a tiny model trained on tests/samples audio, loss threshold): the three
committed sample utterances (tests/golden/fbank_wavs.npz, PCM from the
reference's tests/samples/ASR) through Fbank -> InputNormalization ->
ConvolutionFrontEnd -> 2-layer Conformer -> transducer joint -> RNN-T loss,
trained with speechbrain_amd.core.Brain (fp32 and bf16 autocast).  The
model must overfit the fixed label sequences: final loss < 30 % of the first."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _batch(golden, dev):
    g = golden("fbank_wavs")
    pcms = [g[f"pcm{i}"].astype(np.float32) / 32768.0 for i in range(3)]
    L = max(len(p) for p in pcms)
    wav = torch.zeros(3, L)
    for i, p in enumerate(pcms):
        wav[i, :len(p)] = torch.from_numpy(p)
    wav_lens = torch.tensor([len(p) / L for p in pcms], dtype=torch.float32)
    gen = torch.Generator().manual_seed(0)
    U = torch.tensor([6, 4, 5])
    tokens = torch.randint(1, 20, (3, 6), generator=gen)
    tokens[torch.arange(6)[None] >= U[:, None]] = 0
    return (wav.to(dev), wav_lens.to(dev), F.pad(tokens, (1, 0)).to(dev), tokens.to(dev), (U / 6.0).to(dev))


@pytest.mark.parametrize("amp", [False, "bf16"])
def test_tiny_transducer_overfits(golden, dev, amp):
    from speechbrain_amd.core import Brain, Stage
    from speechbrain_amd.lobes.features import Fbank
    from speechbrain_amd.lobes.models.convolution import ConvolutionFrontEnd
    from speechbrain_amd.lobes.models.transformer.TransformerASR import TransformerASR
    from speechbrain_amd.nnet.linear import Linear
    from speechbrain_amd.nnet.losses import transducer_loss
    from speechbrain_amd.nnet.transducer.transducer_joint import Transducer_joint
    from speechbrain_amd.processing.features import InputNormalization
    V, J, d = 20, 64, 256
    torch.manual_seed(0)
    mods = {"CNN": ConvolutionFrontEnd(input_shape=(8, 10, 80), num_blocks=2, num_layers_per_block=1,
                                       out_channels=(64, 32), kernel_sizes=(3, 3), strides=(2, 2),
                                       residuals=(False, False), dropout=0.0),
            "enc": TransformerASR(tgt_vocab=V, input_size=640, d_model=d, nhead=4, num_encoder_layers=2,
                                  num_decoder_layers=0, d_ffn=512, dropout=0.0, encoder_module="conformer",
                                  attention_type="RelPosMHAXL", normalize_before=True, causal=False),
            "enc_lin": Linear(input_size=d, n_neurons=J),
            "dec": torch.nn.GRU(V - 1, J, batch_first=True),
            "dec_lin": Linear(input_size=J, n_neurons=J, bias=False),
            "Tjoint": Transducer_joint(joint="sum", nonlinearity=torch.nn.LeakyReLU),
            "out": Linear(input_size=J, n_neurons=V, bias=False)}
    hp = {"fbank": Fbank(n_mels=80).to(dev), "norm": InputNormalization().to(dev)}

    class TinyBrain(Brain):
        def compute_forward(self, batch, stage):
            wav, wl, bos, _, _ = batch
            with torch.no_grad():
                feats = self.hparams["norm"](self.hparams["fbank"](wav), wl)
            x = self.modules.enc.encode(self.modules.CNN(feats), wl)
            tn = self.modules.enc_lin(x)
            pn = self.modules.dec_lin(self.modules.dec(F.one_hot(bos, V)[..., 1:].float())[0])
            return self.modules.out(self.modules.Tjoint(tn.unsqueeze(2), pn.unsqueeze(1)))

        def compute_objectives(self, logits, batch, stage):
            _, wl, _, tok, tl = batch
            return transducer_loss(logits.float(), tok, wl, tl, blank_index=0, use_torchaudio=True)

    brain = TinyBrain(modules=mods, opt_class=lambda p: torch.optim.Adam(p, lr=3e-4), hparams=hp,
                      run_opts={"device": str(dev), "auto_mix_prec": amp, "max_grad_norm": 5.0})
    for m in brain.modules.values():
        m.train()
    batch = _batch(golden, dev)
    losses = [float(brain.fit_batch(batch)) for _ in range(40)]
    assert all(np.isfinite(losses)), losses
    assert losses[-1] < 0.3 * losses[0], losses
    ev = float(brain.evaluate_batch(batch, Stage.VALID))
    assert np.isfinite(ev) and ev < 0.5 * losses[0]
