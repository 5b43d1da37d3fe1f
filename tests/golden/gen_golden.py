"""Generate the golden fixtures under tests/golden/ from the REAL reference.

Runs only in the build container (the reference at /root/reference never
travels to the GPU box); the committed .npz files are what the tests read.

    python tests/golden/gen_golden.py

The reference imports three packages that are absent here and unused by the
hot-path arithmetic (hyperpyyaml, torchaudio, ruamel.yaml), so
they are replaced by inert stub modules before `import speechbrain`.  WAVs
are read with the stdlib `wave` module and scaled by 1/32768, the same
normalisation torchaudio.load applies (speechbrain/dataio/dataio.py:216-250).

Fixture inventory (all float32 unless noted):
  fbank_wavs.npz   Fbank(n_mels=80|40) on 3 tests/samples/ASR WAVs, single
                   and zero-padded batch (lobes/features.py:82-147)
  features.npz     STFT (mono + 3-channel), spectral_magnitude, Filterbank
                   (3 shapes, log/linear, freeze=False + grads), DCT,
                   Deltas, ContextWindow, MFCC, Fbank(deltas, context)
                   (processing/features.py:50-937)
  specaug.npz      SpecAugment outputs + every randint draw it made
                   (lobes/augment.py:32-201)
  conformer.npz    ConvolutionFrontEnd + TransformerASR.encode (Conformer,
                   RelPosMHAXL) weights, inputs, outputs, attention maps,
                   RelPosEncXL and rel_shift vectors
                   (lobes/models/convolution.py, lobes/models/transformer/*,
                   nnet/attention.py)
  inputnorm.npz    InputNormalization (global / batch / sentence / speaker,
                   training and eval, running statistics over 4 batches and
                   3 epochs, ragged relative lengths incl. one-frame and
                   rounding-tie lengths) (processing/features.py:940-1231)
  wav2vec.npz      W2VLatentExtractor (default 7-layer stack at 64 channels and a
                   small custom one), EncoderWrapper + TransformerEncoder
                   (pre-norm GELU and post-norm ReLU), MultiheadAttention with
                   a key padding mask, PositionalEncoding — config 5 modules
                   (lobes/models/wav2vec.py:28-106,153-227,
                   lobes/models/transformer/Transformer.py:201-486,
                   nnet/attention.py:642-778)
  decoder.npz      TransducerBeamSearcher greedy and beam search on a small
                   random one-hot-Embedding / GRU / Linear transducer
                   (decoders/transducer.py:10-519)
  dropin.npz       constructor coverage beyond the recipe: the default
                   ConvolutionFrontEnd(input_shape) (3 residual blocks x 5
                   layers; seeded-init checksums and output), a small
                   residual / multi-layer / kernel-5 front-end with weights,
                   output and autograd gradients, RelPosMHAXL with a bool
                   causal and a float 3-D attn_mask, SpecAugment bilinear
                   warp (lobes/models/convolution.py:12-175,
                   nnet/attention.py:598-611, lobes/augment.py:116-148)
  recipe.npz       Fbank(80) on all 12 tests/samples/ASR WAVs; Filterbank
                   param_rand_factor jitter (training mode, seeds 0-2);
                   standalone Conv2d (same / strided / valid / 3-D input,
                   outputs and gradients); TransformerASR with a 2-layer
                   decoder (seeded init, state_dict, forward, encode,
                   decode); six reference Brain.fit_batch steps (SGD,
                   grad accumulation 2, clip 5.0, a NaN loss on a stepping
                   batch) with every parameter after each step
                   (lobes/features.py:82-147, processing/features.py:525-532,
                   nnet/CNN.py:504-700, lobes/models/transformer/*,
                   core.py:882-994)
  train.npz        gradients of sum(R * encode(cnn(feats), wav_len)) w.r.t.
                   every ConvolutionFrontEnd / TransformerASR parameter and
                   the input features (reference autograd, weights of
                   conformer.npz), for the training-path backward kernels
The RNN-T known answer (tests/unittests/test_losses.py:109-152) needs numba
and is pinned as a literal in tests/test_oracle_golden.py instead.
"""
import os
import sys
import types
import wave

import numpy as np

sys.dont_write_bytecode = True
REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))


def _install_stubs():
    def stub(name, **attrs):
        m = types.ModuleType(name)
        for k, v in attrs.items():
            setattr(m, k, v)
        sys.modules[name] = m
        return m

    def _raise(*a, **k):
        raise RuntimeError("stubbed dependency")

    ta = stub("torchaudio", set_audio_backend=lambda *a, **k: None,
              load=_raise, save=_raise, info=_raise)
    ta.transforms = stub("torchaudio.transforms")
    ta.functional = stub("torchaudio.functional")
    stub("hyperpyyaml", resolve_references=_raise, load_hyperpyyaml=_raise)
    r = stub("ruamel")
    r.yaml = stub("ruamel.yaml", YAML=_raise)
    sys.path.insert(0, REF)


_install_stubs()
import torch  # noqa: E402

torch.set_num_threads(8)

from speechbrain.processing import features as F  # noqa: E402
from speechbrain.lobes import features as LF  # noqa: E402
from speechbrain.lobes.augment import SpecAugment  # noqa: E402
from speechbrain.lobes.models.convolution import ConvolutionFrontEnd  # noqa: E402
from speechbrain.lobes.models.transformer.TransformerASR import TransformerASR  # noqa: E402
from speechbrain.lobes.models.transformer.Conformer import ConformerEncoder  # noqa: E402
from speechbrain.nnet.attention import RelPosEncXL, RelPosMHAXL  # noqa: E402


def read_wav(name):
    w = wave.open(os.path.join(REF, "tests/samples/ASR", name + ".wav"))
    assert w.getsampwidth() == 2 and w.getnchannels() == 1
    pcm = np.frombuffer(w.readframes(w.getnframes()), dtype="<i2")
    return pcm


def t2n(x):
    return x.detach().cpu().numpy().astype(np.float32)


def gen_fbank_wavs():
    names = ["spk2_snt2", "spk2_snt6", "spk2_snt3"]
    out = {}
    pcms = [read_wav(n) for n in names]
    L = max(len(p) for p in pcms)
    batch = np.zeros((len(pcms), L), np.float32)
    for i, p in enumerate(pcms):
        out[f"pcm{i}"] = p.astype(np.int16)
        batch[i, : len(p)] = p.astype(np.float32) / 32768.0
    for n_mels in (80, 40):
        fb = LF.Fbank(n_mels=n_mels)
        fb.eval()
        with torch.no_grad():
            for i, p in enumerate(pcms):
                wav = torch.from_numpy(p.astype(np.float32) / 32768.0)[None]
                out[f"fbank{n_mels}_single{i}"] = t2n(fb(wav))
            out[f"fbank{n_mels}_batch"] = t2n(fb(torch.from_numpy(batch)))
    np.savez_compressed(os.path.join(OUT, "fbank_wavs.npz"), **out)


def gen_features():
    out = {}
    g = torch.Generator().manual_seed(0)
    x = 0.1 * torch.randn(2, 16000, generator=g)
    x3 = 0.1 * torch.randn(2, 4000, 3, generator=g)
    out["x"] = t2n(x)
    out["x3"] = t2n(x3)
    stft = F.STFT(sample_rate=16000)
    s = stft(x)
    out["stft"] = t2n(s)
    out["stft3"] = t2n(stft(x3))
    # non-default STFT geometry: 20 ms window, 5 ms hop, n_fft 512, reflect pad
    stft_b = F.STFT(sample_rate=16000, win_length=20, hop_length=5, n_fft=512,
                    pad_mode="reflect")
    out["stft_b"] = t2n(stft_b(x))
    mag = F.spectral_magnitude(s)
    out["mag_p1"] = t2n(mag)
    out["mag_p05"] = t2n(F.spectral_magnitude(s, power=0.5))
    out["mag_log"] = t2n(F.spectral_magnitude(s, power=1, log=True))
    for shape in ("triangular", "rectangular", "gaussian"):
        fbm = F.Filterbank(n_mels=40, filter_shape=shape)
        out[f"fb_{shape}"] = t2n(fbm(mag))
    out["fb_lin"] = t2n(F.Filterbank(n_mels=23, log_mel=False)(mag))
    out["fb_80"] = t2n(F.Filterbank(n_mels=80)(mag))
    out["fb_fmin_fmax"] = t2n(F.Filterbank(n_mels=40, f_min=100, f_max=7000)(mag))
    # learnable filterbank: forward + grads of sum() wrt f_central/band
    fbl = F.Filterbank(n_mels=40, freeze=False)
    y = fbl(mag)
    y.sum().backward()
    out["fb_learn"] = t2n(y)
    out["fb_learn_grad_fc"] = t2n(fbl.f_central.grad)
    out["fb_learn_grad_band"] = t2n(fbl.band.grad)
    # multichannel filterbank (B,T,F,C)
    out["fb_multi"] = t2n(F.Filterbank(n_mels=40)(F.spectral_magnitude(stft(x3))))
    fbank40 = out["fb_triangular"]
    dct = F.DCT(input_size=40, n_out=20)
    d = dct(torch.from_numpy(fbank40))
    out["dct"] = t2n(d)
    out["dct_noortho"] = t2n(F.DCT(input_size=40, n_out=13, ortho_norm=False)(torch.from_numpy(fbank40)))
    deltas = F.Deltas(input_size=20)
    d1 = deltas(d)
    out["delta1"] = t2n(d1)
    out["delta2"] = t2n(deltas(d1))
    out["delta_w7"] = t2n(F.Deltas(input_size=20, window_length=7)(d))
    for lf, rf in ((5, 5), (0, 2), (3, 1), (0, 0)):
        cw = F.ContextWindow(left_frames=lf, right_frames=rf)
        out[f"cw_{lf}_{rf}"] = t2n(cw(d))
    mf = LF.MFCC()
    out["mfcc"] = t2n(mf(x))
    fbdc = LF.Fbank(n_mels=40, deltas=True, context=True, left_frames=2, right_frames=2)
    out["fbank_dc"] = t2n(fbdc(x))
    np.savez_compressed(os.path.join(OUT, "features.npz"), **out)


def gen_specaug():
    """Run the reference SpecAugment, recording every torch.randint draw."""
    out = {}
    g = torch.Generator().manual_seed(123)
    feats = torch.randn(4, 150, 80, generator=g)
    out["feats"] = t2n(feats)
    real_randint = torch.randint
    draws = []

    def rec_randint(*a, **k):
        r = real_randint(*a, **k)
        draws.append(r.detach().cpu().numpy().reshape(-1).astype(np.int64))
        return r

    configs = {
        # conformer_small.yaml:252-262
        "recipe": dict(time_warp=True, time_warp_window=5, time_warp_mode="bicubic",
                       freq_mask=True, n_freq_mask=2, time_mask=True, n_time_mask=2,
                       replace_with_zero=False, freq_mask_width=30, time_mask_width=40),
        "default": dict(),
        "nowarp": dict(time_warp=False, freq_mask_width=(5, 15), time_mask_width=(10, 20),
                       n_freq_mask=3, n_time_mask=1),
    }
    torch.randint = rec_randint
    try:
        for name, cfg in configs.items():
            for seed in range(4):
                aug = SpecAugment(**cfg)
                torch.manual_seed(seed)
                draws.clear()
                y = aug(feats.clone())
                out[f"{name}_s{seed}"] = t2n(y)
                out[f"{name}_s{seed}_draws"] = np.concatenate(draws)
    finally:
        torch.randint = real_randint
    # time-warp only, to pin the bicubic resample in isolation
    aug = SpecAugment(time_warp=True, freq_mask=False, time_mask=False)
    for seed in range(4):
        torch.manual_seed(100 + seed)
        out[f"warp_s{seed}"] = t2n(aug(feats.clone()))
    np.savez_compressed(os.path.join(OUT, "specaug.npz"), **out)


def gen_conformer():
    out = {}
    torch.manual_seed(0)
    # recipe front-end (conformer_small.yaml:123-130)
    cnn = ConvolutionFrontEnd(input_shape=(8, 10, 80), num_blocks=2, num_layers_per_block=1,
                              out_channels=(64, 32), kernel_sizes=(3, 3), strides=(2, 2),
                              residuals=(False, False))
    tr = TransformerASR(tgt_vocab=10, input_size=640, d_model=64, nhead=4,
                        num_encoder_layers=2, num_decoder_layers=0, d_ffn=128,
                        dropout=0.0, encoder_module="conformer",
                        attention_type="RelPosMHAXL", normalize_before=True,
                        causal=False)
    cnn.eval()
    tr.eval()
    for k, v in cnn.state_dict().items():
        out["cnn." + k] = t2n(v)
    for k, v in tr.state_dict().items():
        out["tr." + k] = t2n(v)
    g = torch.Generator().manual_seed(1)
    feats = torch.randn(2, 101, 80, generator=g)
    wav_len = torch.tensor([1.0, 0.8])
    out["feats"] = t2n(feats)
    out["wav_len"] = t2n(wav_len)
    with torch.no_grad():
        c = cnn(feats)
        out["cnn_out"] = t2n(c)
        out["enc_out"] = t2n(tr.encode(c, wav_len))
        out["enc_out_nolen"] = t2n(tr.encode(c))
    # ConformerEncoder directly: returns attention maps too
    torch.manual_seed(2)
    enc = ConformerEncoder(num_layers=2, d_model=64, d_ffn=128, nhead=4, kernel_size=31)
    enc.eval()
    for k, v in enc.state_dict().items():
        out["enc." + k] = t2n(v)
    src = torch.randn(3, 37, 64, generator=g)
    kpm = torch.arange(37)[None, :] >= torch.tensor([37, 30, 21])[:, None]
    pe = RelPosEncXL(64)(src)
    out["enc_src"] = t2n(src)
    out["enc_kpm"] = kpm.numpy()
    out["enc_pos"] = t2n(pe)
    with torch.no_grad():
        y, attn = enc(src, src_key_padding_mask=kpm, pos_embs=pe)
    out["enc_y"] = t2n(y)
    for i, a in enumerate(attn):
        out[f"enc_attn{i}"] = t2n(a)
    # causal conformer (ConvolutionModule chomp; Conformer.py:62-66,108-110)
    torch.manual_seed(3)
    encc = ConformerEncoder(num_layers=1, d_model=64, d_ffn=96, nhead=2, kernel_size=7, causal=True)
    encc.eval()
    for k, v in encc.state_dict().items():
        out["encc." + k] = t2n(v)
    with torch.no_grad():
        yc, _ = encc(src, pos_embs=pe)
    out["encc_y"] = t2n(yc)
    # rel_shift pin: out[i,j] = bd[i, T-1-i+j]
    mha = RelPosMHAXL(embed_dim=64, num_heads=4)
    bd = torch.randn(1, 2, 5, 9, generator=g)
    out["relshift_in"] = t2n(bd)
    out["relshift_out"] = t2n(mha.rel_shift(bd))
    np.savez_compressed(os.path.join(OUT, "conformer.npz"), **out)


def gen_inputnorm():
    out = {}
    g = torch.Generator().manual_seed(11)
    B, T, Fd = 4, 37, 40
    batches = [3.0 * torch.randn(B, T, Fd, generator=g) + 1.5 for _ in range(4)]
    lens = [torch.tensor([1.0, 0.5, 0.8, 0.3]), torch.tensor([1.0, 1.0, 0.9, 0.05]),
            torch.tensor([0.7, 1.0, 0.6, 0.25]), torch.tensor([1.0, 0.2, 1.0, 0.99])]
    spk = [torch.tensor([[0], [1], [0], [2]]), torch.tensor([[1], [1], [3], [0]]),
           torch.tensor([[2], [0], [1], [1]]), torch.tensor([[3], [3], [0], [2]])]
    for i in range(4):
        out[f"x{i}"] = t2n(batches[i])
        out[f"len{i}"] = t2n(lens[i])
        out[f"spk{i}"] = spk[i].numpy()
    cases = {"global": dict(norm_type="global"), "global_avg": dict(norm_type="global", avg_factor=0.1),
             "batch": dict(norm_type="batch"), "sentence": dict(norm_type="sentence"),
             "speaker": dict(norm_type="speaker"), "global_nostd": dict(norm_type="global", std_norm=False),
             "global_until1": dict(norm_type="global", update_until_epoch=1)}
    for name, kw in cases.items():
        m = F.InputNormalization(**kw)
        m.train()
        step = 0
        for epoch in range(3):
            for i in range(4):
                y = m(batches[i].clone(), lens[i], spk_ids=spk[i], epoch=epoch)
                if epoch != 1:
                    out[f"{name}_train_e{epoch}_b{i}"] = t2n(y)
                step += 1
        if kw["norm_type"] == "global":
            out[f"{name}_glob_mean"] = t2n(m.glob_mean)
            out[f"{name}_glob_std"] = t2n(m.glob_std)
            out[f"{name}_count"] = np.array(m.count)
        m.eval()
        out[f"{name}_eval_b0"] = t2n(m(batches[0].clone(), lens[0], spk_ids=spk[0], epoch=5))
    np.savez_compressed(os.path.join(OUT, "inputnorm.npz"), **out)


def gen_train():
    """Reference autograd through ConvolutionFrontEnd + TransformerASR.encode
    (dropout 0, so train and eval arithmetic agree), weights from conformer.npz."""
    g0 = np.load(os.path.join(OUT, "conformer.npz"))
    cnn = ConvolutionFrontEnd(input_shape=(8, 10, 80), num_blocks=2, num_layers_per_block=1,
                              out_channels=(64, 32), kernel_sizes=(3, 3), strides=(2, 2),
                              residuals=(False, False), dropout=0.0)
    tr = TransformerASR(tgt_vocab=10, input_size=640, d_model=64, nhead=4,
                        num_encoder_layers=2, num_decoder_layers=0, d_ffn=128,
                        dropout=0.0, encoder_module="conformer",
                        attention_type="RelPosMHAXL", normalize_before=True,
                        causal=False)
    for pre, m in (("cnn.", cnn), ("tr.", tr)):
        m.load_state_dict({k[len(pre):]: torch.from_numpy(g0[k]) for k in g0.files if k.startswith(pre)})
        m.train()
    out = {}
    feats = torch.from_numpy(g0["feats"]).clone().requires_grad_(True)
    wav_len = torch.from_numpy(g0["wav_len"])
    y = tr.encode(cnn(feats), wav_len)
    R = torch.randn(y.shape, generator=torch.Generator().manual_seed(7))
    (y * R).sum().backward()
    out["R"] = t2n(R)
    out["y"] = t2n(y)
    out["grad_feats"] = t2n(feats.grad)
    for pre, m in (("cnn.", cnn), ("tr.", tr)):
        for k, p in m.named_parameters():
            if p.grad is not None:
                out["grad." + pre + k] = t2n(p.grad)
    np.savez_compressed(os.path.join(OUT, "train.npz"), **out)


def gen_wav2vec():
    from speechbrain.lobes.models.wav2vec import W2VLatentExtractor, EncoderWrapper
    from speechbrain.lobes.models.transformer.Transformer import TransformerEncoder, PositionalEncoding
    from speechbrain.nnet.attention import MultiheadAttention
    out = {}
    g = torch.Generator().manual_seed(11)
    wav = 0.1 * torch.randn(2, 6000, generator=g)
    wav[1, 4500:] = 0.0  # a zero-padded tail
    out["wav"] = t2n(wav)
    torch.manual_seed(4)
    # default kernels / strides (7 layers, k 11/5 then 3/2); 64 channels keep
    # the fixture small (the 512-channel stack is checked against the oracle)
    ext = W2VLatentExtractor(out_channels=[64] * 7)
    ext.eval()
    for k, v in ext.state_dict().items():
        out["ext." + k] = t2n(v)
    with torch.no_grad():
        lat = ext(wav)
        out["latents"] = t2n(lat)
        out["latents_nonorm"] = t2n(ext(wav, normalize_signal=False))
    out["out_lengths"] = ext.get_output_lengths(torch.tensor([6000, 4500])).numpy().astype(np.int64)
    torch.manual_seed(5)
    ext2 = W2VLatentExtractor(out_channels=[32, 32, 48], kernel_sizes=[5, 3, 3], strides=[3, 2, 2])
    ext2.eval()
    for k, v in ext2.state_dict().items():
        out["ext2." + k] = t2n(v)
    with torch.no_grad():
        out["latents2"] = t2n(ext2(wav))
    # encoder wrapper + pre-norm GELU transformer (the wav2vec2 recipe's form,
    # recipes/LibriSpeech/self-supervised-learning/wav2vec2/hparams/wav2vec2_base.yaml:79-93)
    torch.manual_seed(6)
    enc = TransformerEncoder(num_layers=2, nhead=4, d_ffn=128, d_model=64, dropout=0.0,
                             activation=torch.nn.GELU, normalize_before=True)
    wrap = EncoderWrapper(64, 64, enc, dropout_encoder_input=0.0)
    wrap.eval()
    for k, v in wrap.state_dict().items():
        out["wrap." + k] = t2n(v)
    wav_lens = torch.tensor([1.0, 0.7])
    out["wav_lens"] = t2n(wav_lens)
    with torch.no_grad():
        out["embeddings"] = t2n(wrap(lat, wav_lens=wav_lens)["embeddings"])
        out["embeddings_nolen"] = t2n(wrap(lat)["embeddings"])
    # post-norm ReLU TransformerEncoder directly, with attention maps
    torch.manual_seed(7)
    enc2 = TransformerEncoder(num_layers=2, nhead=2, d_ffn=96, d_model=32, dropout=0.0)
    enc2.eval()
    for k, v in enc2.state_dict().items():
        out["enc2." + k] = t2n(v)
    src = torch.randn(3, 19, 32, generator=g)
    kpm = torch.arange(19)[None, :] >= torch.tensor([19, 12, 7])[:, None]
    out["enc2_src"] = t2n(src)
    out["enc2_kpm"] = kpm.numpy()
    with torch.no_grad():
        y, attn = enc2(src, src_key_padding_mask=kpm)
    out["enc2_y"] = t2n(y)
    for i, a in enumerate(attn):
        out[f"enc2_attn{i}"] = t2n(a)
    # MultiheadAttention wrapper alone (cross attention, L != S)
    torch.manual_seed(8)
    mha = MultiheadAttention(nhead=4, d_model=64)
    mha.eval()
    for k, v in mha.state_dict().items():
        out["mha." + k] = t2n(v)
    q = torch.randn(2, 9, 64, generator=g)
    kv = torch.randn(2, 13, 64, generator=g)
    kpm2 = torch.arange(13)[None, :] >= torch.tensor([13, 10])[:, None]
    out["mha_q"], out["mha_kv"], out["mha_kpm"] = t2n(q), t2n(kv), kpm2.numpy()
    with torch.no_grad():
        o, w = mha(q, kv, kv, key_padding_mask=kpm2)
    out["mha_out"], out["mha_w"] = t2n(o), t2n(w)
    out["posenc_64"] = t2n(PositionalEncoding(64)(torch.zeros(1, 37, 64)))
    np.savez_compressed(os.path.join(OUT, "wav2vec.npz"), **out)


def gen_decoder():
    """TransducerBeamSearcher (decoders/transducer.py:10-519) on a small random
    Conformer-Transducer-shaped decoder: one-hot Embedding → GRU → Linear PN,
    "sum" joint + LeakyReLU, Linear classifier; greedy and beam search."""
    import speechbrain as sb
    from speechbrain.decoders.transducer import TransducerBeamSearcher
    from speechbrain.nnet.transducer.transducer_joint import Transducer_joint
    out = {}
    V, J, H, B, T = 7, 16, 10, 3, 12
    torch.manual_seed(9)
    emb = sb.nnet.embedding.Embedding(num_embeddings=V, consider_as_one_hot=True, blank_id=0)
    dec = sb.nnet.RNN.GRU(hidden_size=H, input_shape=(1, 4, V - 1), bidirectional=False)
    dec_lin = sb.nnet.linear.Linear(input_shape=(1, 4, H), n_neurons=J, bias=False)
    tjoint = Transducer_joint(joint="sum", nonlinearity=torch.nn.LeakyReLU)
    cls = sb.nnet.linear.Linear(input_shape=(1, 1, 1, J), n_neurons=V)
    # blank bias per mode: +1.5 gives the greedy decode plenty of emissions;
    # the beam search (no max-symbols-per-frame bound in the reference) only
    # terminates reasonably when blank is usually in the top-k: +3.0
    bias0 = cls.w.bias.detach().clone()
    for name, m in (("emb", emb), ("dec", dec), ("dec_lin", dec_lin), ("cls", cls)):
        for k, v in m.state_dict().items():
            out[f"{name}.{k}"] = t2n(v)
    g = torch.Generator().manual_seed(10)
    tn = 2.0 * torch.randn(B, T, J, generator=g)
    out["tn"] = t2n(tn)
    for beam, tag, db in ((1, "greedy", 1.5), (3, "beam", 3.0)):
        with torch.no_grad():
            cls.w.bias.copy_(bias0)
            cls.w.bias[0] += db
        out[f"{tag}_cls_bias"] = t2n(cls.w.bias)
        searcher = TransducerBeamSearcher(decode_network_lst=[emb, dec, dec_lin], tjoint=tjoint,
                                          classifier_network=[cls], blank_id=0, beam_size=beam, nbest=2,
                                          lm_module=None, lm_weight=0.0, state_beam=2.3, expand_beam=2.3)
        with torch.no_grad():
            hyps, score, nbest, nbest_scores = searcher(tn)
        out[f"{tag}_score"] = np.asarray(float(score), np.float64)
        for b in range(B):
            out[f"{tag}_hyp{b}"] = np.asarray(hyps[b], np.int64)
        if nbest is not None:
            for b in range(B):
                for i, (h, sc) in enumerate(zip(nbest[b], nbest_scores[b])):
                    out[f"{tag}_nbest{b}_{i}"] = np.asarray(h, np.int64)
                    out[f"{tag}_nbest_score{b}_{i}"] = np.asarray(float(sc), np.float64)
    np.savez_compressed(os.path.join(OUT, "decoder.npz"), **out)


def gen_dropin():
    out = {}
    g = torch.Generator().manual_seed(21)
    # 1. ConvolutionFrontEnd with every default (the doctest shape)
    torch.manual_seed(0)
    fe = ConvolutionFrontEnd(input_shape=(8, 30, 10))
    fe.eval()
    for k, v in fe.state_dict().items():
        v64 = v.double()
        out["fe_def_sum." + k] = np.asarray(float(v64.sum()), np.float64)
        out["fe_def_sq." + k] = np.asarray(float((v64 * v64).sum()), np.float64)
    x = torch.rand((8, 30, 10), generator=g)
    with torch.no_grad():
        y = fe(x)
    out["fe_def_x"] = t2n(x)
    out["fe_def_y"] = t2n(y)
    # 2. residual, 2 layers per block, kernel 5, strides (1, 2): weights,
    #    output and gradients of sum(R * y)
    torch.manual_seed(1)
    fe2 = ConvolutionFrontEnd(input_shape=(3, 37, 20), num_blocks=2, num_layers_per_block=2, out_channels=(8, 16),
                              kernel_sizes=(3, 5), strides=(1, 2), residuals=(True, True), dropout=0.1)
    fe2.eval()
    for k, v in fe2.state_dict().items():
        out["fe2." + k] = t2n(v)
    x2 = torch.randn(3, 37, 20, generator=g).requires_grad_(True)
    y2 = fe2(x2)
    R = torch.randn(y2.shape, generator=g)
    (y2 * R).sum().backward()
    out["fe2_x"], out["fe2_y"], out["fe2_R"] = t2n(x2), t2n(y2), t2n(R)
    out["fe2_grad_x"] = t2n(x2.grad)
    for k, p in fe2.named_parameters():
        out["fe2_grad." + k] = t2n(p.grad)
    # 3. RelPosMHAXL attn_mask: bool (T, T) causal and float (B*H, T, T) additive
    torch.manual_seed(2)
    mha = RelPosMHAXL(embed_dim=64, num_heads=4)
    mha.eval()
    for k, v in mha.state_dict().items():
        out["mha." + k] = t2n(v)
    T = 29
    q = torch.randn(2, T, 64, generator=g)
    pe = RelPosEncXL(64)(q)
    kpm = torch.arange(T)[None, :] >= torch.tensor([T, 23])[:, None]
    causal = torch.triu(torch.ones(T, T, dtype=torch.bool), diagonal=1)
    fmask = 0.5 * torch.randn(2 * 4, T, T, generator=g)
    out["mha_q"], out["mha_pe"], out["mha_kpm"] = t2n(q), t2n(pe), kpm.numpy()
    out["mha_fmask"] = t2n(fmask)
    with torch.no_grad():
        for tag, am in (("causal", causal), ("float", fmask)):
            o, a = mha(q, q, q, pe, key_padding_mask=kpm, attn_mask=am)
            out[f"mha_{tag}_out"], out[f"mha_{tag}_attn"] = t2n(o), t2n(a)
    # vbias=True (attention.py:576-579), the value bias set away from its zero init
    torch.manual_seed(3)
    mhv = RelPosMHAXL(embed_dim=64, num_heads=4, vbias=True)
    with torch.no_grad():
        mhv.value_bias_weight.copy_(0.3 * torch.randn(64, generator=g))
    mhv.eval()
    for k, v in mhv.state_dict().items():
        out["mhv." + k] = t2n(v)
    with torch.no_grad():
        o, a = mhv(q, q, q, pe, key_padding_mask=kpm)
    out["mhv_out"], out["mhv_attn"] = t2n(o), t2n(a)
    # 4. SpecAugment with bilinear time warp (seeds 0..2)
    feats = torch.randn(3, 120, 40, generator=g)
    out["warp_feats"] = t2n(feats)
    aug = SpecAugment(time_warp=True, time_warp_mode="bilinear", freq_mask=False, time_mask=False)
    for sd in range(3):
        torch.manual_seed(sd)
        out[f"warp_bilinear_s{sd}"] = t2n(aug(feats.clone()))
    np.savez_compressed(os.path.join(OUT, "dropin.npz"), **out)


def gen_recipe():
    """recipe.npz: the recipe-level drop-ins beyond the encoder fixtures."""
    out = {}
    g = torch.Generator().manual_seed(41)
    # 1. Fbank(n_mels=80) on every tests/samples/ASR WAV (dataio.py:216-250 scaling)
    names = sorted(f[:-4] for f in os.listdir(os.path.join(REF, "tests/samples/ASR")) if f.endswith(".wav"))
    fb = LF.Fbank(n_mels=80)
    fb.eval()
    out["wav_names"] = np.array(names)
    with torch.no_grad():
        for n in names:
            pcm = read_wav(n)
            out[f"pcm.{n}"] = pcm.astype(np.int16)
            out[f"fbank80.{n}"] = t2n(fb(torch.from_numpy(pcm.astype(np.float32) / 32768.0)[None]))
    # 2. Filterbank(param_rand_factor=0.1) in training mode: the per-call
    #    torch.rand(2) jitter of central frequencies and bands
    #    (processing/features.py:525-532), seeds 0..2, and eval mode (no jitter)
    spec = torch.rand(2, 37, 201, generator=g) * 3
    out["fbj_spec"] = t2n(spec)
    fbj = F.Filterbank(n_mels=40, param_rand_factor=0.1)
    fbj.train()
    with torch.no_grad():
        for sd in range(3):
            torch.manual_seed(sd)
            out[f"fbj_train_s{sd}"] = t2n(fbj(spec))
        fbj.eval()
        out["fbj_eval"] = t2n(fbj(spec))
    # 3. standalone Conv2d (nnet/CNN.py:504-700): "same" reflect padding
    #    (stride 1 and 2, non-square kernels), "valid", a 3-D input
    from speechbrain.nnet.CNN import Conv2d
    convs = {
        "c33": dict(out_channels=5, kernel_size=(3, 3), input_shape=(2, 21, 13, 3)),
        "c53s21": dict(out_channels=6, kernel_size=(5, 3), stride=(2, 1), input_shape=(2, 19, 16, 4)),
        "cvalid": dict(out_channels=4, kernel_size=(3, 5), padding="valid", input_shape=(2, 17, 12, 2)),
        "c3d": dict(out_channels=3, kernel_size=(3, 3), input_shape=(2, 15, 11)),
    }
    for tag, kw in convs.items():
        torch.manual_seed(5)
        conv = Conv2d(**kw)
        for k, v in conv.state_dict().items():
            out[f"{tag}.{k}"] = t2n(v)
        x = torch.randn(*kw["input_shape"], generator=g).requires_grad_(True)
        y = conv(x)
        R = torch.randn(y.shape, generator=g)
        (y * R).sum().backward()
        out[f"{tag}_x"], out[f"{tag}_y"], out[f"{tag}_R"] = t2n(x), t2n(y), t2n(R)
        out[f"{tag}_grad_x"] = t2n(x.grad)
        for k, p in conv.named_parameters():
            out[f"{tag}_grad.{k}"] = t2n(p.grad)
    # 4. TransformerASR with the decoder (conformer_small.yaml's shape of
    #    model at a small size): seeded-init checksums, state_dict, forward
    #    (encoder + decoder), encode and decode
    torch.manual_seed(9)
    asr = TransformerASR(tgt_vocab=31, input_size=40, d_model=64, nhead=4, num_encoder_layers=2,
                         num_decoder_layers=2, d_ffn=128, dropout=0.1, activation=torch.nn.GELU,
                         encoder_module="conformer", attention_type="RelPosMHAXL", normalize_before=True,
                         causal=False)
    asr.eval()
    params = dict(asr.named_parameters())
    for k, v in asr.state_dict().items():
        if k in params:  # buffers (the sine tables) are checked by their checksums only
            out[f"asr.{k}"] = t2n(v)
        v64 = v.double()
        out[f"asr_sum.{k}"] = np.asarray(float(v64.sum()), np.float64)
    src = torch.randn(3, 23, 40, generator=g)
    tgt = torch.randint(1, 31, (3, 9), generator=g)
    tgt[1, 6:] = 0  # padding (pad_idx 0)
    tgt[2, 4:] = 0
    wav_len = torch.tensor([1.0, 0.7, 0.45])
    with torch.no_grad():
        enc_out, dec_out = asr(src, tgt, wav_len)
        enc = asr.encode(src, wav_len)
        enc_len = torch.round(wav_len * 23).long()
        pred, att = asr.decode(tgt, enc, enc_len)
    out["asr_src"], out["asr_tgt"], out["asr_wav_len"] = t2n(src), tgt.numpy(), t2n(wav_len)
    out["asr_fwd_enc"], out["asr_fwd_dec"], out["asr_enc"] = t2n(enc_out), t2n(dec_out), t2n(enc)
    out["asr_enc_len"] = enc_len.numpy()
    out["asr_dec_pred"], out["asr_dec_att"] = t2n(pred), t2n(att)
    # 5. the reference Brain step (core.py:882-994) on CPU: ConvolutionFrontEnd +
    #    2-layer TransformerASR encoder (weights of conformer.npz), SGD,
    #    grad_accumulation_factor 2, max_grad_norm 5.0, a NaN loss on the
    #    4th batch (an optimizer step: skipped, nonfinite_count 1)
    from speechbrain.core import Brain, Stage  # noqa: F401
    g0 = np.load(os.path.join(OUT, "conformer.npz"))
    cnn = ConvolutionFrontEnd(input_shape=(8, 10, 80), num_blocks=2, num_layers_per_block=1,
                              out_channels=(64, 32), kernel_sizes=(3, 3), strides=(2, 2),
                              residuals=(False, False), dropout=0.0)
    tr = TransformerASR(tgt_vocab=10, input_size=640, d_model=64, nhead=4, num_encoder_layers=2,
                        num_decoder_layers=0, d_ffn=128, dropout=0.0, encoder_module="conformer",
                        attention_type="RelPosMHAXL", normalize_before=True, causal=False)
    for pre, m in (("cnn.", cnn), ("tr.", tr)):
        m.load_state_dict({k[len(pre):]: torch.from_numpy(g0[k]) for k in g0.files if k.startswith(pre)})

    class StepBrain(Brain):
        def compute_forward(self, batch, stage):
            feats, wl, _, _ = batch
            return self.modules.tr.encode(self.modules.cnn(feats), wl)

        def compute_objectives(self, y, batch, stage):
            _, _, tgt, bad = batch
            loss = 0.5 * ((y - tgt) ** 2).sum()
            return loss * float("nan") if bad else loss

    brain = StepBrain(modules={"cnn": cnn, "tr": tr}, opt_class=lambda ps: torch.optim.SGD(ps, lr=0.01),
                      run_opts={"device": "cpu", "grad_accumulation_factor": 2, "max_grad_norm": 5.0})
    brain.modules.train()
    brain.init_optimizers()
    brain.nonfinite_count = 0
    wl = torch.tensor([1.0, 0.8])
    for i in range(6):
        feats = torch.randn(2, 40, 80, generator=g)
        tgt = torch.randn(2, 10, 64, generator=g)
        bad = i == 3
        out[f"brain_feats{i}"], out[f"brain_tgt{i}"] = t2n(feats), t2n(tgt)
        brain.step += 1
        loss = brain.fit_batch((feats, wl, tgt, bad))
        out[f"brain_loss{i}"] = np.asarray(float(loss), np.float64)
        # parameters after the two optimizer steps that run (batches 1 and 5;
        # batch 3's step is the skipped one), a float64 checksum after each batch
        for name, m in (("cnn.", cnn), ("tr.", tr)):
            for k, p in m.named_parameters():
                if i in (1, 5):
                    out[f"brain_p{i}.{name}{k}"] = t2n(p)
        out[f"brain_psum{i}"] = np.asarray(sum(float((p.double() ** 2).sum()) for p in brain.modules.parameters()),
                                           np.float64)
        out[f"brain_state{i}"] = np.array([brain.step, brain.optimizer_step, brain.nonfinite_count], np.int64)
    out["brain_wav_len"] = t2n(wl)
    np.savez_compressed(os.path.join(OUT, "recipe.npz"), **out)


def gen_xattn():
    """xattn.npz: RelPosMHAXL with query != key/value and q_len != k_len
    (nnet/attention.py:554-564 separate projections, rel_shift :468-483 on a
    (q_len, 2*k_len-1) band, mask_pos_future's tril).  Cases "u*": the 16
    combinations of tests/unittests/test_attention.py:4-27 (emb 4, 2 heads,
    k_len 12|10 x q_len 10|12 x vbias x vdim 4|None), seeded; "c*": wider
    cases (emb 64, 4 heads) with mask_pos_future, key padding, a bool and a
    float attn_mask, key != value.  Every case records the state_dict, the
    inputs, out and attention weights, and the autograd gradients of
    sum(R * out) w.r.t. the parameters, query, key and value."""
    out = {}
    g = torch.Generator().manual_seed(61)
    cases = []
    n = 0
    for kl in (12, 10):
        for ql in (10, 12):
            for b in (True, False):
                for h in (4, None):
                    cases.append(dict(tag=f"u{n}", E=4, H=2, vbias=b, vdim=h, ql=ql, kl=kl, same_kv=True))
                    n += 1
    cases += [
        dict(tag="c0", E=64, H=4, vbias=False, vdim=None, ql=37, kl=23, same_kv=True, mpf=True),
        dict(tag="c1", E=64, H=4, vbias=True, vdim=None, ql=19, kl=41, same_kv=False, mpf=True, kpm=True),
        dict(tag="c2", E=64, H=4, vbias=False, vdim=None, ql=29, kl=17, same_kv=False, kpm=True, bmask=True),
        dict(tag="c3", E=64, H=4, vbias=True, vdim=None, ql=16, kl=33, same_kv=True, fmask=True),
        dict(tag="c4", E=32, H=2, vbias=False, vdim=None, ql=21, kl=21, same_kv=False, mpf=True),
        dict(tag="c5", E=64, H=4, vbias=False, vdim=None, ql=50, kl=7, same_kv=True, mpf=True),
    ]
    out["cases"] = np.array([c["tag"] for c in cases])
    for i, c in enumerate(cases):
        t, E, H, ql, kl = c["tag"], c["E"], c["H"], c["ql"], c["kl"]
        torch.manual_seed(100 + i)
        m = RelPosMHAXL(E, num_heads=H, vbias=c["vbias"], vdim=c["vdim"], mask_pos_future=c.get("mpf", False))
        if c["vbias"]:
            with torch.no_grad():
                m.value_bias_weight.copy_(0.3 * torch.randn(E, generator=g))
        B = 2
        q = torch.rand((B, ql, E), generator=g).requires_grad_(True)
        k = torch.rand((B, kl, E), generator=g).requires_grad_(True)
        v = k if c["same_kv"] else torch.rand((B, kl, E), generator=g).requires_grad_(True)
        pe = torch.rand((1, 2 * kl - 1, E), generator=g)
        kpm = None
        if c.get("kpm"):
            kpm = torch.arange(kl)[None, :] >= torch.tensor([kl, kl - 5])[:, None]
        am = None
        if c.get("bmask"):
            am = torch.rand((ql, kl), generator=g) < 0.25
            am[:, 0] = False  # no fully masked row
        if c.get("fmask"):
            am = 0.5 * torch.randn(B * H, ql, kl, generator=g)
        o, a = m(q, k, v, pos_embs=pe, key_padding_mask=kpm, attn_mask=am)
        R = torch.randn(o.shape, generator=g)
        (o * R).sum().backward()
        meta = np.array([E, H, int(c["vbias"]), ql, kl, int(c["same_kv"]), int(c.get("mpf", False)),
                         int(kpm is not None), 0 if am is None else (1 if am.dtype == torch.bool else 2)], np.int64)
        out[f"{t}.meta"] = meta
        for kk, vv in m.state_dict().items():
            out[f"{t}.sd.{kk}"] = t2n(vv)
        out[f"{t}.q"], out[f"{t}.k"], out[f"{t}.pe"], out[f"{t}.R"] = t2n(q), t2n(k), t2n(pe), t2n(R)
        if not c["same_kv"]:
            out[f"{t}.v"] = t2n(v)
            out[f"{t}.grad_v"] = t2n(v.grad)
        if kpm is not None:
            out[f"{t}.kpm"] = kpm.numpy()
        if am is not None:
            out[f"{t}.am"] = am.numpy() if am.dtype == torch.bool else t2n(am)
        out[f"{t}.out"], out[f"{t}.attn"] = t2n(o), t2n(a)
        out[f"{t}.grad_q"], out[f"{t}.grad_k"] = t2n(q.grad), t2n(k.grad)
        for kk, p in m.named_parameters():
            out[f"{t}.grad.{kk}"] = t2n(p.grad)
    np.savez_compressed(os.path.join(OUT, "xattn.npz"), **out)


def _doctest_ns():
    """The reference's classes under the names doctest_cases.py uses."""
    from types import SimpleNamespace
    from speechbrain.processing import features as PF
    from speechbrain.lobes import features as LFe
    from speechbrain.lobes.models.transformer import Conformer as RC, Transformer as RT, TransformerASR as RA
    from speechbrain.lobes.models import convolution as RCV, wav2vec as RW
    from speechbrain.nnet import attention as RAT, CNN as RCNN, linear as RL, normalization as RN, activations as RACT
    from speechbrain.nnet.transducer import transducer_joint as RJ
    return SimpleNamespace(
        STFT=PF.STFT, spectral_magnitude=PF.spectral_magnitude, Filterbank=PF.Filterbank, DCT=PF.DCT,
        Deltas=PF.Deltas, ContextWindow=PF.ContextWindow, InputNormalization=PF.InputNormalization,
        Fbank=LFe.Fbank, MFCC=LFe.MFCC, SpecAugment=SpecAugment, ConvolutionFrontEnd=RCV.ConvolutionFrontEnd,
        ConvBlock=RCV.ConvBlock, Conv2d=RCNN.Conv2d, Linear=RL.Linear, LayerNorm=RN.LayerNorm, Swish=RACT.Swish,
        RelPosMHAXL=RAT.RelPosMHAXL, MultiheadAttention=RAT.MultiheadAttention,
        PositionalwiseFeedForward=RAT.PositionalwiseFeedForward, ConvolutionModule=RC.ConvolutionModule,
        ConformerEncoderLayer=RC.ConformerEncoderLayer, ConformerEncoder=RC.ConformerEncoder,
        PositionalEncoding=RT.PositionalEncoding, TransformerEncoderLayer=RT.TransformerEncoderLayer,
        TransformerEncoder=RT.TransformerEncoder, TransformerDecoderLayer=RT.TransformerDecoderLayer,
        TransformerDecoder=RT.TransformerDecoder, NormalizedEmbedding=RT.NormalizedEmbedding,
        TransformerASR=RA.TransformerASR, EncoderWrapper=RA.EncoderWrapper, GELU=torch.nn.GELU,
        Transducer_joint=RJ.Transducer_joint, W2VLatentExtractor=RW.W2VLatentExtractor,
        W2VEncoderWrapper=RW.EncoderWrapper)


def gen_doctests():
    """doctests.npz: the reference's doctest examples (tests/golden/doctest_cases.py)
    run on the reference modules with detinit weights and inputs: the output
    shape (asserted equal to the doctest's printed shape) and the kept slice
    of the output."""
    sys.path.insert(0, OUT)
    from detinit import det_state
    from doctest_cases import cases
    ns = _doctest_ns()
    out = {}
    for c in cases():
        m = c.build(ns) if c.build is not None else None
        if m is not None:
            if c.det:
                m.load_state_dict(det_state(m, c.seed), strict=True)
            m.train(not c.eval_mode)
        xs = c.make_inputs(torch)
        torch.manual_seed(c.seed)
        with torch.no_grad():
            y = c.call(ns, m, *xs)
        assert tuple(y.shape) == c.shape, (c.name, tuple(y.shape), c.shape)
        out[c.name + ".shape"] = np.array(y.shape, np.int64)
        out[c.name + ".out"] = t2n(c.keep(y))
        print(c.name, tuple(y.shape))
    np.savez_compressed(os.path.join(OUT, "doctests.npz"), **out)


def _variant_model(ctor):
    from speechbrain.nnet.activations import Swish
    sys.path.insert(0, OUT)
    kw = dict(ctor)
    act = kw.pop("act", None)
    if act is not None:
        kw["activation"] = {"gelu": torch.nn.GELU, "relu": torch.nn.ReLU, "swish": Swish}[act]
    return TransformerASR(**kw)


def _recipe_cnn():
    """transformer.yaml:122-130."""
    return ConvolutionFrontEnd(input_shape=(8, 10, 80), num_blocks=3, num_layers_per_block=1,
                               out_channels=(64, 64, 64), kernel_sizes=(5, 5, 1), strides=(2, 2, 1),
                               residuals=(False, False, True))


def gen_variants():
    """variants.npz: TransformerASR / encoder constructor variants beyond the
    Conformer + RelPosMHAXL recipe (TransformerASR.py:87-316,
    Transformer.py:83-192,246-486, Conformer.py:118-383), weights from
    detinit.  Per case: forward (with and without wav_len), encode, decode,
    and (grads=True) the gradients of sum(R * encode(src, wav_len)) w.r.t.
    the encoder-side parameters and the input.  Plus a regularMHA
    ConformerEncoder called directly with a bool src_mask and key padding."""
    sys.path.insert(0, OUT)
    from detinit import det_state, det_input
    from variant_cases import VARIANTS
    out = {}
    for i, (tag, c) in enumerate(VARIANTS.items()):
        model = _variant_model(c["ctor"])
        model.load_state_dict(det_state(model, 50 + i), strict=True)
        model.eval()
        B, T, Fd, U = c["B"], c["T"], c["F"], c["U"]
        cnn = None
        if c.get("cnn"):
            cnn = _recipe_cnn()
            cnn.load_state_dict(det_state(cnn, 150 + i), strict=True)
            cnn.eval()
        x = torch.from_numpy(det_input((B, T, Fd), 200 + i))
        rng = np.random.default_rng(300 + i)
        tgt = torch.from_numpy(rng.integers(1, c["ctor"]["tgt_vocab"], size=(B, U))).long()
        tgt[1, U - 2:] = 0
        if B > 2:
            tgt[2, U - 4:] = 0
        wav_len = torch.tensor([1.0, 0.8, 0.55][:B])
        with torch.no_grad():
            src = cnn(x) if cnn is not None else x
            Te = src.shape[1]
            e1, d1 = model(src, tgt, wav_len)
            e0, d0 = model(src, tgt)
            out[f"{tag}.fwd_enc"], out[f"{tag}.fwd_dec"] = t2n(e1), t2n(d1)
            out[f"{tag}.fwd0_enc"], out[f"{tag}.fwd0_dec"] = t2n(e0), t2n(d0)
            enc = model.encode(src, wav_len)
            out[f"{tag}.enc"] = t2n(enc)
            out[f"{tag}.enc0"] = t2n(model.encode(src))
            enc_len = torch.round(wav_len * Te).long()
            pred, att = model.decode(tgt, enc, enc_len)
            out[f"{tag}.dec_pred"], out[f"{tag}.dec_att"] = t2n(pred), t2n(att)
        out[f"{tag}.x"], out[f"{tag}.tgt"], out[f"{tag}.wav_len"] = t2n(x), tgt.numpy(), t2n(wav_len)
        out[f"{tag}.enc_len"] = enc_len.numpy()
        if c["grads"]:
            xg = x.clone().requires_grad_(True)
            y = model.encode(cnn(xg) if cnn is not None else xg, wav_len)
            R = torch.from_numpy(det_input(tuple(y.shape), 400 + i))
            (y * R).sum().backward()
            out[f"{tag}.grad_x"] = t2n(xg.grad)
            for k, p in model.named_parameters():
                if p.grad is not None:
                    out[f"{tag}.grad.{k}"] = t2n(p.grad)
        print(tag, tuple(enc.shape))
    # ConformerEncoder(regularMHA) directly: src_mask (bool, True = masked), key padding, attention maps
    enc = ConformerEncoder(2, 64, 128, 4, kernel_size=7, attention_type="regularMHA")
    enc.load_state_dict(det_state(enc, 90), strict=True)
    enc.eval()
    x = torch.from_numpy(det_input((2, 17, 64), 91)).requires_grad_(True)
    kpm = torch.arange(17)[None, :] >= torch.tensor([17, 12])[:, None]
    am = torch.triu(torch.ones(17, 17), diagonal=3).bool()
    y, attns = enc(x, src_mask=am, src_key_padding_mask=kpm)
    R = torch.from_numpy(det_input(tuple(y.shape), 92))
    (y * R).sum().backward()
    out["cenc.x"], out["cenc.kpm"], out["cenc.am"] = t2n(x), kpm.numpy(), am.numpy()
    out["cenc.y"] = t2n(y)
    for j, a in enumerate(attns):
        out[f"cenc.attn{j}"] = t2n(a)
    out["cenc.grad_x"] = t2n(x.grad)
    for k, p in enc.named_parameters():
        out[f"cenc.grad.{k}"] = t2n(p.grad)
    np.savez_compressed(os.path.join(OUT, "variants.npz"), **out)


if __name__ == "__main__":
    if sys.argv[1:] == ["variants"]:
        gen_variants()
        sys.exit(0)
    if sys.argv[1:] == ["doctests"]:
        gen_doctests()
        sys.exit(0)
    if sys.argv[1:] == ["xattn"]:
        gen_xattn()
        sys.exit(0)
    if sys.argv[1:] == ["recipe"]:
        gen_recipe()
        sys.exit(0)
    if sys.argv[1:] == ["dropin"]:
        gen_dropin()
        sys.exit(0)
    if sys.argv[1:] == ["decoder"]:
        gen_decoder()
        sys.exit(0)
    if sys.argv[1:] == ["wav2vec"]:
        gen_wav2vec()
        sys.exit(0)
    if sys.argv[1:] == ["train"]:
        gen_train()
        sys.exit(0)
    if sys.argv[1:] == ["inputnorm"]:
        gen_inputnorm()
        sys.exit(0)
    gen_fbank_wavs()
    gen_features()
    gen_specaug()
    gen_conformer()
    gen_train()
    gen_inputnorm()
    gen_wav2vec()
    gen_decoder()
    gen_dropin()
    gen_recipe()
    gen_xattn()
    gen_variants()
    gen_doctests()
    for f in sorted(os.listdir(OUT)):
        if f.endswith(".npz"):
            print(f, os.path.getsize(os.path.join(OUT, f)))
