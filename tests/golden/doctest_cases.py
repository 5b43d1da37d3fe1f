"""The reference's doctest examples for the drop-in modules, as data
(test infrastructure; SURVEY.md §4 "Doctests pin shapes").

Each case restates one `>>>` example of the reference (cited) — constructor,
input shapes, call and the printed output shape — over a namespace `ns` of
module classes, so the same case runs on the reference's modules
(tests/golden/gen_golden.py → doctests.npz) and on the drop-ins
(tests/test_gpu_doctests.py).  Inputs come from detinit.det_input (numpy
PCG64, machine independent) instead of the doctests' unseeded torch.rand /
torch.randn; models with learned parameters load detinit.det_state.  The
fixture keeps the first batch element of each output (`keep`), enough to pin
values while the shape is checked at the doctest's full size.
"""
import numpy as np

from detinit import det_input


class Case:
    def __init__(self, name, cite, build, inputs, call, shape, det=False, keep=None, eval_mode=True, seed=0):
        self.name = name
        self.cite = cite
        self.build = build          # ns -> module (or None for a function)
        self.inputs = inputs        # [(kind, shape)] kind: rand | randn | randint:N | ones | lens
        self.call = call            # (ns, module, *tensors) -> output tensor
        self.shape = tuple(shape)   # the shape the doctest prints
        self.det = det              # load detinit.det_state
        self.keep = keep if keep is not None else (lambda y: y[0])
        self.eval_mode = eval_mode
        self.seed = seed  # also torch.manual_seed(seed) right before the call (SpecAugment's draws)

    def make_inputs(self, torch, device="cpu"):
        out = []
        for i, (kind, shp) in enumerate(self.inputs):
            s = 1000 * self.seed + i
            if kind.startswith("randint:"):
                hi = int(kind.split(":")[1])
                x = torch.from_numpy(np.random.default_rng(s).integers(0, hi, size=shp)).long()
            elif kind == "ones":
                x = torch.ones(shp)
            else:
                x = torch.from_numpy(det_input(shp, s, kind))
            out.append(x.to(device))
        return out


def _first(y):
    return y[0] if isinstance(y, (tuple, list)) else y


def cases():
    C = []
    a = C.append
    # processing/features.py
    a(Case("stft", "speechbrain/processing/features.py:91-98",
           lambda ns: ns.STFT(sample_rate=16000, win_length=25, hop_length=10, n_fft=400),
           [("randn", (10, 16000))], lambda ns, m, x: m(x), (10, 101, 201, 2), seed=1))
    a(Case("spectral_magnitude", "speechbrain/processing/features.py:343-345", None,
           [("rand", (4, 7, 2))], lambda ns, m, x: ns.spectral_magnitude(x, power=0.5), (4, 7), seed=2,
           keep=lambda y: y))
    a(Case("filterbank", "speechbrain/processing/features.py:407-412", lambda ns: ns.Filterbank(),
           [("randn", (10, 101, 201))], lambda ns, m, x: m(x), (10, 101, 40), seed=3))
    a(Case("dct", "speechbrain/processing/features.py:732-737", lambda ns: ns.DCT(input_size=40),
           [("randn", (10, 101, 40))], lambda ns, m, x: m(x), (10, 101, 20), seed=4))
    a(Case("deltas", "speechbrain/processing/features.py:799-803", lambda ns: ns.Deltas(input_size=20),
           [("randn", (10, 101, 20))], lambda ns, m, x: m(x), (10, 101, 20), seed=5))
    a(Case("context_window", "speechbrain/processing/features.py:871-876",
           lambda ns: ns.ContextWindow(left_frames=5, right_frames=5),
           [("randn", (10, 101, 20))], lambda ns, m, x: m(x), (10, 101, 220), seed=6))
    a(Case("input_normalization", "speechbrain/processing/features.py:962-966", lambda ns: ns.InputNormalization(),
           [("randn", (10, 101, 20)), ("ones", (10,))], lambda ns, m, x, l: m(x, l), (10, 101, 20), seed=7,
           eval_mode=False))
    # lobes/features.py
    a(Case("spec_augment", "speechbrain/lobes/augment.py:63-67", lambda ns: ns.SpecAugment(),
           [("rand", (8, 120, 80))], lambda ns, m, x: m(x), (8, 120, 80), seed=33, eval_mode=False))
    a(Case("fbank", "speechbrain/lobes/features.py:74-79", lambda ns: ns.Fbank(),
           [("randn", (10, 16000))], lambda ns, m, x: m(x), (10, 101, 40), seed=8))
    a(Case("mfcc", "speechbrain/lobes/features.py:204-209", lambda ns: ns.MFCC(),
           [("randn", (10, 16000))], lambda ns, m, x: m(x), (10, 101, 660), seed=9))
    # lobes/models/convolution.py, nnet/CNN.py, nnet/linear.py, nnet/normalization.py, nnet/activations.py
    a(Case("conv_frontend", "speechbrain/lobes/models/convolution.py:41-45",
           lambda ns: ns.ConvolutionFrontEnd(input_shape=(8, 30, 10)),
           [("rand", (8, 30, 10))], lambda ns, m, x: m(x), (8, 8, 3, 512), det=True, seed=10))
    a(Case("conv_block", "speechbrain/lobes/models/convolution.py:109-114",
           lambda ns: ns.ConvBlock(2, 16, input_shape=(8, 30, 10)),
           [("rand", (8, 30, 10))], lambda ns, m, x: m(x), (8, 30, 10, 16), det=True, seed=11))
    a(Case("conv2d", "speechbrain/nnet/CNN.py:547-553",
           lambda ns: ns.Conv2d(input_shape=(10, 40, 16, 8), out_channels=5, kernel_size=(7, 3)),
           [("rand", (10, 40, 16, 8))], lambda ns, m, x: m(x), (10, 40, 16, 5), det=True, seed=12))
    a(Case("linear", "speechbrain/nnet/linear.py:34-38",
           lambda ns: ns.Linear(input_shape=(10, 50, 40), n_neurons=100),
           [("rand", (10, 50, 40))], lambda ns, m, x: m(x), (10, 50, 100), det=True, seed=13))
    a(Case("layer_norm", "speechbrain/nnet/normalization.py:188-192",
           lambda ns: ns.LayerNorm(input_shape=(100, 101, 128)),
           [("randn", (100, 101, 128))], lambda ns, m, x: m(x), (100, 101, 128), det=True, seed=14))
    a(Case("swish", "speechbrain/nnet/activations.py:124-127", lambda ns: ns.Swish(),
           [("randn", (8, 40, 120))], lambda ns, m, x: m(x), (8, 40, 120), seed=15))
    # nnet/attention.py
    a(Case("relpos_mhaxl", "speechbrain/nnet/attention.py:383-388",
           lambda ns: ns.RelPosMHAXL(num_heads=8, embed_dim=512),
           [("rand", (6, 60, 512)), ("rand", (1, 119, 512))], lambda ns, m, x, p: _first(m(x, x, x, p)),
           (6, 60, 512), det=True, seed=16))
    a(Case("mha", "speechbrain/nnet/attention.py:666-670", lambda ns: ns.MultiheadAttention(nhead=8, d_model=512),
           [("rand", (8, 60, 512))], lambda ns, m, x: _first(m(x, x, x)), (8, 60, 512), det=True, seed=17))
    a(Case("pos_ffn", "speechbrain/nnet/attention.py:800-804",
           lambda ns: ns.PositionalwiseFeedForward(256, input_size=512),
           [("rand", (8, 60, 512))], lambda ns, m, x: m(x), (8, 60, 512), det=True, seed=18))
    # lobes/models/transformer/Conformer.py
    a(Case("conv_module", "speechbrain/lobes/models/transformer/Conformer.py:46-51",
           lambda ns: ns.ConvolutionModule(512, 3),
           [("rand", (8, 60, 512))], lambda ns, m, x: m(x), (8, 60, 512), det=True, seed=19))
    a(Case("conformer_layer", "speechbrain/lobes/models/transformer/Conformer.py:148-154",
           lambda ns: ns.ConformerEncoderLayer(d_ffn=512, nhead=8, d_model=512, kernel_size=3),
           [("rand", (8, 60, 512)), ("rand", (1, 119, 512))], lambda ns, m, x, p: m(x, pos_embs=p)[0],
           (8, 60, 512), det=True, seed=20))
    a(Case("conformer_encoder", "speechbrain/lobes/models/transformer/Conformer.py:296-302",
           lambda ns: ns.ConformerEncoder(1, 512, 512, 8),
           [("rand", (8, 60, 512)), ("rand", (1, 119, 512))], lambda ns, m, x, p: m(x, pos_embs=p)[0],
           (8, 60, 512), det=True, seed=21))
    # lobes/models/transformer/Transformer.py
    a(Case("positional_encoding", "speechbrain/lobes/models/transformer/Transformer.py:214-218",
           lambda ns: ns.PositionalEncoding(input_size=512),
           [("rand", (8, 120, 512))], lambda ns, m, x: m(x), (1, 120, 512), seed=22))
    a(Case("transformer_layer", "speechbrain/lobes/models/transformer/Transformer.py:275-280",
           lambda ns: ns.TransformerEncoderLayer(512, 8, d_model=512),
           [("rand", (8, 60, 512))], lambda ns, m, x: m(x)[0], (8, 60, 512), det=True, seed=23))
    a(Case("transformer_encoder", "speechbrain/lobes/models/transformer/Transformer.py:401-406",
           lambda ns: ns.TransformerEncoder(1, 8, 512, d_model=512),
           [("rand", (8, 60, 512))], lambda ns, m, x: m(x)[0], (8, 60, 512), det=True, seed=24))
    a(Case("transformer_decoder_layer", "speechbrain/lobes/models/transformer/Transformer.py:509-514",
           lambda ns: ns.TransformerDecoderLayer(1024, 8, d_model=512),
           [("rand", (8, 60, 512)), ("rand", (8, 60, 512))], lambda ns, m, s, t: m(s, t)[0], (8, 60, 512),
           det=True, seed=25))
    a(Case("transformer_decoder", "speechbrain/lobes/models/transformer/Transformer.py:677-682",
           lambda ns: ns.TransformerDecoder(1, 8, 1024, d_model=512),
           [("rand", (8, 60, 512)), ("rand", (8, 60, 512))], lambda ns, m, s, t: m(s, t)[0], (8, 60, 512),
           det=True, seed=26))
    a(Case("normalized_embedding", "speechbrain/lobes/models/transformer/Transformer.py:782-787",
           lambda ns: ns.NormalizedEmbedding(512, 1000),
           [("randint:999", (8, 50))], lambda ns, m, x: m(x), (8, 50, 512), det=True, seed=27))
    # lobes/models/transformer/TransformerASR.py
    a(Case("transformer_asr", "speechbrain/lobes/models/transformer/TransformerASR.py:75-85",
           lambda ns: ns.TransformerASR(720, 512, 512, 8, 1, 1, 1024, activation=ns.GELU),
           [("rand", (8, 120, 512)), ("randint:720", (8, 120))], lambda ns, m, s, t: m.forward(s, t)[1],
           (8, 120, 512), det=True, seed=28))
    a(Case("encoder_wrapper", "speechbrain/lobes/models/transformer/TransformerASR.py:338-347",
           lambda ns: ns.EncoderWrapper(ns.TransformerASR(720, 512, 512, 8, 1, 1, 1024, activation=ns.GELU)),
           [("rand", (8, 120, 512))], lambda ns, m, s: m(s), (8, 120, 512), det=True, seed=29))
    # nnet/transducer/transducer_joint.py
    a(Case("transducer_joint", "speechbrain/nnet/transducer/transducer_joint.py:29-37",
           lambda ns: ns.Transducer_joint(ns.Linear(input_size=80, n_neurons=80), joint="concat"),
           [("rand", (8, 200, 1, 40)), ("rand", (8, 1, 12, 40))], lambda ns, m, t, p: m(t, p),
           (8, 200, 12, 80), det=True, seed=30, keep=lambda y: y[0, :16]))
    # lobes/models/wav2vec.py
    a(Case("w2v_latent_extractor", "speechbrain/lobes/models/wav2vec.py:45-49", lambda ns: ns.W2VLatentExtractor(),
           [("rand", (10, 5000))], lambda ns, m, x: m(x), (10, 14, 512), det=True, seed=31))
    a(Case("w2v_encoder_wrapper", "speechbrain/lobes/models/wav2vec.py:173-179",
           lambda ns: ns.W2VEncoderWrapper(1024, 768, ns.TransformerEncoder(d_model=768, num_layers=4, nhead=4,
                                                                            d_ffn=1024)),
           [("rand", (10, 12, 1024))], lambda ns, m, x: m(x)["embeddings"], (10, 12, 768), det=True, seed=32))
    return C
