"""Constructor coverage (CPU): modules the reference builds with its
defaults construct here with the same state_dict keys and — under the same
torch.manual_seed — bit-identical initial weights (tests/golden/dropin.npz,
generated from the reference by tests/golden/gen_golden.py):
ConvolutionFrontEnd(input_shape) with every default (3 residual blocks x 5
layers; convolution.py:12-175 incl. the Sequential shape-inference dropout
draws, nnet/containers.py get_output_shape), a residual multi-layer front-end
with kernel 5, RelPosMHAXL (attention.py:362-420), TransformerASR with its
decoder and the standalone Conv2d (tests/golden/recipe.npz)."""
import numpy as np
import torch


def test_default_frontend_seeded_init(golden):
    from speechbrain_amd.lobes.models.convolution import ConvolutionFrontEnd
    g = golden("dropin")
    torch.manual_seed(0)
    fe = ConvolutionFrontEnd(input_shape=(8, 30, 10))
    sd = fe.state_dict()
    keys = sorted(k[len("fe_def_sum."):] for k in g.files if k.startswith("fe_def_sum."))
    assert sorted(sd) == keys
    for k in keys:
        v = sd[k].double()
        assert float(v.sum()) == float(g["fe_def_sum." + k]), k
        assert float((v * v).sum()) == float(g["fe_def_sq." + k]), k


def test_residual_frontend_seeded_init(golden):
    from speechbrain_amd.lobes.models.convolution import ConvolutionFrontEnd
    g = golden("dropin")
    torch.manual_seed(1)
    fe = ConvolutionFrontEnd(input_shape=(3, 37, 20), num_blocks=2, num_layers_per_block=2, out_channels=(8, 16),
                             kernel_sizes=(3, 5), strides=(1, 2), residuals=(True, True), dropout=0.1)
    sd = fe.state_dict()
    keys = sorted(k[len("fe2."):] for k in g.files if k.startswith("fe2."))
    assert sorted(sd) == keys
    for k in keys:
        assert np.array_equal(sd[k].numpy(), g["fe2." + k]), k


def test_relposmha_seeded_init(golden):
    from speechbrain_amd.nnet.attention import RelPosMHAXL
    g = golden("dropin")
    torch.manual_seed(2)
    mha = RelPosMHAXL(embed_dim=64, num_heads=4)
    for k, v in mha.state_dict().items():
        assert np.array_equal(v.numpy(), g["mha." + k]), k


def test_transformer_asr_with_decoder_seeded_init_and_strict_load(golden):
    """TransformerASR(num_decoder_layers=2) — conformer_small.yaml's model
    shape (TransformerASR.py:87-141, Transformer.py:177-192,489-797) — has
    the reference's state_dict keys (decoder included) and, under the same
    seed, bit-identical initial weights; a reference checkpoint of it loads
    with strict=True (tests/golden/recipe.npz)."""
    from speechbrain_amd.lobes.models.transformer.TransformerASR import TransformerASR
    g = golden("recipe")
    torch.manual_seed(9)
    asr = TransformerASR(tgt_vocab=31, input_size=40, d_model=64, nhead=4, num_encoder_layers=2,
                         num_decoder_layers=2, d_ffn=128, dropout=0.1, activation=torch.nn.GELU,
                         encoder_module="conformer", attention_type="RelPosMHAXL", normalize_before=True,
                         causal=False)
    sd = asr.state_dict()
    keys = sorted(k[len("asr_sum."):] for k in g.files if k.startswith("asr_sum."))
    assert sorted(sd) == keys
    assert any(k.startswith("decoder.layers.1.mutihead_attn.att.") for k in keys)
    for k in keys:
        assert float(sd[k].double().sum()) == float(g["asr_sum." + k]), k
        if "asr." + k in g.files:
            assert np.array_equal(sd[k].numpy(), g["asr." + k]), k
    ckpt = {k: (torch.from_numpy(g["asr." + k]) if "asr." + k in g.files else v) for k, v in sd.items()}
    fresh = TransformerASR(tgt_vocab=31, input_size=40, d_model=64, nhead=4, num_encoder_layers=2,
                           num_decoder_layers=2, d_ffn=128, activation=torch.nn.GELU, encoder_module="conformer",
                           attention_type="RelPosMHAXL", normalize_before=True, causal=False)
    fresh.load_state_dict(ckpt, strict=True)


def test_conv2d_seeded_init(golden):
    """Standalone Conv2d (nnet/CNN.py:504-615): keys and seeded weights."""
    from speechbrain_amd.nnet.CNN import Conv2d
    g = golden("recipe")
    cfg = {"c33": dict(out_channels=5, kernel_size=(3, 3), input_shape=(2, 21, 13, 3)),
           "c53s21": dict(out_channels=6, kernel_size=(5, 3), stride=(2, 1), input_shape=(2, 19, 16, 4)),
           "cvalid": dict(out_channels=4, kernel_size=(3, 5), padding="valid", input_shape=(2, 17, 12, 2)),
           "c3d": dict(out_channels=3, kernel_size=(3, 3), input_shape=(2, 15, 11))}
    for tag, kw in cfg.items():
        torch.manual_seed(5)
        sd = Conv2d(**kw).state_dict()
        assert sorted(sd) == sorted(k[len(tag) + 1:] for k in g.files if k.startswith(tag + ".")), tag
        for k, v in sd.items():
            assert np.array_equal(v.numpy(), g[f"{tag}.{k}"]), (tag, k)
