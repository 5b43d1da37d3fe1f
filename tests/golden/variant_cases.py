"""TransformerASR constructor variants pinned by tests/golden/variants.npz
(test infrastructure, shared by gen_golden.py and tests/test_gpu_variants.py).
Activations by name ("gelu" | "relu" | "swish"); the case index i seeds the
detinit weights (50 + i), CNN weights (150 + i), inputs (200 + i), targets
(300 + i) and the backward weights R (400 + i)."""

VARIANTS = {
    # the reference's TransformerASR doctest constructor (TransformerASR.py:77-79): transformer
    # encoder, regularMHA, fixed_abs_sine, post-norm, GELU
    "doc": dict(ctor=dict(tgt_vocab=720, input_size=512, d_model=512, nhead=8, num_encoder_layers=1,
                          num_decoder_layers=1, d_ffn=1024, act="gelu"), B=2, T=24, F=512, U=10, grads=False),
    # recipes/LibriSpeech/ASR/transformer/hparams/transformer.yaml:122-150 at d_model 64 / 2 layers, with its
    # 3-block CNN front end (input_size 1280)
    "tyaml": dict(ctor=dict(tgt_vocab=50, input_size=1280, d_model=64, nhead=4, num_encoder_layers=2,
                            num_decoder_layers=1, d_ffn=128, dropout=0.1, act="gelu", encoder_module="transformer",
                            attention_type="regularMHA", normalize_before=True, causal=False),
                  cnn=True, B=3, T=41, F=80, U=9, grads=True),
    # transformer encoder with RelPosMHAXL (Transformer.py:307-310), the reference's other defaults
    # (post-norm, ReLU, causal=True -> mask_pos_future)
    "trel": dict(ctor=dict(tgt_vocab=40, input_size=40, d_model=64, nhead=4, num_encoder_layers=2,
                           num_decoder_layers=1, d_ffn=128, encoder_module="transformer",
                           attention_type="RelPosMHAXL"), B=3, T=19, F=40, U=7, grads=True),
    # ... pre-norm with a Swish FFN (the TransformerEncoder module path)
    "trels": dict(ctor=dict(tgt_vocab=40, input_size=40, d_model=64, nhead=4, num_encoder_layers=2,
                            num_decoder_layers=1, d_ffn=128, act="swish", encoder_module="transformer",
                            attention_type="RelPosMHAXL", normalize_before=True, causal=False),
                  B=2, T=23, F=40, U=6, grads=True),
    # Conformer encoder with regularMHA (Conformer.py:173-180) and the absolute sine table
    "cmha": dict(ctor=dict(tgt_vocab=40, input_size=40, d_model=64, nhead=4, num_encoder_layers=2,
                           num_decoder_layers=1, d_ffn=128, kernel_size=15, encoder_module="conformer",
                           attention_type="regularMHA", normalize_before=True, causal=False),
                 B=3, T=21, F=40, U=8, grads=True),
    # ... causal (chomped depthwise conv)
    "cmhac": dict(ctor=dict(tgt_vocab=40, input_size=40, d_model=64, nhead=4, num_encoder_layers=1,
                            num_decoder_layers=1, d_ffn=128, kernel_size=7, encoder_module="conformer",
                            attention_type="regularMHA", normalize_before=True, causal=True),
                  B=2, T=16, F=40, U=5, grads=False),
}
