"""CPU checks of the drop-in boundary: libsbk.so builds/loads without a GPU and
exports exactly the entry points include/sbk.h declares; module structure
(state_dict keys, seeded init) matches the reference fixtures; the product
package never imports the oracle and refuses CPU tensors (no fallback)."""
import ctypes
import os
import re

import numpy as np
import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _header_symbols():
    txt = open(os.path.join(ROOT, "include", "sbk.h")).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(sbk_\w+)\s*\(", txt)))


def test_header_matches_binding_table():
    from speechbrain_amd import _lib
    assert _header_symbols() == sorted(_lib.exported_symbols())


def test_library_exports_header_symbols():
    from speechbrain_amd import _lib
    if not os.path.exists(_lib.LIB_PATH):
        from speechbrain_amd import _build
        _build.build()
    lib = ctypes.CDLL(_lib.LIB_PATH)
    missing = [s for s in _header_symbols() if not hasattr(lib, s)]
    assert not missing, missing
    # host-only entry points can be called without a GPU
    assert lib.sbk_fft_supported(400) == 1
    assert lib.sbk_fft_supported(512) == 1
    assert lib.sbk_fft_supported(402) == 0  # 201 = 3 * 67: no plan
    # wide-row LayerNorm: the forward refuses the rows its backward cannot
    # take (D > 16384), before any launch (argument check only, no GPU)
    lib.sbk_layernorm_wide.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                                       ctypes.c_float, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]
    lib.sbk_layernorm_bwd.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                      ctypes.c_void_p, ctypes.c_float, ctypes.c_void_p, ctypes.c_void_p,
                                      ctypes.c_void_p, ctypes.c_void_p]
    assert lib.sbk_layernorm_wide(None, 4, 16385, None, None, 1e-5, None, 0, None) == 1001
    assert lib.sbk_layernorm_bwd(None, None, 0, 4, 16385, None, 1e-5, None, None, None, None) == 1001


def test_no_cpu_fallback():
    from speechbrain_amd.lobes.features import Fbank
    from speechbrain_amd._lib import SbkError
    with pytest.raises(SbkError):
        Fbank(n_mels=40)(torch.randn(1, 1600))


def test_product_does_not_import_oracle():
    pkg = os.path.join(ROOT, "speechbrain_amd")
    for dp, _, fs in os.walk(pkg):
        for f in fs:
            if f.endswith(".py"):
                src = open(os.path.join(dp, f)).read()
                assert not re.search(r"^\s*(import|from)\s+oracle", src, re.M), f


def _sub(g, prefix):
    return {k[len(prefix):]: torch.from_numpy(g[k]) for k in g.files if k.startswith(prefix)}


def test_state_dict_parity(golden):
    from speechbrain_amd.lobes.models.convolution import ConvolutionFrontEnd
    from speechbrain_amd.lobes.models.transformer.Conformer import ConformerEncoder
    from speechbrain_amd.lobes.models.transformer.TransformerASR import TransformerASR
    g = golden("conformer")
    tr = TransformerASR(tgt_vocab=10, input_size=640, d_model=64, nhead=4, num_encoder_layers=2,
                        num_decoder_layers=0, d_ffn=128, dropout=0.0, encoder_module="conformer",
                        attention_type="RelPosMHAXL", normalize_before=True, causal=False)
    tr.load_state_dict(_sub(g, "tr."), strict=True)
    cnn = ConvolutionFrontEnd(input_shape=(8, 10, 80), num_blocks=2, num_layers_per_block=1, out_channels=(64, 32),
                              kernel_sizes=(3, 3), strides=(2, 2), residuals=(False, False))
    cnn.load_state_dict(_sub(g, "cnn."), strict=True)
    enc = ConformerEncoder(num_layers=2, d_model=64, d_ffn=128, nhead=4, kernel_size=31)
    enc.load_state_dict(_sub(g, "enc."), strict=True)


def test_seeded_init_matches_reference_weights(golden):
    """Same torch.manual_seed → bit-identical parameters to the reference
    (module construction order is the reference's)."""
    from speechbrain_amd.lobes.models.convolution import ConvolutionFrontEnd
    from speechbrain_amd.lobes.models.transformer.TransformerASR import TransformerASR
    g = golden("conformer")
    torch.manual_seed(0)
    cnn = ConvolutionFrontEnd(input_shape=(8, 10, 80), num_blocks=2, num_layers_per_block=1, out_channels=(64, 32),
                              kernel_sizes=(3, 3), strides=(2, 2), residuals=(False, False))
    tr = TransformerASR(tgt_vocab=10, input_size=640, d_model=64, nhead=4, num_encoder_layers=2,
                        num_decoder_layers=0, d_ffn=128, dropout=0.0, encoder_module="conformer",
                        attention_type="RelPosMHAXL", normalize_before=True, causal=False)
    for k, v in cnn.state_dict().items():
        assert np.array_equal(v.numpy(), g["cnn." + k]), k
    for k, v in tr.state_dict().items():
        assert np.array_equal(v.numpy(), g["tr." + k]), k


def test_feature_module_attributes():
    from speechbrain_amd.processing.features import STFT, Filterbank, Deltas, DCT, ContextWindow
    st = STFT(sample_rate=16000)
    assert (st.win_length, st.hop_length, st.n_fft) == (400, 160, 400)
    fb = Filterbank(n_mels=40)
    assert fb.f_central.shape == (40,) and fb.multiplier == 10
    assert Deltas(input_size=20).kernel.shape == (20, 1, 5)
    with pytest.raises(ValueError):
        DCT(input_size=10, n_out=20)
    assert ContextWindow(2, 3).context_len == 6


def test_fp16_autocast_computes_fp32_not_bf16():
    """fp16 autocast (the reference's --auto_mix_prec) has no fp16 kernels:
    the modules compute in fp32 (at least as precise as the fp16 request),
    never silently in bf16; bf16 autocast selects bf16."""
    import torch
    from speechbrain_amd import _enc
    prev = (torch.is_autocast_enabled("cuda"), torch.get_autocast_dtype("cuda"))
    try:
        torch.set_autocast_enabled("cuda", True)
        torch.set_autocast_dtype("cuda", torch.float16)
        assert _enc.compute_dtype() == torch.float32
        torch.set_autocast_dtype("cuda", torch.bfloat16)
        assert _enc.compute_dtype() == torch.bfloat16
    finally:
        torch.set_autocast_enabled("cuda", prev[0])
        torch.set_autocast_dtype("cuda", prev[1])
    assert _enc.compute_dtype() == torch.float32


def test_brain_fp16_amp_uses_grad_scaler():
    import torch
    from speechbrain_amd.core import Brain
    b = Brain(modules={}, run_opts={"device": "cpu", "auto_mix_prec": "fp16"})
    assert b.amp_dtype == torch.float16 and b.scaler is not None
    assert Brain(modules={}, run_opts={"device": "cpu", "auto_mix_prec": True}).amp_dtype is not None
