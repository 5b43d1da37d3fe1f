"""Drop-in for speechbrain.lobes.models.transformer.TransformerASR — the
encoder side (TransformerASR.py:87-141 constructor, :279-316 encode).

Supported configuration (the LibriSpeech Conformer recipes,
conformer_small.yaml:132-146): encoder_module="conformer",
attention_type="RelPosMHAXL".  The module tree mirrors the reference so
encoder checkpoints load with strict=True (positional_encoding,
positional_encoding_decoder, encoder.*, custom_src_module.layers.0.w.*,
custom_tgt_module.layers.0.emb.Embedding.weight).  Decoding
(num_decoder_layers > 0 → TransformerDecoder, forward/decode) is outside the
accelerated path and raises NotImplementedError.  EncoderWrapper
(:325-356) makes encode() the forward of a DDP-wrappable module.
"""
import math
from typing import Optional

import torch
import torch.nn as nn

from .... import _autograd as A
from .... import _enc
from ....nnet.activations import Swish
from ....nnet.attention import RelPosEncXL
from ....nnet.linear import Linear
from .Conformer import ConformerEncoder

_f32 = torch.float32


class PositionalEncoding(nn.Module):
    """Transformer.py:199-243 absolute sine table (buffer `pe`, kept for
    state_dict parity; used only by the decoder)."""

    def __init__(self, input_size, max_len=2500):
        super().__init__()
        self.max_len = max_len
        pe = torch.zeros(self.max_len, input_size, requires_grad=False)
        positions = torch.arange(0, self.max_len).unsqueeze(1).float()
        denominator = torch.exp(torch.arange(0, input_size, 2).float() * -(math.log(10000.0) / input_size))
        pe[:, 0::2] = torch.sin(positions * denominator)
        pe[:, 1::2] = torch.cos(positions * denominator)
        pe = pe.unsqueeze(0)
        self.register_buffer("pe", pe)

    def forward(self, x):
        return self.pe[:, : x.size(1)].clone().detach()


class _ModuleList(nn.Module):
    """nnet/containers.py ModuleList: children under `.layers`."""

    def __init__(self, *modules):
        super().__init__()
        self.layers = nn.ModuleList(modules)


class _Embedding(nn.Module):
    """nnet/embedding.py Embedding: nn.Embedding under `.Embedding`."""

    def __init__(self, num_embeddings, embedding_dim=128, blank_id=0):
        super().__init__()
        self.Embedding = nn.Embedding(num_embeddings, embedding_dim)


class NormalizedEmbedding(nn.Module):
    """Transformer.py NormalizedEmbedding (parameters only: decoder side)."""

    def __init__(self, d_model, vocab):
        super().__init__()
        self.emb = _Embedding(num_embeddings=vocab, embedding_dim=d_model, blank_id=0)
        self.d_model = d_model


class TransformerASR(nn.Module):
    def __init__(self, tgt_vocab, input_size, d_model=512, nhead=8, num_encoder_layers=6, num_decoder_layers=6,
                 d_ffn=2048, dropout=0.1, activation=nn.ReLU, positional_encoding="fixed_abs_sine",
                 normalize_before=False, kernel_size: Optional[int] = 31, bias: Optional[bool] = True,
                 encoder_module: Optional[str] = "transformer", conformer_activation: Optional[nn.Module] = Swish,
                 attention_type: Optional[str] = "regularMHA", max_length: Optional[int] = 2500,
                 causal: Optional[bool] = True):
        super().__init__()
        if encoder_module != "conformer" or attention_type != "RelPosMHAXL":
            raise NotImplementedError("accelerated TransformerASR: encoder_module='conformer', "
                                      "attention_type='RelPosMHAXL'")
        if num_decoder_layers > 0:
            raise NotImplementedError("the Transformer decoder is outside the accelerated encoder path")
        assert num_encoder_layers > 0
        assert normalize_before, "normalize_before must be True for Conformer"
        self.causal = causal
        self.attention_type = attention_type
        self.positional_encoding_type = positional_encoding
        self.positional_encoding = RelPosEncXL(d_model)
        self.positional_encoding_decoder = PositionalEncoding(d_model, max_length)
        self.encoder = ConformerEncoder(nhead=nhead, num_layers=num_encoder_layers, d_ffn=d_ffn, d_model=d_model,
                                        dropout=dropout, activation=conformer_activation, kernel_size=kernel_size,
                                        bias=bias, causal=self.causal, attention_type=self.attention_type)
        self.custom_src_module = _ModuleList(Linear(input_size=input_size, n_neurons=d_model, bias=True,
                                                    combine_dims=False), torch.nn.Dropout(dropout))
        self.custom_tgt_module = _ModuleList(NormalizedEmbedding(d_model, tgt_vocab))
        self._init_params()

    def _init_params(self):
        for p in self.parameters():
            if p.dim() > 1:
                torch.nn.init.xavier_normal_(p)

    def forward(self, src, tgt, wav_len=None, pad_idx=0):
        raise NotImplementedError("TransformerASR.forward needs the decoder (outside the accelerated path); "
                                  "use encode()")

    def key_padding_mask(self, T, wav_len, device):
        """TransformerASR.py:295-301: arange(T) > floor(wav_len·T) (uint8)."""
        if wav_len is None:
            return None
        return _enc.length_mask(wav_len.to(device=device), T)

    def encode(self, src, wav_len=None):
        """Encoder forward (TransformerASR.py:279-316) → (B, T, d_model) fp32."""
        if src.dim() == 4:
            bz, t, ch1, ch2 = src.shape
            src = src.reshape(bz, t, ch1 * ch2)
        B, T, Fin = src.shape
        dtype = _enc.compute_dtype()
        kpm = self.key_padding_mask(T, wav_len, src.device)
        lin = self.custom_src_module.layers[0]
        drop = self.custom_src_module.layers[1]
        if A.needs_grad(self, src) or (self.training and (drop.p > 0 or self.encoder.wants_train_path(src))):
            # training path: differentiable HIP chain (_autograd)
            x = A.linear(src.reshape(B * T, Fin), lin.w.weight, lin.w.bias, dtype, lin._wc, "t_w", out_dtype=_f32)
            x = A.dropout(x, drop.p, self.training)
            pos = self.positional_encoding.table(T, src.device, _f32)
            y, _ = self.encoder.train_run(x, B, T, pos, kpm, dtype)
            return y.view(B, T, -1)
        a = _enc.to_compute(src.reshape(B * T, Fin), dtype)
        x = _enc.gemm(a, lin.kernel_weight(dtype), bias=lin.w.bias.detach(), out_dtype=_f32)
        pos = self.positional_encoding.table(T, src.device, dtype)  # a constant table: cached in the compute dtype
        y, _ = self.encoder.run(x, B, T, pos, kpm, dtype, False)
        return y.view(B, T, -1)


class EncoderWrapper(nn.Module):
    """TransformerASR.py:325-356: a module whose forward is
    transformer.encode(x, wav_lens), so the encoder can be wrapped by DDP
    (Brain._wrap_distributed wraps modules, and DDP only runs forward)."""

    def __init__(self, transformer, *args, **kwargs):
        super().__init__(*args, **kwargs)
        self.transformer = transformer

    def forward(self, x, wav_lens=None):
        return self.transformer.encode(x, wav_lens)
