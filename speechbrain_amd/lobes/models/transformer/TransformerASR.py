"""Drop-in for speechbrain.lobes.models.transformer.TransformerASR
(TransformerASR.py:87-141 constructor, :143-211 forward, :213-247
make_masks, :249-300 decode, :279-316 encode).

Accelerated configuration (the LibriSpeech Conformer recipes,
conformer_small.yaml:132-146): encoder_module="conformer",
attention_type="RelPosMHAXL"; encode() runs on the HIP kernels.  The module
tree mirrors the reference (positional_encoding, positional_encoding_decoder,
encoder.*, decoder.* when num_decoder_layers > 0,
custom_src_module.layers.0.w.*, custom_tgt_module.layers.0.emb.Embedding.weight),
so a recipe checkpoint — decoder included — loads with strict=True.  The
attention decoder (forward / decode) keeps the reference's semantics with its
LayerNorms and FFNs on the HIP drop-ins and its masked attentions on the
wrapped torch.nn.MultiheadAttention (outside the accelerated path).
EncoderWrapper (:325-356) makes encode() the forward of a DDP-wrappable module.
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
from .Transformer import NormalizedEmbedding, TransformerDecoder, get_key_padding_mask, get_lookahead_mask

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
        if num_decoder_layers > 0:  # Transformer.py:177-192 (always regularMHA, causal)
            self.decoder = TransformerDecoder(num_layers=num_decoder_layers, nhead=nhead, d_ffn=d_ffn, d_model=d_model,
                                              dropout=dropout, activation=activation,
                                              normalize_before=normalize_before, causal=True,
                                              attention_type="regularMHA")
        self.custom_src_module = _ModuleList(Linear(input_size=input_size, n_neurons=d_model, bias=True,
                                                    combine_dims=False), torch.nn.Dropout(dropout))
        self.custom_tgt_module = _ModuleList(NormalizedEmbedding(d_model, tgt_vocab))
        self._init_params()

    def _init_params(self):
        for p in self.parameters():
            if p.dim() > 1:
                torch.nn.init.xavier_normal_(p)

    def forward(self, src, tgt, wav_len=None, pad_idx=0):
        """TransformerASR.py:143-211 → (encoder_out, decoder_out).  The encoder
        runs on HIP with make_masks' src key padding mask (positions ≥
        round(wav_len·T), unlike encode()'s > floor(wav_len·T)); the decoder
        with the reference's lookahead and target padding masks."""
        if not hasattr(self, "decoder"):
            raise ValueError("TransformerASR.forward needs num_decoder_layers > 0 (use encode())")
        if src.dim() == 4:
            bz, t, ch1, ch2 = src.shape
            src = src.reshape(bz, t, ch1 * ch2)
        src_kpm, tgt_kpm, src_mask, tgt_mask = self.make_masks(src, tgt, wav_len, pad_idx=pad_idx)
        if src_kpm is not None and src_kpm.shape[1] != src.shape[1]:
            # the reference's rel-pos attention cannot view a narrower mask as (B, 1, 1, T) either
            raise ValueError(f"src key padding mask width {src_kpm.shape[1]} != T = {src.shape[1]} "
                             "(no utterance fills the batch: max(wav_len) < 1)")
        encoder_out = self._encode(src, None if src_kpm is None else src_kpm.to(torch.uint8))
        tgt = self.custom_tgt_module.layers[0](tgt)
        tgt = tgt + self.positional_encoding_decoder(tgt)
        encoder_out = encoder_out + self.positional_encoding_decoder(encoder_out)
        decoder_out, _, _ = self.decoder(tgt=tgt, memory=encoder_out, memory_mask=src_mask, tgt_mask=tgt_mask,
                                         tgt_key_padding_mask=tgt_kpm, memory_key_padding_mask=src_kpm)
        return encoder_out, decoder_out

    def make_masks(self, src, tgt, wav_len=None, pad_idx=0):
        """TransformerASR.py:213-247."""
        src_key_padding_mask = None
        if wav_len is not None:
            abs_len = torch.round(wav_len * src.shape[1])
            # ~length_to_mask(abs_len): its width is max(abs_len), which is T
            # whenever the longest utterance fills the batch (wav_len max 1)
            width = int(abs_len.max().long().item())
            src_key_padding_mask = ~(torch.arange(width, device=abs_len.device, dtype=abs_len.dtype)[None, :]
                                     < abs_len[:, None])
            src_key_padding_mask = src_key_padding_mask.to(src.device)
        tgt_key_padding_mask = get_key_padding_mask(tgt, pad_idx=pad_idx)
        src_mask = None
        tgt_mask = get_lookahead_mask(tgt)
        return src_key_padding_mask, tgt_key_padding_mask, src_mask, tgt_mask

    @torch.no_grad()
    def decode(self, tgt, encoder_out, enc_len=None):
        """TransformerASR.py:249-300 → (prediction, last cross-attention map)."""
        if not hasattr(self, "decoder"):
            raise ValueError("TransformerASR.decode needs num_decoder_layers > 0")
        tgt_mask = get_lookahead_mask(tgt)
        src_key_padding_mask = None
        if enc_len is not None:
            el = enc_len.to(encoder_out.device)
            src_key_padding_mask = ~(torch.arange(int(el.max().long().item()), device=el.device,
                                                  dtype=el.dtype)[None, :] < el[:, None])
        tgt = self.custom_tgt_module.layers[0](tgt)
        tgt = tgt + self.positional_encoding_decoder(tgt)
        encoder_out = encoder_out + self.positional_encoding_decoder(encoder_out)
        prediction, self_attns, multihead_attns = self.decoder(tgt, encoder_out, tgt_mask=tgt_mask,
                                                               memory_key_padding_mask=src_key_padding_mask)
        return prediction, multihead_attns[-1]

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
        return self._encode(src, self.key_padding_mask(src.shape[1], wav_len, src.device))

    def _encode(self, src, kpm):
        """src (B, T, F) and a uint8 key padding mask (B, T) or None → encoder output."""
        B, T, Fin = src.shape
        dtype = _enc.compute_dtype()
        if kpm is not None:
            kpm = kpm.to(device=src.device, dtype=torch.uint8).contiguous()
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
