"""Drop-in for speechbrain.lobes.models.transformer.TransformerASR
(TransformerASR.py:87-141 constructor over TransformerInterface,
Transformer.py:83-192; :143-211 forward, :213-247 make_masks, :236-277
decode, :279-316 encode).

Every constructor variant of the reference builds the reference's module
tree, so a recipe checkpoint — decoder included — loads with strict=True:
  encoder_module "conformer" | "transformer" (Transformer.py:141-175),
  attention_type "RelPosMHAXL" | "regularMHA" (:131-135; the rel-pos table
  overrides the absolute one, and the decoder then takes
  positional_encoding_decoder), positional_encoding "fixed_abs_sine" | None.
The metric configuration (the LibriSpeech Conformer recipes,
conformer_small.yaml:132-146: conformer + RelPosMHAXL) runs encode() as the
fused HIP schedule of ConformerEncoder.run; the other combinations run the
drop-in encoder modules (TransformerEncoder's fused step for the
transformer.yaml recipe's regularMHA pre-norm GELU stack,
recipes/LibriSpeech/ASR/transformer/hparams/transformer.yaml:133-150; the
module path with RelPosMHAXL or regularMHA in the Conformer layers).  The
attention decoder (forward / decode) runs the reference's semantics on the
HIP drop-ins (LayerNorm, PositionalwiseFeedForward, MultiheadAttention's
general path).  EncoderWrapper (:324-356) makes encode() the forward of a
DDP-wrappable module.
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
from .Conformer import PAD_D, ConformerEncoder
from .Transformer import (NormalizedEmbedding, PositionalEncoding, TransformerDecoder, TransformerEncoder,
                          get_key_padding_mask, get_lookahead_mask)

_f32 = torch.float32
_bf16 = torch.bfloat16


class _ModuleList(nn.Module):
    """nnet/containers.py ModuleList: children under `.layers`, applied in order."""

    def __init__(self, *modules):
        super().__init__()
        self.layers = nn.ModuleList(modules)

    def forward(self, x):
        for layer in self.layers:
            x = layer(x)
        return x


class TransformerASR(nn.Module):
    def __init__(self, tgt_vocab, input_size, d_model=512, nhead=8, num_encoder_layers=6, num_decoder_layers=6,
                 d_ffn=2048, dropout=0.1, activation=nn.ReLU, positional_encoding="fixed_abs_sine",
                 normalize_before=False, kernel_size: Optional[int] = 31, bias: Optional[bool] = True,
                 encoder_module: Optional[str] = "transformer", conformer_activation: Optional[nn.Module] = Swish,
                 attention_type: Optional[str] = "regularMHA", max_length: Optional[int] = 2500,
                 causal: Optional[bool] = True):
        super().__init__()
        # TransformerInterface.__init__ (Transformer.py:108-192)
        self.causal = causal
        self.attention_type = attention_type
        self.positional_encoding_type = positional_encoding
        self.encoder_kdim = self.encoder_vdim = self.decoder_kdim = self.decoder_vdim = None
        assert attention_type in ["regularMHA", "RelPosMHAXL"]
        assert positional_encoding in ["fixed_abs_sine", None]
        assert num_encoder_layers + num_decoder_layers > 0, \
            "number of encoder layers and number of decoder layers cannot both be 0!"
        if positional_encoding == "fixed_abs_sine":
            self.positional_encoding = PositionalEncoding(d_model, max_length)
        if attention_type == "RelPosMHAXL":  # overrides any other pos_embedding (:130-135)
            self.positional_encoding = RelPosEncXL(d_model)
            self.positional_encoding_decoder = PositionalEncoding(d_model, max_length)
        self.encoder_module = encoder_module
        if num_encoder_layers > 0:
            if encoder_module == "transformer":
                self.encoder = TransformerEncoder(nhead=nhead, num_layers=num_encoder_layers, d_ffn=d_ffn,
                                                  d_model=d_model, dropout=dropout, activation=activation,
                                                  normalize_before=normalize_before, causal=self.causal,
                                                  attention_type=self.attention_type)
            elif encoder_module == "conformer":
                self.encoder = ConformerEncoder(nhead=nhead, num_layers=num_encoder_layers, d_ffn=d_ffn,
                                                d_model=d_model, dropout=dropout, activation=conformer_activation,
                                                kernel_size=kernel_size, bias=bias, causal=self.causal,
                                                attention_type=self.attention_type)
                assert normalize_before, "normalize_before must be True for Conformer"
                assert conformer_activation is not None, "conformer_activation must not be None"
        if num_decoder_layers > 0:  # always regularMHA, causal (:177-192)
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

    def _fast_encoder(self):
        """The fused Conformer schedule (ConformerEncoder.run) applies."""
        return (self.encoder_module == "conformer" and self.attention_type == "RelPosMHAXL"
                and not self.encoder.layers[0].module_layer)

    def _abs_pe(self, x):
        """x + the absolute sine table (TransformerASR.py:173-174, 307-308).
        With positional_encoding=None and regularMHA the reference never sets
        its positional term and fails (UnboundLocalError at :177-182 /
        :311-315); the drop-in raises a ValueError there."""
        if self.positional_encoding_type == "fixed_abs_sine":
            return x + self.positional_encoding(x)
        raise ValueError("TransformerASR(positional_encoding=None, attention_type='regularMHA'): the reference "
                         "leaves the positional embeddings unset here (TransformerASR.py:304-315)")

    def forward(self, src, tgt, wav_len=None, pad_idx=0):
        """TransformerASR.py:143-211 → (encoder_out, decoder_out).  The src key
        padding mask is make_masks' (positions ≥ round(wav_len·T), unlike
        encode()'s > floor(wav_len·T)); the decoder takes the reference's
        lookahead and target padding masks."""
        if not hasattr(self, "decoder"):
            raise ValueError("TransformerASR.forward needs num_decoder_layers > 0 (use encode())")
        if src.dim() == 4:
            bz, t, ch1, ch2 = src.shape
            src = src.reshape(bz, t, ch1 * ch2)
        src_kpm, tgt_kpm, src_mask, tgt_mask = self.make_masks(src, tgt, wav_len, pad_idx=pad_idx)
        if src_kpm is not None and src_kpm.shape[1] != src.shape[1]:
            # neither the reference's rel-pos attention nor torch's MHA takes a narrower mask
            raise ValueError(f"src key padding mask width {src_kpm.shape[1]} != T = {src.shape[1]} "
                             "(no utterance fills the batch: max(wav_len) < 1)")
        if self._fast_encoder():
            encoder_out = self._encode(src, kpm=src_kpm)
        else:
            encoder_out = self._module_encode(src, src_kpm, src_mask)
        tgt = self.custom_tgt_module(tgt)
        if self.attention_type == "RelPosMHAXL":
            tgt = tgt + self.positional_encoding_decoder(tgt)
            encoder_out = encoder_out + self.positional_encoding_decoder(encoder_out)
        else:
            tgt = self._abs_pe(tgt)
        decoder_out, _, _ = self.decoder(tgt=tgt, memory=encoder_out, memory_mask=src_mask, tgt_mask=tgt_mask,
                                         tgt_key_padding_mask=tgt_kpm, memory_key_padding_mask=src_kpm)
        return encoder_out, decoder_out

    def make_masks(self, src, tgt, wav_len=None, pad_idx=0):
        """TransformerASR.py:213-234."""
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
        """TransformerASR.py:236-277 → (prediction, last cross-attention map)."""
        if not hasattr(self, "decoder"):
            raise ValueError("TransformerASR.decode needs num_decoder_layers > 0")
        tgt_mask = get_lookahead_mask(tgt)
        src_key_padding_mask = None
        if enc_len is not None:
            el = enc_len.to(encoder_out.device)
            src_key_padding_mask = ~(torch.arange(int(el.max().long().item()), device=el.device,
                                                  dtype=el.dtype)[None, :] < el[:, None])
        tgt = self.custom_tgt_module(tgt)
        if self.attention_type == "RelPosMHAXL":
            tgt = tgt + self.positional_encoding_decoder(tgt)
            encoder_out = encoder_out + self.positional_encoding_decoder(encoder_out)
        else:
            tgt = self._abs_pe(tgt)
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
        if self._fast_encoder():
            return self._encode(src, wav_len)
        kpm = self.key_padding_mask(src.shape[1], wav_len, src.device)
        return self._module_encode(src, None if kpm is None else kpm.bool())

    def _module_encode(self, src, kpm, src_mask=None):
        """TransformerASR.py:303-316 (and :169-182) on the drop-in modules, for
        every encoder / attention combination but the fused Conformer one: the
        src Linear (MFMA GEMM) + dropout, the rel-pos table or the absolute
        sine term, then the encoder module (TransformerEncoder's fused step or
        its module path; the Conformer's regularMHA layers)."""
        B, T, Fin = src.shape
        dtype = _enc.compute_dtype()
        lin = self.custom_src_module.layers[0]
        drop = self.custom_src_module.layers[1]
        x = A.linear(src.reshape(B * T, Fin), lin.w.weight, lin.w.bias, dtype, lin._wc, "t_w", out_dtype=_f32)
        x = A.dropout(x, drop.p, self.training).view(B, T, -1)
        pos = None
        if self.attention_type == "RelPosMHAXL":
            pos = self.positional_encoding(x)
        else:
            x = self._abs_pe(x)
        y, _ = self.encoder(src=x, src_mask=src_mask, src_key_padding_mask=kpm, pos_embs=pos)
        return y

    def _encode(self, src, wav_len=None, kpm=None):
        """Fused Conformer path: src (B, T, F) and the relative lengths (or
        None) or a ready key padding mask (forward's make_masks) → encoder
        output.  (Running the key padding mask and the linear_pos GEMM on a
        side stream beside the src Linear measured 20-30 us slower per
        step: profiles/r06o_preamble_side_stream_ab_rejected.log.)"""
        B, T, Fin = src.shape
        dtype = _enc.compute_dtype()
        lin = self.custom_src_module.layers[0]
        drop = self.custom_src_module.layers[1]
        if A.needs_grad(self, src) or (self.training and (drop.p > 0 or self.encoder.wants_train_path(src))):
            # training path: differentiable HIP chain (_autograd)
            kpm = self._kpm(T, wav_len, kpm, src.device)
            x = A.linear(src.reshape(B * T, Fin), lin.w.weight, lin.w.bias, dtype, lin._wc, "t_w", out_dtype=_f32)
            x = A.dropout(x, drop.p, self.training)
            pos = self.positional_encoding.table(T, src.device, _f32)
            y, _ = self.encoder.train_run(x, B, T, pos, kpm, dtype)
            return y.view(B, T, -1)
        kpm = self._kpm(T, wav_len, kpm, src.device)
        pos = self.positional_encoding.table(T, src.device, dtype)  # a constant table: cached in the compute dtype
        a = _enc.to_compute(src.reshape(B * T, Fin), dtype)
        sh = self.encoder._shadow(lin.w.weight.shape[0], dtype)
        if sh is not None:
            # d_model < 256 on the padded shadow: the src Linear writes the
            # 256-wide zero-padded input itself (no fill + copy launches)
            w, b = self._padded_src(dtype)
            y, _ = sh.run(_enc.gemm(a, w, bias=b, out_dtype=_f32), B, T, pos, kpm, dtype, False)
        else:
            x = _enc.gemm(a, lin.kernel_weight(dtype), bias=lin.w.bias.detach(), out_dtype=_f32)
            y, _ = self.encoder.run(x, B, T, pos, kpm, dtype, False)
        return y.view(B, T, -1)

    def _kpm(self, T, wav_len, kpm, device):
        """uint8 (B, T) key padding mask: the given one, or from wav_len."""
        if kpm is not None:
            return kpm.to(device=device, dtype=torch.uint8).contiguous()
        return self.key_padding_mask(T, wav_len, device)

    def _padded_src(self, dtype):
        """The src Linear with its output rows zero-padded to the encoder
        shadow's 256 channels (weight in the compute dtype, fp32 bias)."""
        lin = self.custom_src_module.layers[0]
        ps = [lin.w.weight] + ([lin.w.bias] if lin.w.bias is not None else [])

        def make():
            wt = lin.w.weight.detach()
            w = torch.zeros(PAD_D, wt.shape[1], device=wt.device, dtype=torch.float32)
            w[:wt.shape[0]] = wt
            b = torch.zeros(PAD_D, device=wt.device, dtype=torch.float32)
            if lin.w.bias is not None:
                b[:wt.shape[0]] = lin.w.bias.detach()
            return (_enc.cast_bf16(w) if dtype == _bf16 else w), b
        return lin._wc.get(("pad", dtype), ps, make)


class EncoderWrapper(nn.Module):
    """TransformerASR.py:325-356: a module whose forward is
    transformer.encode(x, wav_lens), so the encoder can be wrapped by DDP
    (Brain._wrap_distributed wraps modules, and DDP only runs forward)."""

    def __init__(self, transformer, *args, **kwargs):
        super().__init__(*args, **kwargs)
        self.transformer = transformer

    def forward(self, x, wav_lens=None):
        return self.transformer.encode(x, wav_lens)
