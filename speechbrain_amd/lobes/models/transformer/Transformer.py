"""Drop-in for speechbrain.lobes.models.transformer.Transformer
(PositionalEncoding :201-243, TransformerEncoderLayer :246-376,
TransformerEncoder :379-486) on HIP kernels — the encoder of config 5
(wav2vec2: 24 layers, d = 1024, 16 heads, d_ffn 4096, GELU, pre-norm).

State-dict keys match the reference (layers.N.self_att.att.*,
layers.N.pos_ffn.ffn.{0,3}.*, layers.N.norm{1,2}.norm.*, norm.norm.*).

Per layer (normalize_before=True; post-norm mirrors the reference order):
  u  = LN1(x)                         sbk_ln_act  (→ MXFP8 / bf16 / fp32)
  qkv = u·W_inᵀ + b                   GEMM (per-head [q|k|v] rows)
  o  = softmax(q·kᵀ/√dh + mask)·v     fused attention kernel
  x  = x + o·W_outᵀ + b               GEMM, residual in the epilogue
  u  = LN2(x)                         sbk_ln_act
  h  = act(u·W1ᵀ + b1)                GEMM, activation in the epilogue
                                      (MXFP8 output: block scales computed
                                      in the epilogue, no extra pass)
  x  = x + h·W2ᵀ + b2                 GEMM, residual in the epilogue
Compute mode: fp32 (exact-f32 MFMA) by default, bf16 under
torch.autocast(bf16), MXFP8 GEMMs under speechbrain_amd.mxfp8().
"""
import math
from typing import Optional

import numpy as np
import torch
import torch.nn as nn

from .... import _enc
from .... import _autograd as A
from ....nnet.attention import FUSED_DH_MAX, MultiheadAttention, PositionalwiseFeedForward, RelPosMHAXL, _mode_weight
from ....nnet.normalization import LayerNorm

__all__ = ["PositionalEncoding", "TransformerEncoderLayer", "TransformerEncoder", "TransformerDecoderLayer",
           "TransformerDecoder", "NormalizedEmbedding", "get_key_padding_mask", "get_lookahead_mask"]

_f32, _bf16 = torch.float32, torch.bfloat16


class PositionalEncoding(nn.Module):
    """Transformer.py:201-243 (buffer `pe` (1, max_len, d), as the reference)."""

    def __init__(self, input_size, max_len=2500):
        super().__init__()
        self.max_len = max_len
        pe = torch.zeros(self.max_len, input_size, requires_grad=False)
        positions = torch.arange(0, self.max_len).unsqueeze(1).float()
        denominator = torch.exp(torch.arange(0, input_size, 2).float() * -(math.log(10000.0) / input_size))
        pe[:, 0::2] = torch.sin(positions * denominator)
        pe[:, 1::2] = torch.cos(positions * denominator)
        self.register_buffer("pe", pe.unsqueeze(0))

    def forward(self, x):
        return self.pe[:, : x.size(1)].clone().detach()


def _mode():
    """Compute mode of the GEMMs: "mx" under speechbrain_amd.mxfp8(), else the
    autocast dtype (bf16) or fp32."""
    if _enc.mx_enabled():
        return "mx"
    return _enc.compute_dtype()


def _act_dtype(mode):
    """Dtype of activations between kernels (attention runs bf16 under mx)."""
    return _bf16 if mode in ("mx", _bf16) else _f32


class TransformerEncoderLayer(nn.Module):
    def __init__(self, d_ffn, nhead, d_model, kdim=None, vdim=None, dropout=0.0, activation=nn.ReLU,
                 normalize_before=False, attention_type="regularMHA", causal=False):
        super().__init__()
        if attention_type == "regularMHA":
            self.self_att = MultiheadAttention(nhead=nhead, d_model=d_model, dropout=dropout, kdim=kdim, vdim=vdim)
        elif attention_type == "RelPosMHAXL":
            self.self_att = RelPosMHAXL(d_model, nhead, dropout, mask_pos_future=causal)
        self.attention_type = attention_type
        self.pos_ffn = PositionalwiseFeedForward(d_ffn=d_ffn, input_size=d_model, dropout=dropout,
                                                 activation=activation)
        self.norm1 = LayerNorm(d_model, eps=1e-6)
        self.norm2 = LayerNorm(d_model, eps=1e-6)
        self.dropout1 = torch.nn.Dropout(dropout)
        self.dropout2 = torch.nn.Dropout(dropout)
        self.normalize_before = normalize_before
        self._wc = _enc.WeightCache()

    # ------------------------------------------------------------ kernels
    @staticmethod
    def _ln(mod):
        n = mod.norm
        return n.weight.detach(), n.bias.detach(), n.eps

    def _gemm_mode(self, mode, K, N):
        """MXFP8 needs K and N multiples of the 128 tile; others run bf16."""
        if mode == "mx" and (K % 128 or N % 128):
            return _bf16
        return mode

    def _norm(self, x, mod, mode):
        """LayerNorm of the fp32 stream into the next GEMM's operand format."""
        from .... import _w2v
        out = "mx" if mode == "mx" else mode
        return _w2v.ln_act(x, self._ln(mod), None, out)

    def _to(self, x, mode):
        """An activation (bf16 / fp32) as the operand of a GEMM in `mode`."""
        from .... import _w2v
        if mode == "mx":
            return _w2v.ln_act(x, None, None, "mx")
        return _enc.to_compute(x, mode)

    def _gemm(self, a, w, bias, mode, act=None, res=None, out=_f32):
        from .... import _w2v
        if mode == "mx":
            return _w2v.mx_gemm(a, w, bias=bias, act=act, res=res, out=out)
        act_name = {None: None, "gelu": "gelu", "relu": "leaky_relu"}[act]
        return _enc.gemm(a, w, bias=bias, act=act_name, slope=0.0, res=res, out_dtype=out)

    def ffn_weights(self, mode, which):
        lin = self.pos_ffn.ffn[0 if which == 1 else 3]
        return self._wc.get(("ffn", which, str(mode)), [lin.weight],
                            lambda: _mode_weight(lin.weight.detach().contiguous(), mode))

    def _act(self):
        name, slope = self.pos_ffn.act_name()
        if name == "leaky_relu" and slope == 0.0:
            name = "relu"
        if name not in ("gelu", "relu", "swish"):
            raise NotImplementedError(f"activation {name} is not on the TransformerEncoder HIP path")
        if name == "swish":
            raise NotImplementedError("Swish FFN is not on the TransformerEncoder HIP path")
        return name

    def run(self, x, B, T, kpm_u8, mode, need_weights):
        """One layer on the fp32 residual stream x (B*T, d)."""
        if self.attention_type != "regularMHA":
            raise NotImplementedError("TransformerEncoderLayer(RelPosMHAXL) is not on the HIP path")
        att = self.self_att
        att._check()
        d = x.shape[1]
        f1, f2 = self.pos_ffn.ffn[0], self.pos_ffn.ffn[3]
        m_qkv = self._gemm_mode(mode, d, 3 * d)
        m_out = self._gemm_mode(mode, d, d)
        m_f1 = self._gemm_mode(mode, d, f1.out_features)
        m_f2 = self._gemm_mode(mode, f1.out_features, d)
        pre = self.normalize_before
        u = self._norm(x, self.norm1, m_qkv) if pre else self._to(x, m_qkv)
        w_in, b_in = att.qkv_weights(m_qkv)
        qkv = self._gemm(u, w_in, b_in, m_qkv, out=_act_dtype(mode))
        o, probs = att.attend(qkv, B, T, kpm_u8, need_weights)
        x = self._gemm(self._to(o, m_out), att.out_weights(m_out), att.att.out_proj.bias.detach().float(), m_out,
                       res=x)
        if not pre:
            x = _enc.layernorm(x, *self._ln(self.norm1), out1_dtype=_f32)[0]
        u = self._norm(x, self.norm2, m_f1) if pre else self._to(x, m_f1)
        # hidden activation: MXFP8 straight from the FFN1 epilogue when both
        # FFN GEMMs are MXFP8, else bf16 / fp32 (quantised for an MXFP8 FFN2)
        h_out = "mx" if (m_f1 == "mx" and m_f2 == "mx") else _act_dtype(mode)
        h = self._gemm(u, self.ffn_weights(m_f1, 1), f1.bias.detach().float(), m_f1, act=self._act(), out=h_out)
        if m_f2 == "mx" and h_out != "mx":
            h = self._to(h, "mx")
        x = self._gemm(h, self.ffn_weights(m_f2, 2), f2.bias.detach().float(), m_f2, res=x)
        if not pre:
            x = _enc.layernorm(x, *self._ln(self.norm2), out1_dtype=_f32)[0]
        return x, (probs.mean(dim=1) if probs is not None else None)

    def module_forward(self, src, src_mask=None, src_key_padding_mask=None, pos_embs=None):
        """Transformer.py:343-376 step by step on the drop-in submodules — the
        attention's differentiable path (masks, pos_embs, dropout,
        gradients), the HIP LayerNorm / FFN autograd Functions, the residual
        adds with their dropout as one HIP launch each — for everything the
        fused inference step does not take (RelPosMHAXL self-attention,
        Transformer.py:307-310, runs its own fused kernel inside)."""
        src1 = self.norm1(src) if self.normalize_before else src
        if self.attention_type == "RelPosMHAXL":
            output, self_attn = self.self_att(src1, src1, src1, pos_embs, key_padding_mask=src_key_padding_mask,
                                              attn_mask=src_mask)
        else:
            output, self_attn = self.self_att(src1, src1, src1, attn_mask=src_mask,
                                              key_padding_mask=src_key_padding_mask, pos_embs=pos_embs)
        tr = self.training
        src = _add_drop(src, output, self.dropout1.p if tr else 0.0)
        if not self.normalize_before:
            src = self.norm1(src)
        src1 = self.norm2(src) if self.normalize_before else src
        output = _add_drop(src, self.pos_ffn(src1), self.dropout2.p if tr else 0.0)
        if not self.normalize_before:
            output = self.norm2(output)
        return output, self_attn

    def _fused_ok(self, src, src_mask, pos_embs, kpm=None):
        """The fused inference step takes: regularMHA self-attention in the
        default projection layout, no src_mask / pos_embs, a bool / byte key
        padding mask (an additive float one goes to the module path, as in
        MultiheadAttention), a GELU / ReLU FFN, no gradients, no dropout."""
        if not (src_mask is None and pos_embs is None and self.attention_type == "regularMHA"
                and (kpm is None or kpm.dtype in (torch.bool, torch.uint8))
                and not A.needs_grad(self, src) and not (self.training and self.dropout1.p > 0)):
            return False
        a = self.self_att.att
        if (not a._qkv_same_embed_dim or a.bias_k is not None or a.add_zero_attn or a.in_proj_bias is None
                or a.head_dim > FUSED_DH_MAX):
            return False
        try:
            name, slope = self.pos_ffn.act_name()
        except NotImplementedError:
            return False
        return name == "gelu" or (name in ("relu", "leaky_relu") and slope == 0.0)

    def forward(self, src, src_mask: Optional[torch.Tensor] = None,
                src_key_padding_mask: Optional[torch.Tensor] = None, pos_embs: Optional[torch.Tensor] = None):
        if not self._fused_ok(src, src_mask, pos_embs, src_key_padding_mask):
            return self.module_forward(src, src_mask, src_key_padding_mask, pos_embs)
        B, T, d = src.shape
        kpm = src_key_padding_mask.to(torch.uint8).contiguous() if src_key_padding_mask is not None else None
        y, attn = self.run(src.float().reshape(B * T, d).contiguous(), B, T, kpm, _mode(), True)
        return y.view(B, T, d), attn


def _add_drop(res, y, p):
    """res + Dropout(p)(y) (Transformer.py:359,370) as one HIP launch, differentiable."""
    shp = res.shape
    d = shp[-1]
    r = res.float().reshape(-1, d).contiguous()
    return A.DropAddFn.apply(y.float().reshape(-1, d).contiguous(), r, 1.0, None, float(p), _f32).view(shp)


class TransformerEncoder(nn.Module):
    def __init__(self, num_layers, nhead, d_ffn, input_shape=None, d_model=None, kdim=None, vdim=None, dropout=0.0,
                 activation=nn.ReLU, normalize_before=False, causal=False, layerdrop_prob=0.0,
                 attention_type="regularMHA"):
        super().__init__()
        self.layers = torch.nn.ModuleList([
            TransformerEncoderLayer(d_ffn=d_ffn, nhead=nhead, d_model=d_model, kdim=kdim, vdim=vdim, dropout=dropout,
                                    activation=activation, normalize_before=normalize_before, causal=causal,
                                    attention_type=attention_type) for _ in range(num_layers)])
        self.norm = LayerNorm(d_model, eps=1e-6)
        self.layerdrop_prob = layerdrop_prob
        self.rng = np.random.default_rng()

    def run(self, x2d, B, T, kpm_u8, need_weights):
        """(B*T, d) fp32 → (B*T, d) fp32 after the closing LayerNorm, [attn]."""
        mode = _mode()
        attns = []
        keep = self.rng.random(len(self.layers)) if (self.training and self.layerdrop_prob > 0.0) else None
        for i, layer in enumerate(self.layers):
            if keep is None or keep[i] > self.layerdrop_prob:
                x2d, a = layer.run(x2d, B, T, kpm_u8, mode, need_weights)
                attns.append(a)
        n = self.norm.norm
        return _enc.layernorm(x2d, n.weight.detach(), n.bias.detach(), n.eps, out1_dtype=_f32)[0], attns

    def forward(self, src, src_mask: Optional[torch.Tensor] = None,
                src_key_padding_mask: Optional[torch.Tensor] = None, pos_embs: Optional[torch.Tensor] = None):
        if not all(l._fused_ok(src, src_mask, pos_embs, src_key_padding_mask) for l in self.layers):
            # Transformer.py:448-486 with the layers' module path
            keep = self.rng.random(len(self.layers)) if self.layerdrop_prob > 0.0 else None
            out, attns = src, []
            for i, layer in enumerate(self.layers):
                if not self.training or self.layerdrop_prob == 0.0 or keep[i] > self.layerdrop_prob:
                    out, a = layer(out, src_mask=src_mask, src_key_padding_mask=src_key_padding_mask,
                                   pos_embs=pos_embs)
                    attns.append(a)
            return self.norm(out), attns
        B, T, d = src.shape
        kpm = src_key_padding_mask.to(torch.uint8).contiguous() if src_key_padding_mask is not None else None
        y, attns = self.run(src.float().reshape(B * T, d).contiguous(), B, T, kpm, True)
        return y.view(B, T, d), attns


# ---------------------------------------------------------------------------
# Decoder side (Transformer.py:489-797): TransformerDecoderLayer,
# TransformerDecoder, NormalizedEmbedding.  The decoder is outside the
# accelerated path (attention decoders OUT); it exists so that a
# recipe's TransformerASR(num_decoder_layers > 0) constructs with the
# reference's module tree and state_dict keys, loads its checkpoint with
# strict=True, and runs forward()/decode() with the reference's semantics.
# Its LayerNorms, FFNs and its masked self- and cross-attention are the HIP
# drop-ins (nnet.normalization.LayerNorm, nnet.attention
# .PositionalwiseFeedForward, the MultiheadAttention's general path on
# csrc/xattn.hip: attn_mask, key padding, pos_embs, S != L).
# ---------------------------------------------------------------------------


class TransformerDecoderLayer(nn.Module):
    """Transformer.py:489-654 (regularMHA; the decoder TransformerASR builds)."""

    def __init__(self, d_ffn, nhead, d_model, kdim=None, vdim=None, dropout=0.0, activation=nn.ReLU,
                 normalize_before=False, attention_type="regularMHA", causal=None):
        super().__init__()
        if attention_type != "regularMHA":
            raise NotImplementedError("TransformerDecoderLayer: attention_type='regularMHA' (what TransformerASR "
                                      "builds, Transformer.py:180-192)")
        self.nhead = nhead
        self.self_attn = MultiheadAttention(nhead=nhead, d_model=d_model, kdim=kdim, vdim=vdim, dropout=dropout)
        self.mutihead_attn = MultiheadAttention(nhead=nhead, d_model=d_model, kdim=kdim, vdim=vdim, dropout=dropout)
        self.pos_ffn = PositionalwiseFeedForward(d_ffn=d_ffn, input_size=d_model, dropout=dropout,
                                                 activation=activation)
        self.norm1 = LayerNorm(d_model, eps=1e-6)
        self.norm2 = LayerNorm(d_model, eps=1e-6)
        self.norm3 = LayerNorm(d_model, eps=1e-6)
        self.dropout1 = nn.Dropout(dropout)
        self.dropout2 = nn.Dropout(dropout)
        self.dropout3 = nn.Dropout(dropout)
        self.normalize_before = normalize_before

    def forward(self, tgt, memory, tgt_mask=None, memory_mask=None, tgt_key_padding_mask=None,
                memory_key_padding_mask=None, pos_embs_tgt=None, pos_embs_src=None):
        tgt1 = self.norm1(tgt) if self.normalize_before else tgt
        tgt2, self_attn = self.self_attn(tgt1, tgt1, tgt1, attn_mask=tgt_mask, key_padding_mask=tgt_key_padding_mask,
                                         pos_embs=pos_embs_tgt)
        tgt = tgt + self.dropout1(tgt2)
        if not self.normalize_before:
            tgt = self.norm1(tgt)
        tgt1 = self.norm2(tgt) if self.normalize_before else tgt
        tgt2, multihead_attention = self.mutihead_attn(tgt1, memory, memory, attn_mask=memory_mask,
                                                       key_padding_mask=memory_key_padding_mask, pos_embs=pos_embs_src)
        tgt = tgt + self.dropout2(tgt2)
        if not self.normalize_before:
            tgt = self.norm2(tgt)
        tgt1 = self.norm3(tgt) if self.normalize_before else tgt
        tgt2 = self.pos_ffn(tgt1)
        tgt = tgt + self.dropout3(tgt2)
        if not self.normalize_before:
            tgt = self.norm3(tgt)
        return tgt, self_attn, multihead_attention


class TransformerDecoder(nn.Module):
    """Transformer.py:657-763 (layers.N.*, norm.norm.*)."""

    def __init__(self, num_layers, nhead, d_ffn, d_model, kdim=None, vdim=None, dropout=0.0, activation=nn.ReLU,
                 normalize_before=False, causal=False, attention_type="regularMHA"):
        super().__init__()
        self.layers = nn.ModuleList([
            TransformerDecoderLayer(d_ffn=d_ffn, nhead=nhead, d_model=d_model, kdim=kdim, vdim=vdim, dropout=dropout,
                                    activation=activation, normalize_before=normalize_before, causal=causal,
                                    attention_type=attention_type) for _ in range(num_layers)])
        self.norm = LayerNorm(d_model, eps=1e-6)

    def forward(self, tgt, memory, tgt_mask=None, memory_mask=None, tgt_key_padding_mask=None,
                memory_key_padding_mask=None, pos_embs_tgt=None, pos_embs_src=None):
        output = tgt
        self_attns, multihead_attns = [], []
        for dec_layer in self.layers:
            output, self_attn, multihead_attn = dec_layer(
                output, memory, tgt_mask=tgt_mask, memory_mask=memory_mask, tgt_key_padding_mask=tgt_key_padding_mask,
                memory_key_padding_mask=memory_key_padding_mask, pos_embs_tgt=pos_embs_tgt, pos_embs_src=pos_embs_src)
            self_attns.append(self_attn)
            multihead_attns.append(multihead_attn)
        return self.norm(output), self_attns, multihead_attns


class _Embedding(nn.Module):
    """nnet/embedding.py:13-114 Embedding (one-hot off): nn.Embedding under
    `.Embedding`, indices cast to long."""

    def __init__(self, num_embeddings, embedding_dim=128, consider_as_one_hot=False, blank_id=0):
        super().__init__()
        if consider_as_one_hot:
            raise NotImplementedError("one-hot Embedding is not on the accelerated path")
        self.num_embeddings = num_embeddings
        self.embedding_dim = embedding_dim
        self.blank_id = blank_id
        self.Embedding = nn.Embedding(num_embeddings, embedding_dim)

    def forward(self, x):
        return self.Embedding(x.long())


class NormalizedEmbedding(nn.Module):
    """Transformer.py:766-797: emb(x) * sqrt(d_model)."""

    def __init__(self, d_model, vocab):
        super().__init__()
        self.emb = _Embedding(num_embeddings=vocab, embedding_dim=d_model, blank_id=0)
        self.d_model = d_model

    def forward(self, x):
        return self.emb(x) * math.sqrt(self.d_model)


def get_key_padding_mask(padded_input, pad_idx):
    """Transformer.py:800-830."""
    if len(padded_input.shape) == 4:
        bz, time, ch1, ch2 = padded_input.shape
        padded_input = padded_input.reshape(bz, time, ch1 * ch2)
    key_padded_mask = padded_input.eq(pad_idx).to(padded_input.device)
    if len(padded_input.shape) > 2:
        return key_padded_mask.float().prod(dim=-1).bool().detach()
    return key_padded_mask.detach()


def get_lookahead_mask(padded_input):
    """Transformer.py:833-858: (L, L) float mask, -inf above the diagonal."""
    seq_len = padded_input.shape[1]
    mask = (torch.triu(torch.ones((seq_len, seq_len), device=padded_input.device)) == 1).transpose(0, 1)
    mask = mask.float().masked_fill(mask == 0, float("-inf")).masked_fill(mask == 1, float(0.0))
    return mask.detach().to(padded_input.device)
