"""CPU restatement of the config-5 path (test infrastructure only: the product
never imports this module).  Functional, over flat state dicts keyed by the
reference's own state_dict names.  Restates:
  speechbrain/lobes/models/wav2vec.py:28-106 (W2VLatentExtractor: waveform
      layer_norm, 7 x [Conv1d valid, no bias → LayerNorm(C) → GELU], LayerNorm)
      and :153-227 (EncoderWrapper: Linear, positional encoding, padding mask
      from round(wav_lens·T))
  speechbrain/lobes/models/convolution.py:12-175 (ConvBlock ordering)
  speechbrain/nnet/CNN.py:309-516 (Conv1d, padding "valid")
  speechbrain/lobes/models/transformer/Transformer.py:201-243
      (PositionalEncoding), :246-486 (TransformerEncoderLayer / Encoder,
      pre- and post-norm, LayerNorm eps 1e-6)
  speechbrain/nnet/attention.py:642-778 (MultiheadAttention → torch
      nn.MultiheadAttention: in_proj, 1/sqrt(dh) scaling, key padding mask,
      head-averaged weights), :781-839 (PositionalwiseFeedForward)
Pinned to tests/golden/wav2vec.npz (generated from the reference by
tests/golden/gen_golden.py gen_wav2vec).
"""
import math

import torch
import torch.nn.functional as F


def _p(sd, k):
    return sd[k] if isinstance(sd[k], torch.Tensor) else torch.as_tensor(sd[k])


# Operand-rounding emulation (used only to DERIVE the tolerance of the
# reduced-precision GPU paths, never as a result): `_QMM(t)` rounds a GEMM
# operand along its last (contraction) axis, `_QACT(t)` an activation that the
# GPU path keeps in bf16 between kernels.  Both are the identity by default.
_QMM = None
_QACT = None


def set_rounding(mm=None, act=None):
    global _QMM, _QACT
    _QMM, _QACT = mm, act


def _qm(t):
    return _QMM(t) if _QMM is not None else t


def _qa(t):
    return _QACT(t) if _QACT is not None else t


def _linear(x, w, b=None):
    return F.linear(_qm(x), _qm(w), b)


def mx_round(t):
    """MXFP8 rounding of t along its last axis (blocks of 32, power-of-two
    scale 2^ceil(log2(amax/448)), e4m3 RNE) — the format of csrc/mx.h."""
    sh = t.shape
    x = t.float().reshape(-1, sh[-1] // 32, 32)
    am = x.abs().amax(-1, keepdim=True)
    e = torch.where(am > 0, torch.ceil(torch.log2(am / 448.0)), torch.full_like(am, -127.0)).clamp(-127, 127)
    sc = torch.exp2(e)
    q = (x / sc).clamp(-448, 448).to(torch.float8_e4m3fn).float() * sc
    return q.reshape(sh)


def bf16_round(t):
    return t.to(torch.bfloat16).float()


def latent_extractor(wav, sd, prefix="", kernels=(11, 3, 3, 3, 3, 3, 3), strides=(5, 2, 2, 2, 2, 2, 2),
                     normalize_signal=True, ln_eps=1e-5):
    """wav2vec.py:89-95.  wav (B, S) → latents (B, T', C)."""
    x = wav
    if normalize_signal:
        x = F.layer_norm(x, x.shape[1:])
    x = x.unsqueeze(2)  # (B, S, 1)
    for i, (k, s) in enumerate(zip(kernels, strides)):
        pre = f"{prefix}extractor.convblock_{i}.convs."
        w = _p(sd, pre + "conv_0.conv.weight")
        if i == 0 or _QMM is None:
            h = F.conv1d(x.transpose(1, 2), w, None, stride=s).transpose(1, 2)  # (B, T', C)
        else:  # rounding blocks run along the input channels of each tap (the GPU's [tap][in] K order)
            xq = _qm(x).transpose(1, 2)
            wq = _qm(w.permute(0, 2, 1)).permute(0, 2, 1)
            h = F.conv1d(xq, wq, None, stride=s).transpose(1, 2)
        h = F.layer_norm(h, (h.shape[-1],), _p(sd, pre + "norm_0.norm.weight"), _p(sd, pre + "norm_0.norm.bias"),
                         ln_eps)
        x = F.gelu(h)
    return F.layer_norm(x, (x.shape[-1],), _p(sd, prefix + "norm.weight"), _p(sd, prefix + "norm.bias"), 1e-5)


def output_lengths(lengths, kernels=(11, 3, 3, 3, 3, 3, 3), strides=(5, 2, 2, 2, 2, 2, 2)):
    """wav2vec.py:97-106."""
    x = torch.as_tensor(lengths, dtype=torch.float64)
    for k, s in zip(kernels, strides):
        x = torch.floor((x - k) / s + 1)
    return x.to(torch.long)


def positional_encoding(T, d, max_len=2500):
    """Transformer.py:221-243: sinusoidal table, sin on even, cos on odd
    columns (fp32 arithmetic as the reference)."""
    pe = torch.zeros(max_len, d)
    positions = torch.arange(0, max_len).unsqueeze(1).float()
    den = torch.exp(torch.arange(0, d, 2).float() * -(math.log(10000.0) / d))
    pe[:, 0::2] = torch.sin(positions * den)
    pe[:, 1::2] = torch.cos(positions * den)
    return pe[:T].unsqueeze(0)


def mha(q, k, v, sd, prefix, nhead, key_padding_mask=None):
    """nn.MultiheadAttention forward as MultiheadAttention wraps it
    (attention.py:748-778): (B, L, E) inputs; returns (out (B, L, E),
    head-averaged weights (B, L, S))."""
    B, L, E = q.shape
    S = k.shape[1]
    dh = E // nhead
    w = _p(sd, prefix + "att.in_proj_weight")
    b = _p(sd, prefix + "att.in_proj_bias")
    qp = _qa(_linear(q, w[:E], b[:E]))
    kp = _qa(_linear(k, w[E:2 * E], b[E:2 * E]))
    vp = _qa(_linear(v, w[2 * E:], b[2 * E:]))
    qh = qp.view(B, L, nhead, dh).transpose(1, 2)
    kh = kp.view(B, S, nhead, dh).transpose(1, 2)
    vh = vp.view(B, S, nhead, dh).transpose(1, 2)
    s = (qh * (1.0 / math.sqrt(dh))) @ kh.transpose(-1, -2)  # (B, H, L, S)
    if key_padding_mask is not None:
        s = s.masked_fill(key_padding_mask[:, None, None, :].bool(), float("-inf"))
    p = torch.softmax(s, dim=-1)
    o = _qa((_qa(p) @ vh).transpose(1, 2).reshape(B, L, E))
    o = _linear(o, _p(sd, prefix + "att.out_proj.weight"), _p(sd, prefix + "att.out_proj.bias"))
    return o, p.mean(dim=1)


def _ln(x, sd, key, eps):
    return F.layer_norm(x, (x.shape[-1],), _p(sd, key + ".weight"), _p(sd, key + ".bias"), eps)


def encoder_layer(x, sd, prefix, nhead, act=F.relu, normalize_before=False, key_padding_mask=None):
    """Transformer.py:321-376."""
    src1 = _ln(x, sd, prefix + "norm1.norm", 1e-6) if normalize_before else x
    out, attn = mha(src1, src1, src1, sd, prefix + "self_att.", nhead, key_padding_mask)
    x = x + out
    if not normalize_before:
        x = _ln(x, sd, prefix + "norm1.norm", 1e-6)
    src1 = _ln(x, sd, prefix + "norm2.norm", 1e-6) if normalize_before else x
    h = act(_linear(src1, _p(sd, prefix + "pos_ffn.ffn.0.weight"), _p(sd, prefix + "pos_ffn.ffn.0.bias")))
    out = _linear(h, _p(sd, prefix + "pos_ffn.ffn.3.weight"), _p(sd, prefix + "pos_ffn.ffn.3.bias"))
    x = x + out
    if not normalize_before:
        x = _ln(x, sd, prefix + "norm2.norm", 1e-6)
    return x, attn


def transformer_encoder(x, sd, prefix, num_layers, nhead, act=F.relu, normalize_before=False,
                        key_padding_mask=None):
    """Transformer.py:452-486 (eval: no layerdrop)."""
    attns = []
    for i in range(num_layers):
        x, a = encoder_layer(x, sd, f"{prefix}layers.{i}.", nhead, act, normalize_before, key_padding_mask)
        attns.append(a)
    return _ln(x, sd, prefix + "norm.norm", 1e-6), attns


def encoder_wrapper(latents, sd, prefix, num_layers, nhead, act=F.gelu, normalize_before=True, wav_lens=None):
    """wav2vec.py:193-227 (eval, no mask): Linear → + positional encoding →
    TransformerEncoder with the padding mask of round(wav_lens·T)."""
    T = latents.shape[1]
    h = _linear(latents, _p(sd, prefix + "input_projector.weight"), _p(sd, prefix + "input_projector.bias"))
    kpm = None
    if wav_lens is not None:
        n = torch.round(torch.as_tensor(wav_lens) * T)
        kpm = ~(torch.arange(T)[None, :] < n[:, None])
    h = h + positional_encoding(T, h.shape[-1])
    y, _ = transformer_encoder(h, sd, prefix + "latent_encoder.", num_layers, nhead, act, normalize_before, kpm)
    return y


def wav2vec_encode(wav, sd_ext, sd_wrap, num_layers, nhead, wav_lens=None, kernels=(11, 3, 3, 3, 3, 3, 3),
                   strides=(5, 2, 2, 2, 2, 2, 2)):
    """Config 5: W2VLatentExtractor → EncoderWrapper(TransformerEncoder,
    pre-norm, GELU)."""
    lat = latent_extractor(wav, sd_ext, "", kernels, strides)
    return encoder_wrapper(lat, sd_wrap, "", num_layers, nhead, F.gelu, True, wav_lens)
