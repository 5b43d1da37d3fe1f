"""CPU restatement of the Fbank→CNN→Conformer encoder path (test infrastructure).

Functional restatement over a flat state dict whose keys are the
reference's own state_dict names, so a checkpoint of the reference (or of
speechbrain_amd) feeds it directly.  Restates:
  speechbrain/lobes/models/convolution.py:12-175 (ConvolutionFrontEnd/ConvBlock)
  speechbrain/nnet/CNN.py:556-722,1459-1481 (Conv2d "same" reflect padding)
  speechbrain/nnet/attention.py:312-359 (RelPosEncXL), :362-639 (RelPosMHAXL),
      :781-839 (PositionalwiseFeedForward)
  speechbrain/lobes/models/transformer/Conformer.py:24-383
  speechbrain/lobes/models/transformer/TransformerASR.py:279-316 (encode)
"""
import math

import torch
import torch.nn.functional as F


def _p(sd, k):
    return sd[k] if isinstance(sd[k], torch.Tensor) else torch.as_tensor(sd[k])


def conv_block(x, sd, prefix, stride=2, kernel=3, neg_slope=0.01, ln_eps=1e-5):
    """ConvBlock with one Conv2d(k, stride, "same"→reflect pad k//2) →
    LayerNorm over (freq, channels) → LeakyReLU (convolution.py:112-175,
    CNN.py:616-700).  x: (B, T, F) or (B, T, F, C) → (B, T', F', C')."""
    w = _p(sd, prefix + "conv_0.conv.weight")
    b = _p(sd, prefix + "conv_0.conv.bias")
    if x.dim() == 3:
        x = x.unsqueeze(-1)
    h = x.permute(0, 3, 2, 1)  # (B, C, F, T): spatial = (freq, time)
    p = kernel // 2
    h = F.pad(h, (p, p, p, p), mode="reflect")
    h = F.conv2d(h, w, b, stride=stride)
    h = h.permute(0, 3, 2, 1)  # (B, T', F', C')
    g = _p(sd, prefix + "norm_0.norm.weight")
    be = _p(sd, prefix + "norm_0.norm.bias")
    h = F.layer_norm(h, tuple(g.shape), g, be, ln_eps)
    return F.leaky_relu(h, neg_slope)


def conv_frontend(x, sd, prefix="", num_blocks=2):
    """ConvolutionFrontEnd of conformer_small.yaml:123-130."""
    for i in range(num_blocks):
        x = conv_block(x, sd, f"{prefix}convblock_{i}.convs.")
    return x


def rel_pos_enc_xl(T, d, dtype=torch.float32):
    """attention.py:327-359: (1, 2T-1, d); row r holds position |T-1-r| as
    [sin, cos] interleaved (past half flipped; future sin not negated)."""
    inv_freq = torch.exp(torch.arange(0, d, 2, dtype=torch.float32) * -(math.log(10000.0) / d))
    pos = torch.arange(0, T, dtype=dtype).unsqueeze(-1)
    s = torch.sin(pos * inv_freq)
    c = torch.cos(pos * inv_freq)
    pe = torch.zeros(T, d, dtype=dtype)
    pe[:, 0::2] = s
    pe[:, 1::2] = c
    return torch.cat([torch.flip(pe, (0,)), pe[1:]], dim=0).unsqueeze(0)


def rel_shift(bd):
    """attention.py:468-483 in closed form: out[..., i, j] = bd[..., i, T-1-i+j],
    j < T (= pos_len//2 + 1)."""
    T = bd.shape[-2]
    i = torch.arange(T).view(-1, 1)
    j = torch.arange(T).view(1, -1)
    idx = (T - 1 - i + j).expand(*bd.shape[:-2], T, T)
    return torch.gather(bd, -1, idx)


def rel_pos_mha(x, pos_embs, sd, prefix, num_heads, key_padding_mask=None,
                attn_mask=None):
    """attention.py:485-639 (self-attention: query is key is value).
    Returns (out (B,T,d), attn (B,H,T,T))."""
    B, T, d = x.shape
    dh = d // num_heads
    w_in = _p(sd, prefix + "in_proj_weight")
    qkv = F.linear(x, w_in).view(B, T, num_heads, 3 * dh)
    q, k, v = qkv.chunk(3, dim=-1)
    p_k = F.linear(pos_embs, _p(sd, prefix + "linear_pos.weight")).view(1, -1, num_heads, dh)
    u = _p(sd, prefix + "pos_bias_u").reshape(1, 1, num_heads, dh)  # (dh,H) memory read as (H,dh)
    vb = _p(sd, prefix + "pos_bias_v").reshape(1, 1, num_heads, dh)
    ac = torch.matmul((q + u).transpose(1, 2), k.permute(0, 2, 3, 1))
    bd = torch.matmul((q + vb).transpose(1, 2), p_k.permute(0, 2, 3, 1))
    bd = rel_shift(bd)
    score = (ac + bd) * (1.0 / math.sqrt(d))
    if attn_mask is not None:
        am = attn_mask.view(1, 1, T, T) if attn_mask.ndim == 2 else attn_mask.view(-1, num_heads, T, T)
        score = score.masked_fill(am, -float("inf")) if am.dtype == torch.bool else score + am
    if key_padding_mask is not None:
        score = score.masked_fill(key_padding_mask.view(B, 1, 1, T), -float("inf"))
    attn = F.softmax(score, dim=-1)
    o = torch.matmul(attn, v.transpose(1, 2)).transpose(1, 2).reshape(B, T, d)
    out = F.linear(o, _p(sd, prefix + "out_proj.weight"), _p(sd, prefix + "out_proj.bias"))
    return out, attn


def rel_shift_cross(bd, mask_pos_future=False):
    """attention.py:468-483 for any (q_len, P) band, in closed form.  The pad /
    view / drop-row trick maps output element (i, j) to flat position
    p = i*P + j + q_len of the left-padded (q_len, P+1) band: row r = p // (P+1),
    column c = p % (P+1); c == 0 is the pad (0), else bd[r, c-1].  For
    q_len == k_len, r == i always; for q_len > k_len some elements read the
    next row(s), as the reference's view does.  mask_pos_future multiplies by
    tril(ones, P - q_len) before the slice to j < P//2 + 1."""
    Lq, P = bd.shape[-2], bd.shape[-1]
    Lk = P // 2 + 1
    i = torch.arange(Lq).view(-1, 1)
    j = torch.arange(Lk).view(1, -1)
    p = i * P + j + Lq
    r, c = p // (P + 1), p % (P + 1)
    padded = F.pad(bd, (1, 0))  # (..., Lq, P+1)
    out = padded[..., r, c]
    if mask_pos_future:
        out = out * ((j - i) <= (P - Lq)).to(out.dtype)
    return out


def rel_pos_mha_cross(query, key, value, pos_embs, sd, prefix, num_heads, vbias=False, mask_pos_future=False,
                      key_padding_mask=None, attn_mask=None):
    """attention.py:485-639 with query != key/value (the separate q/k/v
    projections of :554-564) and q_len != k_len.  Returns (out (B, Lq, E),
    attn (B, H, Lq, Lk))."""
    B, Lq, E = query.shape
    Lk = key.shape[1]
    dh = E // num_heads
    wq, wk, wv = _p(sd, prefix + "in_proj_weight").chunk(3, dim=0)
    q = F.linear(query, wq).view(B, Lq, num_heads, dh)
    k = F.linear(key, wk).view(B, Lk, num_heads, dh)
    v = F.linear(value, wv).view(B, Lk, num_heads, dh)
    if vbias:
        v = v + _p(sd, prefix + "value_bias_weight").view(1, 1, num_heads, dh)
    p_k = F.linear(pos_embs, _p(sd, prefix + "linear_pos.weight")).view(1, -1, num_heads, dh)
    u = _p(sd, prefix + "pos_bias_u").reshape(1, 1, num_heads, dh)
    vb = _p(sd, prefix + "pos_bias_v").reshape(1, 1, num_heads, dh)
    ac = torch.matmul((q + u).transpose(1, 2), k.permute(0, 2, 3, 1))
    bd = rel_shift_cross(torch.matmul((q + vb).transpose(1, 2), p_k.permute(0, 2, 3, 1)), mask_pos_future)
    score = (ac + bd) * (1.0 / math.sqrt(E))
    if attn_mask is not None:
        am = attn_mask.view(1, 1, Lq, Lk) if attn_mask.ndim == 2 else attn_mask.view(-1, num_heads, Lq, Lk)
        score = score.masked_fill(am, -float("inf")) if am.dtype == torch.bool else score + am
    if key_padding_mask is not None:
        score = score.masked_fill(key_padding_mask.view(B, 1, 1, Lk), -float("inf"))
    attn = F.softmax(score, dim=-1)
    o = torch.matmul(attn, v.transpose(1, 2)).transpose(1, 2).reshape(B, Lq, E)
    out = F.linear(o, _p(sd, prefix + "out_proj.weight"), _p(sd, prefix + "out_proj.bias"))
    return out, attn


def swish(x):
    return x * torch.sigmoid(x)  # activations.py:111-142 (beta=1)


def ffn_module(x, sd, prefix):
    """nn.Sequential(LayerNorm, PositionalwiseFeedForward(Swish), Dropout)
    (Conformer.py:194-214, attention.py:823-839)."""
    d = x.shape[-1]
    h = F.layer_norm(x, (d,), _p(sd, prefix + "0.weight"), _p(sd, prefix + "0.bias"), 1e-5)
    h = F.linear(h, _p(sd, prefix + "1.ffn.0.weight"), _p(sd, prefix + "1.ffn.0.bias"))
    h = swish(h)
    return F.linear(h, _p(sd, prefix + "1.ffn.3.weight"), _p(sd, prefix + "1.ffn.3.bias"))


def conv_module(x, sd, prefix, kernel_size=31, causal=False, pad_mask=None):
    """Conformer.py:101-115: LN → 1x1 conv d→2d → GLU → depthwise conv k
    (zero pad) → LN → Swish → Linear → masked_fill(pad, 0)."""
    B, T, d = x.shape
    h = F.layer_norm(x, (d,), _p(sd, prefix + "layer_norm.weight"), _p(sd, prefix + "layer_norm.bias"), 1e-5)
    h = h.transpose(1, 2)
    h = F.conv1d(h, _p(sd, prefix + "bottleneck.0.weight"), _p(sd, prefix + "bottleneck.0.bias"))
    h = F.glu(h, dim=1)
    pad = (kernel_size - 1) if causal else (kernel_size - 1) // 2
    h = F.conv1d(h, _p(sd, prefix + "conv.weight"), _p(sd, prefix + "conv.bias"), padding=pad, groups=d)
    if causal:
        h = h[..., :-pad]
    h = h.transpose(1, 2)
    h = F.layer_norm(h, (d,), _p(sd, prefix + "after_conv.0.weight"), _p(sd, prefix + "after_conv.0.bias"), 1e-5)
    h = swish(h)
    h = F.linear(h, _p(sd, prefix + "after_conv.2.weight"), _p(sd, prefix + "after_conv.2.bias"))
    if pad_mask is not None:
        h = h.masked_fill(pad_mask, 0.0)
    return h


def conformer_layer(x, pos_embs, sd, prefix, num_heads, kernel_size=31,
                    causal=False, key_padding_mask=None, attn_mask=None):
    """Conformer.py:220-260."""
    d = x.shape[-1]
    conv_mask = key_padding_mask.unsqueeze(-1) if key_padding_mask is not None else None
    x = x + 0.5 * ffn_module(x, sd, prefix + "ffn_module1.")
    skip = x
    h = F.layer_norm(x, (d,), _p(sd, prefix + "norm1.norm.weight"), _p(sd, prefix + "norm1.norm.bias"), 1e-5)
    h, attn = rel_pos_mha(h, pos_embs, sd, prefix + "mha_layer.", num_heads, key_padding_mask, attn_mask)
    x = h + skip
    x = x + conv_module(x, sd, prefix + "convolution_module.", kernel_size, causal, conv_mask)
    x = x + 0.5 * ffn_module(x, sd, prefix + "ffn_module2.")
    x = F.layer_norm(x, (d,), _p(sd, prefix + "norm2.norm.weight"), _p(sd, prefix + "norm2.norm.bias"), 1e-5)
    return x, attn


def conformer_encoder(src, pos_embs, sd, prefix, num_layers, num_heads,
                      kernel_size=31, causal=False, key_padding_mask=None,
                      attn_mask=None):
    """Conformer.py:343-383: layers then final LayerNorm(eps=1e-6)."""
    if pos_embs is None:
        raise ValueError("pos_embs are mandatory for RelPosMHAXL")
    x = src
    attns = []
    for i in range(num_layers):
        x, a = conformer_layer(x, pos_embs, sd, f"{prefix}layers.{i}.", num_heads,
                               kernel_size, causal, key_padding_mask, attn_mask)
        attns.append(a)
    d = x.shape[-1]
    x = F.layer_norm(x, (d,), _p(sd, prefix + "norm.norm.weight"), _p(sd, prefix + "norm.norm.bias"), 1e-6)
    return x, attns


def transformer_asr_encode(src, sd, prefix, num_layers, num_heads,
                           wav_len=None, kernel_size=31, causal=False):
    """TransformerASR.py:279-316: 4-D→3-D, key padding mask
    arange(T) > floor(wav_len·T), Linear(in→d), RelPosEncXL, encoder."""
    if src.dim() == 4:
        b, t, c1, c2 = src.shape
        src = src.reshape(b, t, c1 * c2)
    kpm = None
    if wav_len is not None:
        abs_len = torch.floor(wav_len * src.shape[1])
        kpm = torch.arange(src.shape[1])[None, :].to(abs_len) > abs_len[:, None]
    h = F.linear(src, _p(sd, prefix + "custom_src_module.layers.0.w.weight"),
                 _p(sd, prefix + "custom_src_module.layers.0.w.bias"))
    pe = rel_pos_enc_xl(h.shape[1], h.shape[2], h.dtype)
    out, _ = conformer_encoder(h, pe, sd, prefix + "encoder.", num_layers, num_heads,
                               kernel_size, causal, kpm)
    return out


def fbank_to_encoder(wav, sd_cnn, sd_tr, num_layers, num_heads, n_mels=80,
                     wav_len=None, kernel_size=31):
    """The metric path (BASELINE.json): Fbank → ConvolutionFrontEnd →
    TransformerASR.encode."""
    from oracle.features import fbank
    feats = fbank(wav, n_mels=n_mels)
    c = conv_frontend(feats, sd_cnn)
    return transformer_asr_encode(c, sd_tr, "", num_layers, num_heads, wav_len, kernel_size)
