"""Drop-in for speechbrain.lobes.models.wav2vec (W2VLatentExtractor :28-106,
EncoderWrapper :153-227) — config 5's front-end — on HIP kernels.

W2VLatentExtractor (defaults: 7 blocks, 512 channels, kernels
[11, 3, 3, 3, 3, 3, 3], strides [5, 2, 2, 2, 2, 2, 2], no conv bias,
padding "valid", LayerNorm over channels, GELU; B x 15 s → 748 frames):
  F.layer_norm(wav)         sbk_w2v_wav_stats (applied on load by layer 0)
  layer 0 (Cin = 1)         sbk_w2v_conv0: conv + LayerNorm + GELU in one
                            kernel, written straight in the next GEMM's
                            operand format (MXFP8 / bf16 / fp32)
  layers 1..6               the conv as ONE GEMM over overlapping rows
                            (K = k*C, lda = stride*C; sbk_mx_gemm under
                            mxfp8(), sbk_gemm per utterance otherwise), then
                            sbk_ln_act (LayerNorm + GELU → next operand)
  closing nn.LayerNorm      sbk_ln_act
State-dict keys match the reference (extractor.convblock_i.convs.conv_0.conv.
weight, .norm_0.norm.{weight,bias}, norm.{weight,bias}).
"""
import torch
import torch.nn as nn

from ... import _enc
from ... import _autograd as A
from ...nnet.normalization import LayerNorm
from .transformer.Transformer import PositionalEncoding, TransformerEncoder, _mode

__all__ = ["W2VLatentExtractor", "EncoderWrapper"]

_f32, _bf16 = torch.float32, torch.bfloat16


class _Named(nn.Module):
    def add(self, name, module):
        self.add_module(name, module)
        return module


class Conv1d(nn.Module):
    """Parameter carrier with the key layout of speechbrain.nnet.CNN.Conv1d
    (CNN.py:309-516: `conv` = nn.Conv1d, kaiming init when asked).  Runs
    inside W2VLatentExtractor's fused kernels."""

    def __init__(self, out_channels, kernel_size, in_channels, stride=1, bias=True, padding="valid",
                 conv_init=None):
        super().__init__()
        if padding != "valid":
            raise NotImplementedError("only padding='valid' (the wav2vec2 extractor) is on the HIP path")
        self.conv = nn.Conv1d(in_channels, out_channels, kernel_size, stride=stride, padding=0, bias=bias)
        if conv_init == "kaiming":
            nn.init.kaiming_normal_(self.conv.weight)
        elif conv_init == "zero":
            nn.init.zeros_(self.conv.weight)
        elif conv_init == "normal":
            nn.init.normal_(self.conv.weight, std=1e-6)


class W2VLatentExtractor(nn.Module):
    def __init__(self, out_channels=[512, 512, 512, 512, 512, 512, 512], kernel_sizes=[11, 3, 3, 3, 3, 3, 3],
                 strides=[5, 2, 2, 2, 2, 2, 2], dropout=0.0, conv_init="kaiming"):
        super().__init__()
        assert len(out_channels) == len(kernel_sizes) == len(strides)
        self.kernel_sizes = kernel_sizes
        self.strides = strides
        self.out_dim = out_channels[-1]
        self.extractor = _Named()
        cin = 1
        for i, (c, k, s) in enumerate(zip(out_channels, kernel_sizes, strides)):
            blk = self.extractor.add(f"convblock_{i}", _Named())
            convs = blk.add("convs", _Named())
            convs.add("conv_0", Conv1d(c, k, cin, stride=s, bias=False, conv_init=conv_init))
            convs.add("norm_0", LayerNorm(input_shape=(None, None, c)))
            convs.add("act_0", nn.GELU())
            convs.add("dropout_0", nn.Dropout(dropout))
            cin = c
        self.norm = nn.LayerNorm(out_channels[-1])
        self._wc = _enc.WeightCache()

    def _block(self, i):
        c = getattr(self.extractor, f"convblock_{i}").convs
        return c.conv_0.conv, c.norm_0.norm

    def _wmat(self, i, mode):
        """Layer-i weight as a GEMM operand: (Cout, k*Cin) with K ordered
        [tap][in] to match the overlapping channels-last input rows."""
        conv, _ = self._block(i)

        def make():
            w = conv.weight.detach().permute(0, 2, 1).reshape(conv.out_channels, -1).float().contiguous()
            if mode == "mx":
                from ... import _w2v
                return _w2v.mx_quant(w)
            return _enc.cast_bf16(w) if mode == _bf16 else w
        return self._wc.get(("w", i, str(mode)), [conv.weight], make)

    def _layer_mode(self, mode, i):
        """MXFP8 for a conv layer needs K = k*Cin and Cout multiples of 128."""
        conv, _ = self._block(i)
        if mode == "mx" and ((conv.in_channels * conv.kernel_size[0]) % 128 or conv.out_channels % 128
                             or conv.in_channels % 32):
            return _bf16
        return mode

    def run(self, wav, normalize_signal=True, out_dtype=_f32):
        """(B, S) fp32 → (B*T', C) after the closing LayerNorm (out_dtype
        fp32 / bf16 / "mx"), and T'."""
        from ... import _w2v
        if self.training and any(isinstance(m, nn.Dropout) and m.p > 0 for m in self.modules()):
            raise NotImplementedError("W2VLatentExtractor has no training path yet (inference only)")
        mode = _mode()
        B, S = wav.shape
        wav = wav.float().contiguous()
        stats = _w2v.wav_stats(wav, 1e-5) if normalize_signal else None
        n = len(self.kernel_sizes)
        conv, ln = self._block(0)
        if conv.in_channels != 1:
            raise ValueError("the first extractor layer takes the 1-channel waveform")
        # each layer's output goes straight out in the NEXT layer's operand format
        nxt = [self._layer_mode(mode, i + 1) for i in range(n - 1)] + [_f32]
        first = nxt[0]
        x = _w2v.conv0(wav, stats, conv.weight.detach().reshape(conv.out_channels, -1), ln.weight.detach(),
                       ln.bias.detach(), ln.eps, self.strides[0], "mx" if first == "mx" else first)
        T = (S - self.kernel_sizes[0]) // self.strides[0] + 1
        for i in range(1, n):
            conv, ln = self._block(i)
            lm = self._layer_mode(mode, i)
            k, s, C = self.kernel_sizes[i], self.strides[i], conv.in_channels
            if lm == "mx":
                y, T_out = _w2v.mx_conv_gemm(x, B, T, C, k, s, self._wmat(i, "mx"), out=_f32)
            else:
                T_out = (T - k) // s + 1
                w = self._wmat(i, lm)
                y = torch.empty(B * T_out, conv.out_channels, device=wav.device, dtype=_f32)
                for b in range(B):  # one GEMM per utterance over its overlapping input rows
                    a = torch.as_strided(x, (T_out, k * C), (s * C, 1), x.storage_offset() + b * T * C)
                    y[b * T_out:(b + 1) * T_out] = _enc.gemm(a, w, out_dtype=_f32)
            T = T_out
            nm = nxt[i] if i + 1 < n else _f32
            x = _w2v.ln_act(y, (ln.weight.detach(), ln.bias.detach(), ln.eps), "gelu", "mx" if nm == "mx" else nm)
        x = _w2v.ln_act(x, (self.norm.weight.detach(), self.norm.bias.detach(), self.norm.eps), None,
                        "mx" if out_dtype == "mx" else out_dtype)
        return x, T

    def module_forward(self, x, normalize_signal=True):
        """wav2vec.py:88-95 layer by layer, differentiable (training, conv
        dropout, gradients): F.layer_norm of the waveform (HIP LayerNorm with
        unit affine), then per block the valid strided Conv1d as a (k x 1)
        Conv2d on sbk_im2col_x + the MFMA GEMM, LayerNorm over channels,
        GELU and dropout (HIP kernels with backward), the closing LayerNorm."""
        B, S = x.shape
        dtype = _enc.compute_dtype()
        x = x.float().contiguous()
        if normalize_signal:
            ones = torch.ones(S, device=x.device)
            x = A.LayerNormFn.apply(x, ones, torch.zeros_like(ones), 1e-5, _f32)
        h = x.view(B, S, 1, 1)  # (B, T, F = 1, C) for the 2-D im2col
        T = S
        for i in range(len(self.kernel_sizes)):
            conv, ln = self._block(i)
            drop = getattr(self.extractor, f"convblock_{i}").convs.dropout_0
            k, s = self.kernel_sizes[i], self.strides[i]
            To = (T - k) // s + 1
            hin = h if h.dtype == dtype else A.to_dtype(h, dtype)
            y = A.Conv2dXFn.apply(hin, conv.weight.unsqueeze(2), None, dtype, _f32,
                                  (k, 1, s, 1, 1, 1, 0, 0, To, 1, 1))  # (B, To, 1, Cout)
            C = y.shape[-1]
            y = A.layer_norm(y.reshape(B * To, C), ln)
            y = A.act(y, "gelu")
            y = A.dropout(y, drop.p, self.training)
            h, T = y.view(B, To, 1, C), To
        return A.layer_norm(h.reshape(B * T, -1), self.norm).view(B, T, -1)

    def forward(self, x, normalize_signal=True):
        """(B, S) waveform → (B, T', C) latents (fp32)."""
        if A.needs_grad(self, x) or (self.training and any(isinstance(m, nn.Dropout) and m.p > 0
                                                           for m in self.modules())):
            return self.module_forward(x, normalize_signal)
        B = x.shape[0]
        y, T = self.run(x, normalize_signal, _f32)
        return y.view(B, T, -1)

    def get_output_lengths(self, input_lengths: torch.LongTensor):
        """wav2vec.py:97-106."""
        def _conv_out_length(input_length, kernel_size, stride):
            return torch.floor((input_length - kernel_size) / stride + 1)

        for kernel_size, stride in zip(self.kernel_sizes, self.strides):
            input_lengths = _conv_out_length(input_lengths, kernel_size, stride)
        return input_lengths.to(torch.long)


class EncoderWrapper(nn.Module):
    """wav2vec.py:153-227: input projector Linear → (+ mask_emb on masked
    frames) → + positional encoding → latent encoder with the padding mask of
    round(wav_lens·T)."""

    def __init__(self, in_dim, embedding_dim, latent_encoder, positional_encoding=PositionalEncoding,
                 dropout_encoder_input=0.05):
        super().__init__()
        self.input_projector = nn.Linear(in_dim, embedding_dim)
        self.latent_encoder = latent_encoder
        self.positional_encoding = positional_encoding(embedding_dim)
        self.dropout_encoder_input = nn.Dropout(dropout_encoder_input)
        self.mask_emb = nn.Parameter(torch.FloatTensor(embedding_dim).uniform_(), requires_grad=True)
        self._wc = _enc.WeightCache()

    def _proj_weight(self, mode):
        w = self.input_projector.weight
        from ...nnet.attention import _mode_weight
        return self._wc.get(("proj", str(mode)), [w], lambda: _mode_weight(w.detach().contiguous(), mode))

    def embed(self, latents2d, B, T, wav_lens=None, padding_mask=None, need_weights=False):
        """latents2d (B*T, in_dim) fp32 / bf16 / MX → (B*T, d) fp32 embeddings."""
        from ... import _w2v
        if self.training and self.dropout_encoder_input.p > 0:
            raise NotImplementedError("EncoderWrapper has no training path yet (inference only)")
        if not isinstance(self.latent_encoder, TransformerEncoder):
            raise NotImplementedError("EncoderWrapper: the HIP path wraps a TransformerEncoder")
        mode = _mode()
        pm = mode if not (mode == "mx" and (self.input_projector.in_features % 128
                                            or self.input_projector.out_features % 128)) else _bf16
        bias = self.input_projector.bias.detach().float()
        if pm == "mx":
            a = latents2d if hasattr(latents2d, "q") else _w2v.ln_act(latents2d, None, None, "mx")
            h = _w2v.mx_gemm(a, self._proj_weight("mx"), bias=bias, out=_f32)
        else:
            a = _enc.to_compute(latents2d, pm) if not hasattr(latents2d, "q") else None
            if a is None:
                raise TypeError("MXFP8 latents need the MXFP8 projector")
            h = _enc.gemm(a, self._proj_weight(pm), bias=bias, out_dtype=_f32)
        d = h.shape[1]
        pe = self.positional_encoding.pe[0, :T].float().contiguous()
        _w2v.add_posenc(h, pe, T)
        kpm = None
        if wav_lens is not None:
            n = torch.round(wav_lens.to(h.device).float() * T)
            kpm = (torch.arange(T, device=h.device)[None, :] >= n[:, None]).to(torch.uint8).contiguous()
        elif padding_mask is not None:
            kpm = padding_mask.to(torch.uint8).contiguous()
        y, _ = self.latent_encoder.run(h, B, T, kpm, need_weights)
        return y

    def module_forward(self, latents, wav_lens=None, padding_mask=None, mask=None):
        """wav2vec.py:199-227 step by step (training, gradients, masked
        pre-training): projector on the MFMA GEMM, HIP dropout, mask_emb on
        the masked frames, the positional table, the latent encoder's module
        path with the key padding of round(wav_lens·T)."""
        results = {}
        B, T, C = latents.shape
        dtype = _enc.compute_dtype()
        lin = self.input_projector
        h = A.linear(latents.reshape(B * T, C), lin.weight, lin.bias, dtype, self._wc, "t_proj")
        h = A.dropout(h, self.dropout_encoder_input.p, self.training).view(B, T, -1)
        if mask is not None:
            h = h.clone()
            h[mask] = self.mask_emb.to(h.dtype)
            num_masked = mask.sum()
            results["num_masked"] = num_masked
            results["ratio_masked"] = num_masked / mask.numel()
        if wav_lens is not None:
            n = torch.round(wav_lens.to(h.device).float() * T)
            padding_mask = torch.arange(T, device=h.device)[None, :] >= n[:, None]
        h = h + self.positional_encoding(h)
        feats, _ = self.latent_encoder(h, src_key_padding_mask=padding_mask)
        results["embeddings"] = feats
        return results

    def forward(self, latents, wav_lens=None, padding_mask=None, mask=None):
        if (mask is not None or A.needs_grad(self, latents)
                or not isinstance(self.latent_encoder, TransformerEncoder)
                or not all(layer._fused_ok(latents, None, None, padding_mask) for layer in self.latent_encoder.layers)
                or (self.training and (self.dropout_encoder_input.p > 0
                                       or any(isinstance(m, nn.Dropout) and m.p > 0
                                              for m in self.latent_encoder.modules())))):
            return self.module_forward(latents, wav_lens, padding_mask, mask)
        B, T, C = latents.shape
        y = self.embed(latents.float().reshape(B * T, C).contiguous(), B, T, wav_lens, padding_mask)
        return {"embeddings": y.view(B, T, -1)}
