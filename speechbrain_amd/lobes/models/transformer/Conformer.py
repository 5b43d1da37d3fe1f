"""Drop-in for speechbrain.lobes.models.transformer.Conformer encoder side
(ConvolutionModule, ConformerEncoderLayer, ConformerEncoder;
speechbrain/lobes/models/transformer/Conformer.py:24-383).

Same constructor arguments and submodule tree (so state_dict keys match the
reference); forward runs a fused kernel schedule per layer:

  LN                      → u        (bf16 | f32)
  GEMM+bias+Swish         → h        FFN1 up
  GEMM+bias, x += 0.5·val → x        FFN1 down (residual fused)
  LN(norm1)               → u
  GEMM in_proj            → qkv      ; GEMM linear_pos → p_k
  rel-pos attention       → o        (scores, rel_shift, mask, softmax, P·V)
  GEMM out_proj, x += val → x
  LN(conv.layer_norm)     → u
  GEMM pointwise + GLU    → g
  depthwise conv+LN+Swish → v
  GEMM after_conv, mask, x += val → x
  LN ; FFN2 (as FFN1, 0.5 residual) → z
  LN(norm2)[+ next layer's FFN1 LN] → x, u
The residual stream stays fp32; GEMM/attention operands are bf16 under
torch.autocast (bf16 MFMA) and fp32 otherwise (exact-f32 MFMA, the parity
path).
"""
from typing import Optional

import torch
import torch.nn as nn

from .... import _autograd as A
from .... import _enc
from ....nnet.activations import Swish
from ....nnet.attention import FUSED_DH_MAX, MultiheadAttention, PositionalwiseFeedForward, RelPosMHAXL
from ....nnet.normalization import LayerNorm

__all__ = ["ConvolutionModule", "ConformerEncoderLayer", "ConformerEncoder"]

_f32 = torch.float32
_bf16 = torch.bfloat16

# Fused convolution-module kernel on the bf16 path (sbk_conv_module); the
# four-launch chain (LN, GLU GEMM, dwconv+LN+Swish, projection) otherwise.
USE_CONV_MODULE_KERNEL = True
# FFN2 (+ norm2) of layer i and FFN1 (+ norm1 + in_proj) of layer i+1 in one
# launch (sbk_ffn_chain), the out_proj in the conv module's prologue
USE_LAYER_CHAIN = True
# bf16 stacks with d_model < 256 (conformer_small.yaml: 144) on a zero-padded
# D = 256 copy, so they take the fused kernels (_PaddedEncoder)
USE_PADDED_SHADOW = True
PAD_D = 256


def _check_swish(act_module):
    if not (isinstance(act_module, Swish) or type(act_module).__name__ == "Swish"):
        raise NotImplementedError("fused conv module supports the Swish activation only")
    if getattr(act_module, "beta", 1) != 1:
        raise NotImplementedError("Swish(beta != 1) is not fused")


class ConvolutionModule(nn.Module):
    """Conformer.py:24-115."""

    _deff = None  # zero-padded shadow copies (_PaddedEncoder): LN statistics over this many channels

    def __init__(self, input_size, kernel_size=31, bias=True, activation=Swish, dropout=0.0, causal=False,
                 dilation=1):
        super().__init__()
        self.causal = causal
        if dilation != 1:
            raise NotImplementedError("dilated depthwise conv is not on the hot path")
        if self.causal:
            self.padding = (kernel_size - 1) * 2 ** (dilation - 1)
        else:
            self.padding = (kernel_size - 1) * 2 ** (dilation - 1) // 2
        self.layer_norm = nn.LayerNorm(input_size)
        self.bottleneck = nn.Sequential(
            nn.Conv1d(input_size, 2 * input_size, kernel_size=1, stride=1, bias=bias), nn.GLU(dim=1))
        self.conv = nn.Conv1d(input_size, input_size, kernel_size=kernel_size, stride=1, padding=self.padding,
                              dilation=dilation, groups=input_size, bias=bias)
        self.after_conv = nn.Sequential(nn.LayerNorm(input_size), activation(), nn.Linear(input_size, input_size,
                                                                                          bias=bias),
                                        nn.Dropout(dropout))
        self._wc = _enc.WeightCache()

    def kernel_weights(self, dtype):
        """(GLU-permuted pointwise weight, permuted bias, after_conv weight)."""
        w1 = self.bottleneck[0].weight
        b1 = self.bottleneck[0].bias
        w2 = self.after_conv[2].weight

        def make():
            d = w2.shape[0]
            grp = _enc.glu_group()  # output channels per wave tile of the GLU GEMM
            perm = []
            for q in range(d // grp):
                perm += list(range(q * grp, (q + 1) * grp))
                perm += list(range(d + q * grp, d + (q + 1) * grp))
            idx = torch.tensor(perm, device=w1.device)
            w1p = w1.detach().reshape(2 * d, d).index_select(0, idx).contiguous()
            b1p = b1.detach().index_select(0, idx).contiguous() if b1 is not None else None
            w2d = w2.detach().contiguous()
            if dtype == _bf16:
                w1p, w2d = _enc.cast_bf16(w1p), _enc.cast_bf16(w2d)
            return w1p, b1p, w2d
        ps = [w1, w2] + ([b1] if b1 is not None else [])
        return self._wc.get(str(dtype), ps, make)

    def ln_params(self):
        return (self.layer_norm.weight.detach(), self.layer_norm.bias.detach(), self.layer_norm.eps)

    def run(self, x2d, B, T, dtype, pad_mask_u8=None, residual=None, u=None):
        """x2d: (B*T, d) fp32 → residual + mask(ConvolutionModule(x)) (fp32).
        u: LN(x2d) in `dtype` when the producer already computed it."""
        d = x2d.shape[1]
        if d % _enc.glu_group():
            raise NotImplementedError("fused GLU needs d_model % 16 == 0")
        _check_swish(self.after_conv[1])
        w1p, b1p, w2 = self.kernel_weights(dtype)
        if u is None:
            u, _ = _enc.layernorm(x2d, *self.ln_params(), out1_dtype=dtype)
        g = _enc.gemm(u, w1p, bias=b1p, act="glu", out_dtype=dtype)
        ln = self.after_conv[0]
        v = _enc.dwconv_ln_swish(g, B, T, self.conv.weight.detach(), self.conv.bias.detach() if self.conv.bias is not None
                                 else None, self.causal, ln.weight.detach(), ln.bias.detach(), ln.eps, dtype)
        lin = self.after_conv[2]
        return _enc.gemm(v, w2, bias=lin.bias.detach() if lin.bias is not None else None, rowmask=pad_mask_u8,
                         res=residual, out_dtype=_f32)

    def fusable(self, dtype, d):
        """True when the whole module can run as one kernel (sbk_conv_module)."""
        return (dtype == _bf16 and _enc.conv_module_supported(d, self.conv.weight.shape[-1])
                and self.bottleneck[0].bias is not None and isinstance(self.after_conv[1], Swish)
                and getattr(self.after_conv[1], "beta", 1) == 1)

    def run_fused(self, x2d, B, T, pad_mask_u8=None, pre=None):
        """x2d + mask(ConvolutionModule(x2d)) in one launch (bf16 MFMA);
        pre = (o, wo, bo): on x2d + o wo^T + bo (the MHSA out_proj fused in)."""
        w1p, b1p, w2 = self.kernel_weights(_bf16)
        ln = self.after_conv[0]
        lin = self.after_conv[2]
        wc = self._wc.get("taps", [self.conv.weight], lambda: self.conv.weight.detach().reshape(
            self.conv.weight.shape[0], -1).t().contiguous())  # (K, d): coalesced tap loads
        return _enc.conv_module(x2d, B, T, self.ln_params(), w1p, b1p, wc,
                                self.conv.bias.detach() if self.conv.bias is not None else None, self.causal,
                                (ln.weight.detach(), ln.bias.detach(), ln.eps), w2,
                                lin.bias.detach() if lin.bias is not None else None, pad_mask_u8, pre=pre,
                                deff=self._deff)

    def train_run(self, x2d, B, T, dtype, pad_mask_u8=None, residual=None):
        """Differentiable chain (training path, _autograd): residual +
        mask(ConvolutionModule(x2d)), each op a HIP kernel with its backward."""
        _check_swish(self.after_conv[1])
        d = x2d.shape[1]
        u = A.layer_norm(x2d, self.layer_norm, out_dtype=dtype)
        pw = self.bottleneck[0]
        h = A.linear(u, pw.weight, pw.bias, dtype, self._wc, "t_pw", out_dtype=dtype)
        g = A.act(h, "glu")
        c = A.DwConvFn.apply(g, self.conv.weight, self.conv.bias, B, T, self.causal)
        n = A.layer_norm(c, self.after_conv[0], out_dtype=_f32)
        s = A.act(n, "swish", out_dtype=dtype)
        lin = self.after_conv[2]
        p = self.after_conv[3].p if self.training else 0.0
        if p == 0:
            return A.linear(s, lin.weight, lin.bias, dtype, self._wc, "t_lin", res=residual, rowmask=pad_mask_u8)
        y = A.linear(s, lin.weight, lin.bias, dtype, self._wc, "t_lin")
        return A.DropAddFn.apply(y, residual, 1.0, pad_mask_u8, float(p), _f32)

    def forward(self, x, mask=None):
        B, T, d = x.shape
        m = mask.reshape(B * T).to(torch.uint8).contiguous() if mask is not None else None
        x2d = x.float().reshape(B * T, d).contiguous()
        if A.needs_grad(self, x) or (self.training and self.after_conv[3].p > 0):
            return self.train_run(x2d, B, T, _enc.compute_dtype(), m).view(B, T, d)
        return self.run(x2d, B, T, _enc.compute_dtype(), m).view(B, T, d)


class ConformerEncoderLayer(nn.Module):
    """Conformer.py:118-260."""

    def __init__(self, d_model, d_ffn, nhead, kernel_size=31, kdim=None, vdim=None, activation=Swish, bias=True,
                 dropout=0.0, causal=False, attention_type="RelPosMHAXL"):
        super().__init__()
        if attention_type == "regularMHA":  # Conformer.py:173-180
            self.mha_layer = MultiheadAttention(nhead=nhead, d_model=d_model, dropout=dropout, kdim=kdim, vdim=vdim)
        elif attention_type == "RelPosMHAXL":  # :181-188
            self.mha_layer = RelPosMHAXL(num_heads=nhead, embed_dim=d_model, dropout=dropout,
                                         mask_pos_future=causal)
        else:
            raise ValueError(f"attention_type {attention_type!r}: 'regularMHA' or 'RelPosMHAXL'")
        self.attention_type = attention_type
        # the per-module layer (mha_layer_forward): regularMHA, or heads wider than the fused kernels take
        self.module_layer = attention_type == "regularMHA" or d_model // nhead > FUSED_DH_MAX
        self.convolution_module = ConvolutionModule(d_model, kernel_size, bias, activation, dropout, causal=causal)
        self.ffn_module1 = nn.Sequential(
            nn.LayerNorm(d_model),
            PositionalwiseFeedForward(d_ffn=d_ffn, input_size=d_model, dropout=dropout, activation=activation),
            nn.Dropout(dropout))
        self.ffn_module2 = nn.Sequential(
            nn.LayerNorm(d_model),
            PositionalwiseFeedForward(d_ffn=d_ffn, input_size=d_model, dropout=dropout, activation=activation),
            nn.Dropout(dropout))
        self.norm1 = LayerNorm(d_model)
        self.norm2 = LayerNorm(d_model)
        self.drop = nn.Dropout(dropout)

    def _ln(self, mod):
        return mod.weight.detach(), mod.bias.detach(), mod.eps

    def chainable(self, dtype, d):
        """Every block of this layer has its fused kernel (the chained stack)."""
        if self.training and self.drop.p > 0 or self.module_layer:
            return False
        f1, f2 = self.ffn_module1, self.ffn_module2
        mha = self.mha_layer
        return (f1[1].fusable(dtype) and f2[1].fusable(dtype) and f1[1].act_name() == f2[1].act_name()
                and f1[1].ffn[0].out_features == f2[1].ffn[0].out_features
                and hasattr(mha, "fused_in_proj") and mha.fused_in_proj(dtype) is not None
                and self.convolution_module.fusable(dtype, d))

    def fused(self, x, B, T, pos, kpm_u8, dtype, need_attn, u_in=None, next_ln=None, final_ln=None, pk=None,
              am=None):
        """One layer.  x: (B*T, d) fp32 residual stream; pos: (2T-1, d) in
        dtype; u_in: LN_ffn1(x) if a previous kernel already produced it;
        next_ln: (w, b, eps) of the NEXT consumer's LayerNorm to chain after
        norm2; final_ln: the encoder's closing LayerNorm, applied on chip by
        the fused-FFN path; pk: this layer's linear_pos(pos) if precomputed;
        am: the attention mask (_enc.attn_mask_arg) or None.
        Returns (x_out fp32, u_next or None, attn or None, final_ln_applied)."""
        if self.training and self.drop.p > 0:
            raise NotImplementedError("dropout in training mode is not implemented in HIP yet")
        f1, f2 = self.ffn_module1, self.ffn_module2
        if f1[1].fusable(dtype) and f2[1].fusable(dtype):
            # FFN1 + norm1 in one kernel, FFN2 + norm2 in one kernel (LayerNorms
            # computed on chip; the next layer's FFN1 normalises its own input)
            wq = self.mha_layer.fused_in_proj(dtype) if hasattr(self.mha_layer, "fused_in_proj") else None
            qkv = None
            if wq is not None:
                # ... and the MHSA in_proj on chip too (norm1's output never leaves the CU)
                x, qkv = f1[1].run_fused_proj(x, self._ln(f1[0]), 0.5, self._ln(self.norm1.norm), wq)
                u = None
            else:
                x, u = f1[1].run_fused(x, self._ln(f1[0]), 0.5, next_ln=self._ln(self.norm1.norm),
                                       next_dtype=dtype)
            cm = self.convolution_module
            if USE_CONV_MODULE_KERNEL and cm.fusable(dtype, x.shape[1]):
                # attention, then the output projection + residual + the whole
                # convolution module (its LayerNorms included) in one launch
                if hasattr(self.mha_layer, "attend_heads"):
                    o, attn, pre = self.mha_layer.attend_heads(u, B, T, pos, kpm_u8, dtype, need_attn, pk=pk,
                                                               qkv=qkv, am=am)
                    x = cm.run_fused(x, B, T, kpm_u8, pre=pre)
                else:
                    x, attn = self.mha_layer.attend(u, B, T, pos, kpm_u8, dtype, need_attn, residual=x, pk=pk,
                                                    qkv=qkv, am=am)
                    x = cm.run_fused(x, B, T, kpm_u8)
            else:
                # attention output projection + residual + the conv module's LayerNorm in one launch
                x, attn, uc = self.mha_layer.attend(u, B, T, pos, kpm_u8, dtype, need_attn, residual=x,
                                                    post_ln=cm.ln_params(), pk=pk, qkv=qkv, am=am)
                x = cm.run(x, B, T, dtype, kpm_u8, residual=x, u=uc)
            x, y = f2[1].run_fused(x, self._ln(f2[0]), 0.5, post_ln=self._ln(self.norm2.norm), out=x,
                                   next_ln=final_ln, next_dtype=_f32)
            return (y, None, attn, True) if final_ln is not None else (x, None, attn, False)
        if u_in is None:
            u_in, _ = _enc.layernorm(x, *self._ln(f1[0]), out1_dtype=dtype)
        x = f1[1].run(u_in, dtype, residual=x, alpha=0.5)
        u, _ = _enc.layernorm(x, *self._ln(self.norm1.norm), out1_dtype=dtype)
        x, attn, uc = self.mha_layer.attend(u, B, T, pos, kpm_u8, dtype, need_attn, residual=x,
                                            post_ln=self.convolution_module.ln_params(), pk=pk, am=am)
        x = self.convolution_module.run(x, B, T, dtype, kpm_u8, residual=x, u=uc)
        u, _ = _enc.layernorm(x, *self._ln(f2[0]), out1_dtype=dtype)
        z = f2[1].run(u, dtype, residual=x, alpha=0.5)
        w2, b2, e2 = self._ln(self.norm2.norm)
        if next_ln is not None:
            x, u_next = _enc.layernorm(z, w2, b2, e2, out1_dtype=_f32, w2=next_ln[0], b2=next_ln[1],
                                       eps2=next_ln[2], out2_dtype=dtype)
            return x, u_next, attn, False
        x, _ = _enc.layernorm(z, w2, b2, e2, out1_dtype=_f32)
        return x, None, attn, False

    def train_layer(self, x, B, T, pos, kpm_u8, dtype, am=None):
        """Differentiable layer (training path): x (B*T, d) fp32 → (x_out, attn).
        Same arithmetic as `fused`, as HIP kernels with backward (_autograd);
        dropout (training mode) after the FFN activation, on the FFN and conv
        outputs and on the attention probabilities, as the reference places it."""
        f1, f2 = self.ffn_module1, self.ffn_module2
        tr = self.training
        u = A.layer_norm(x, f1[0], out_dtype=dtype)
        x = f1[1].train_run(u, dtype, residual=x, alpha=0.5, out_p=f1[2].p if tr else 0.0)
        u = A.layer_norm(x, self.norm1.norm, out_dtype=dtype)
        x, attn = self.mha_layer.train_attend(u, B, T, pos, kpm_u8, dtype, residual=x, am=am)
        x = self.convolution_module.train_run(x, B, T, dtype, kpm_u8, residual=x)
        u = A.layer_norm(x, f2[0], out_dtype=dtype)
        z = f2[1].train_run(u, dtype, residual=x, alpha=0.5, out_p=f2[2].p if tr else 0.0)
        return A.layer_norm(z, self.norm2.norm, out_dtype=_f32), attn

    def mha_layer_forward(self, x, B, T, kpm_u8, src_mask, pos_embs, dtype):
        """Conformer.py:239-260 block by block on the drop-in modules, for the
        regularMHA attention (:173-180) and for heads wider than the fused
        kernels take: x (B*T, d) fp32 → (x_out, attention).  The FFN,
        LayerNorm and convolution-module blocks are the training path's HIP
        autograd Functions (they run as plain kernels under no_grad); the
        attention is the mha_layer drop-in on norm1's output —
        MultiheadAttention's fused kernels at inference and its general path
        (src_mask, pos_embs added to the mask as attention.py:756-761,
        dropout, gradients) otherwise; RelPosMHAXL's xattn core."""
        f1, f2 = self.ffn_module1, self.ffn_module2
        tr = self.training
        d = x.shape[1]
        u = A.layer_norm(x, f1[0], out_dtype=dtype)
        x = f1[1].train_run(u, dtype, residual=x, alpha=0.5, out_p=f1[2].p if tr else 0.0)
        u = A.layer_norm(x, self.norm1.norm, out_dtype=_f32).view(B, T, d)
        o, attn = self.mha_layer(u, u, u, attn_mask=src_mask, key_padding_mask=kpm_u8, pos_embs=pos_embs)
        x = A.DropAddFn.apply(o.reshape(B * T, d).float(), x, 1.0, None, 0.0, _f32)
        x = self.convolution_module.train_run(x, B, T, dtype, kpm_u8, residual=x)
        u = A.layer_norm(x, f2[0], out_dtype=dtype)
        z = f2[1].train_run(u, dtype, residual=x, alpha=0.5, out_p=f2[2].p if tr else 0.0)
        return A.layer_norm(z, self.norm2.norm, out_dtype=_f32), attn

    def wants_train_path(self, x):
        return A.needs_grad(self, x) or (self.training and self.ffn_module1[2].p > 0)

    def forward(self, x, src_mask: Optional[torch.Tensor] = None,
                src_key_padding_mask: Optional[torch.Tensor] = None, pos_embs: Optional[torch.Tensor] = None):
        B, T, d = x.shape
        dtype = _enc.compute_dtype()
        kpm = src_key_padding_mask.to(torch.uint8).contiguous() if src_key_padding_mask is not None else None
        if self.module_layer:
            y, attn = self.mha_layer_forward(x.float().reshape(B * T, d).contiguous(), B, T, kpm, src_mask,
                                             pos_embs, dtype)
            return y.view(B, T, d), attn
        am = _enc.attn_mask_arg(src_mask, B, T, self.mha_layer.num_heads, x.device)
        x2d = x.float().reshape(B * T, d).contiguous()
        if self.wants_train_path(x):
            y, attn = self.train_layer(x2d, B, T, pos_embs.reshape(-1, d).float(), kpm, dtype, am=am)
            return y.view(B, T, d), attn
        pos = _enc.to_compute(pos_embs.reshape(-1, d), dtype)
        y, _, attn, _ = self.fused(x2d, B, T, pos, kpm, dtype, True, am=am)
        return y.view(B, T, d), attn


class ConformerEncoder(nn.Module):
    """Conformer.py:263-383."""

    def __init__(self, num_layers, d_model, d_ffn, nhead, kernel_size=31, kdim=None, vdim=None, activation=Swish,
                 bias=True, dropout=0.0, causal=False, attention_type="RelPosMHAXL"):
        super().__init__()
        self.layers = torch.nn.ModuleList([
            ConformerEncoderLayer(d_ffn=d_ffn, nhead=nhead, d_model=d_model, kdim=kdim, vdim=vdim, dropout=dropout,
                                  activation=activation, kernel_size=kernel_size, bias=bias, causal=causal,
                                  attention_type=attention_type) for i in range(num_layers)])
        self.norm = LayerNorm(d_model, eps=1e-6)
        self.attention_type = attention_type
        self._wc = _enc.WeightCache()

    def stacked_pos_weight(self, dtype):
        """linear_pos weights of all layers stacked (L*d, d) in the compute dtype,
        so p_k of every layer comes from one GEMM (p_k depends only on the
        positional table, not on the layer input)."""
        ws = [layer.mha_layer.linear_pos.weight for layer in self.layers]

        def make():
            w = torch.cat([p.detach() for p in ws], dim=0).contiguous()
            return _enc.cast_bf16(w) if dtype == _bf16 else w
        return self._wc.get(("pos", dtype), ws, make)

    def train_run(self, src2d, B, T, pos_embs, kpm_u8, dtype, am=None):
        """Differentiable stack (training path) on (B*T, d) fp32 → (y, [attn])."""
        d = src2d.shape[1]
        pos = pos_embs.reshape(-1, d).float()
        x = src2d
        attns = []
        for layer in self.layers:
            x, a = layer.train_layer(x, B, T, pos, kpm_u8, dtype, am=am)
            attns.append(a)
        return A.layer_norm(x, self.norm.norm, out_dtype=_f32), attns

    def wants_train_path(self, x):
        return any(layer.wants_train_path(x) for layer in self.layers) or A.needs_grad(self.norm, x)

    def _shadow(self, d, dtype, am=None):
        if USE_PADDED_SHADOW and am is None and dtype == _bf16 and d < PAD_D:
            return _PaddedEncoder.of(self)
        return None

    def run(self, src2d, B, T, pos_embs, kpm_u8, dtype, need_attn, am=None):
        """Fused stack on (B*T, d) fp32 → ((B*T, d) fp32, [attn]); am: the
        src_mask as _enc.attn_mask_arg (takes the per-layer path).  A bf16
        stack with d_model < 256 runs on its zero-padded D = 256 shadow
        (_PaddedEncoder) when that shadow takes the layer chain."""
        if self.wants_train_path(src2d):
            return self.train_run(src2d, B, T, pos_embs, kpm_u8, dtype, am=am)
        d = src2d.shape[1]
        sh = self._shadow(d, dtype, am)
        if sh is not None:
            return sh.run(src2d, B, T, pos_embs, kpm_u8, dtype, need_attn)
        pos = _enc.to_compute(pos_embs.reshape(-1, d), dtype)
        pk_all = _enc.gemm(pos, self.stacked_pos_weight(dtype), out_dtype=dtype)  # (2T-1, L*d)
        x = src2d
        u = None
        attns = []
        n = len(self.layers)
        if (USE_LAYER_CHAIN and am is None and all(layer.chainable(dtype, d) for layer in self.layers)
                and self._uniform_ffns()):
            return self._run_chain(x, B, T, pos, kpm_u8, dtype, need_attn, pk_all)
        for i, layer in enumerate(self.layers):
            nxt = self.layers[i + 1].ffn_module1[0] if i + 1 < n else None
            next_ln = (nxt.weight.detach(), nxt.bias.detach(), nxt.eps) if nxt is not None else None
            fn = self.norm.norm
            final_ln = (fn.weight.detach(), fn.bias.detach(), fn.eps) if nxt is None else None
            x, u, a, done = layer.fused(x, B, T, pos, kpm_u8, dtype, need_attn, u_in=u, next_ln=next_ln,
                                        final_ln=final_ln, pk=pk_all[:, i * d:(i + 1) * d], am=am)
            attns.append(a)
            if done:
                return x, attns
        fn = self.norm.norm
        y, _ = _enc.layernorm(x, fn.weight.detach(), fn.bias.detach(), fn.eps, out1_dtype=_f32)
        return y, attns

    def _uniform_ffns(self):
        """The chain kernel runs layer i's FFN2 with layer i+1's FFN1 under one
        activation and hidden size: every layer's FFNs must agree."""
        f = [m[1] for layer in self.layers for m in (layer.ffn_module1, layer.ffn_module2)]
        return all(x.act_name() == f[0].act_name() and x.ffn[0].out_features == f[0].ffn[0].out_features for x in f)

    def _run_chain(self, x, B, T, pos, kpm_u8, dtype, need_attn, pk_all):
        """The fused stack as 3 launches per layer: [FFN2_i + norm2_i +
        FFN1_{i+1} + norm1_{i+1} + in_proj_{i+1}] (sbk_ffn_chain), attention,
        [out_proj + residual + conv module] (sbk_conv_module_pre); layer 0's
        FFN1 is sbk_ffn_proj, the last FFN2 carries the closing LayerNorm."""
        d = x.shape[1]
        ln = ConformerEncoderLayer._ln
        L = self.layers
        l0 = L[0]
        f1 = l0.ffn_module1
        x, qkv = f1[1].run_fused_proj(x, ln(l0, f1[0]), 0.5, ln(l0, l0.norm1.norm), l0.mha_layer.fused_in_proj(dtype))
        attns = []
        for i, layer in enumerate(L):
            _, attn, pre = layer.mha_layer.attend_heads(None, B, T, pos, kpm_u8, dtype, need_attn,
                                                        pk=pk_all[:, i * d:(i + 1) * d], qkv=qkv)
            attns.append(attn)
            x = layer.convolution_module.run_fused(x, B, T, kpm_u8, pre=pre)
            f2 = layer.ffn_module2
            if i + 1 < len(L):
                nl = L[i + 1]
                a = f2[1].chain_block(ln(layer, f2[0]), 0.5, post_ln=ln(layer, layer.norm2.norm))
                b = nl.ffn_module1[1].chain_block(ln(nl, nl.ffn_module1[0]), 0.5)
                act, slope = f2[1].act_name()
                x, qkv = _enc.ffn_chain(x, a, b, act, slope, ln(nl, nl.norm1.norm), nl.mha_layer.fused_in_proj(dtype),
                                        deff=f2[1]._deff)
            else:
                fn = self.norm.norm
                _, y = f2[1].run_fused(x, ln(layer, f2[0]), 0.5, post_ln=ln(layer, layer.norm2.norm),
                                       next_ln=(fn.weight.detach(), fn.bias.detach(), fn.eps), next_dtype=_f32)
                return y, attns

    def forward(self, src, src_mask: Optional[torch.Tensor] = None,
                src_key_padding_mask: Optional[torch.Tensor] = None, pos_embs: Optional[torch.Tensor] = None):
        if self.attention_type == "RelPosMHAXL" and pos_embs is None:
            raise ValueError("The chosen attention type for the Conformer is RelPosMHAXL. For this attention type, "
                             "the positional embeddings are mandatory")
        B, T, d = src.shape
        kpm = src_key_padding_mask.to(torch.uint8).contiguous() if src_key_padding_mask is not None else None
        if self.layers[0].module_layer:
            # Conformer.py:371-383 on the per-module layers (regularMHA: pos_embs
            # reach the attention mask as in the reference, None from TransformerASR)
            x = src.float().reshape(B * T, d).contiguous()
            attns = []
            for layer in self.layers:
                x, a = layer.mha_layer_forward(x, B, T, kpm, src_mask, pos_embs, _enc.compute_dtype())
                attns.append(a)
            return A.layer_norm(x, self.norm.norm, out_dtype=_f32).view(B, T, d), attns
        am = _enc.attn_mask_arg(src_mask, B, T, self.layers[0].mha_layer.num_heads, src.device)
        y, attns = self.run(src.float().reshape(B * T, d).contiguous(), B, T, pos_embs, kpm,
                            _enc.compute_dtype(), True, am=am)
        return y.view(B, T, d), attns


class _PaddedEncoder:
    """A ConformerEncoder with d_model < 256 (conformer_small.yaml:96-100:
    144) as a zero-padded D = 256 shadow, so its bf16 inference runs the
    fused layer chain, rel-pos attention and convolution-module kernels,
    which are built for 256 channels and 64-dim heads.

    Residual-stream channels d..255 are zero and stay zero: every LayerNorm
    gain / bias, weight row that writes them and weight column that reads
    them is zero, so GEMM sums, the GLU, the depthwise taps and Swish see
    exact zeros there; the kernels take d_eff = d for their LayerNorm
    statistics (sbk_ffn / sbk_conv_module: mean over d, the centred sum less
    the (256 - d) mean^2 the padded zeros add).  Attention heads are padded
    from d / H to 64 dims (q, k, v, the positional rows, pos_bias_u / v), with
    the reference's scale 1 / sqrt(d) kept — identical scores and
    probabilities.  Results equal the unpadded bf16 arithmetic up to MFMA
    summation order.  Built once per parameter version (weights are copied,
    not shared) and cached on the encoder."""

    def __init__(self, enc, dev):
        d = enc.norm.norm.weight.shape[0]
        l0 = enc.layers[0]
        H = l0.mha_layer.num_heads
        K = l0.convolution_module.conv.weight.shape[-1]
        F = l0.ffn_module1[1].ffn[0].out_features
        act = type(l0.ffn_module1[1].ffn[1])
        self.d = d
        with torch.random.fork_rng(devices=[]):  # the shadow's own init must not move the global RNG
            sh = ConformerEncoder(len(enc.layers), PAD_D, F, H, kernel_size=K, activation=act,
                                  bias=l0.convolution_module.conv.bias is not None,
                                  causal=l0.convolution_module.causal)
        sh = sh.to(dev).eval()
        dh, dp = d // H, PAD_D // H
        hmap = torch.tensor([h * dp + i for h in range(H) for i in range(dh)], device=dev)
        qmap = torch.tensor([h * 3 * dp + p * dp + i for h in range(H) for p in range(3) for i in range(dh)],
                            device=dev)
        gmap = torch.cat([torch.arange(d, device=dev), PAD_D + torch.arange(d, device=dev)])

        def put(dst, src, rows=None, cols=None):
            """zero dst, then dst[rows][:, cols] = src (None: the leading range)."""
            src = src.detach().to(dev, torch.float32)
            dst.zero_()
            r = rows if rows is not None else torch.arange(src.shape[0], device=dev)
            if dst.dim() == 1:
                dst[r] = src
                return
            tmp = torch.zeros(src.shape[0], *dst.shape[1:], device=dev)
            if cols is None:
                tmp[:, :src.shape[1]] = src
            else:
                tmp[:, cols] = src
            dst[r] = tmp

        with torch.no_grad():
            for lr, ls in zip(enc.layers, sh.layers):
                for fr_, fs in ((lr.ffn_module1, ls.ffn_module1), (lr.ffn_module2, ls.ffn_module2)):
                    put(fs[0].weight, fr_[0].weight)
                    put(fs[0].bias, fr_[0].bias)
                    put(fs[1].ffn[0].weight, fr_[1].ffn[0].weight, rows=torch.arange(F, device=dev))
                    put(fs[1].ffn[0].bias, fr_[1].ffn[0].bias, rows=torch.arange(F, device=dev))
                    put(fs[1].ffn[3].weight, fr_[1].ffn[3].weight)
                    put(fs[1].ffn[3].bias, fr_[1].ffn[3].bias)
                    fs[1]._deff = d
                mr, ms = lr.mha_layer, ls.mha_layer
                put(ms.in_proj_weight, mr.in_proj_weight, rows=qmap)
                # the (dh, H) biases are read as (H, dh) (attention.py:586-592): flat h * dh + i -> h * 64 + i
                put(ms.pos_bias_u.view(-1), mr.pos_bias_u.reshape(-1), rows=hmap)
                put(ms.pos_bias_v.view(-1), mr.pos_bias_v.reshape(-1), rows=hmap)
                put(ms.linear_pos.weight, mr.linear_pos.weight, rows=hmap)
                put(ms.out_proj.weight, mr.out_proj.weight, cols=hmap)
                put(ms.out_proj.bias, mr.out_proj.bias)
                ms.scale = mr.scale
                cr, cs = lr.convolution_module, ls.convolution_module
                put(cs.layer_norm.weight, cr.layer_norm.weight)
                put(cs.layer_norm.bias, cr.layer_norm.bias)
                put(cs.bottleneck[0].weight.view(2 * PAD_D, PAD_D), cr.bottleneck[0].weight.view(2 * d, d), rows=gmap)
                if cr.bottleneck[0].bias is not None:
                    put(cs.bottleneck[0].bias, cr.bottleneck[0].bias, rows=gmap)
                put(cs.conv.weight.view(PAD_D, K), cr.conv.weight.view(d, K))
                if cr.conv.bias is not None:
                    put(cs.conv.bias, cr.conv.bias)
                put(cs.after_conv[0].weight, cr.after_conv[0].weight)
                put(cs.after_conv[0].bias, cr.after_conv[0].bias)
                put(cs.after_conv[2].weight, cr.after_conv[2].weight)
                if cr.after_conv[2].bias is not None:
                    put(cs.after_conv[2].bias, cr.after_conv[2].bias)
                cs._deff = d
                for nr, ns in ((lr.norm1.norm, ls.norm1.norm), (lr.norm2.norm, ls.norm2.norm)):
                    put(ns.weight, nr.weight)
                    put(ns.bias, nr.bias)
                    ns.eps = nr.eps
                for a, b in ((lr.ffn_module1[0], ls.ffn_module1[0]), (lr.ffn_module2[0], ls.ffn_module2[0]),
                             (cr.layer_norm, cs.layer_norm), (cr.after_conv[0], cs.after_conv[0])):
                    b.eps = a.eps
            put(sh.norm.norm.weight, enc.norm.norm.weight)
            put(sh.norm.norm.bias, enc.norm.norm.bias)
            sh.norm.norm.eps = enc.norm.norm.eps
        self.sh = sh
        self._pos = {}

    @staticmethod
    def of(enc):
        """The encoder's shadow for its current parameters (None when the
        padded stack would not take the layer chain)."""
        ps = list(enc.parameters())
        dev = ps[0].device
        sig = (str(dev),) + tuple((p.data_ptr(), p._version) for p in ps)
        hit = getattr(enc, "_padded_shadow", None)
        if hit is not None and hit[0] == sig:
            return hit[1]
        l0 = enc.layers[0]
        d = enc.norm.norm.weight.shape[0]
        ok = (l0.attention_type == "RelPosMHAXL" and not l0.module_layer and d % l0.mha_layer.num_heads == 0
              and PAD_D % l0.mha_layer.num_heads == 0 and l0.mha_layer.vbias is None
              and l0.mha_layer._qkv_same_embed_dim and enc._uniform_ffns())
        shadow = None
        if ok:
            shadow = _PaddedEncoder(enc, dev)
            if not (all(layer.chainable(_bf16, PAD_D) for layer in shadow.sh.layers) and shadow.sh._uniform_ffns()):
                shadow = None
        enc._padded_shadow = (sig, shadow)
        return shadow

    def padded_pos(self, pos_embs, dtype):
        """The positional table (a per-T constant) padded to 256 columns, once."""
        d = self.d
        key = (pos_embs.data_ptr(), tuple(pos_embs.shape), dtype)
        pos = self._pos.get(key)
        if pos is None:
            p = pos_embs.reshape(-1, d)
            pos = torch.zeros(p.shape[0], PAD_D, device=p.device, dtype=dtype)
            pos[:, :d] = p.to(dtype)
            self._pos = {key: pos}
        return pos

    def run(self, src2d, B, T, pos_embs, kpm_u8, dtype, need_attn):
        d = self.d
        if src2d.shape[1] == PAD_D:  # already padded by the producer (TransformerASR's padded src Linear)
            x = src2d
        else:
            x = torch.zeros(src2d.shape[0], PAD_D, device=src2d.device, dtype=torch.float32)
            x[:, :d] = src2d
        y, attns = self.sh.run(x, B, T, self.padded_pos(pos_embs, dtype), kpm_u8, dtype, need_attn)
        return y[:, :d].contiguous(), attns
