"""Drop-in for speechbrain.nnet.attention: RelPosEncXL, RelPosMHAXL,
PositionalwiseFeedForward (speechbrain/nnet/attention.py:312-839).

Parameter names and shapes match the reference so checkpoints load with
strict=True.  RelPosMHAXL self-attention runs as: in_proj GEMM (MFMA) →
linear_pos GEMM → one fused rel-pos attention kernel (scores, closed-form
rel_shift, mask, softmax, P·V) → out_proj GEMM.  With query != key / value
(any q_len, k_len) it runs separate q / k / v GEMMs → the cross-length
rel-pos core of csrc/xattn.hip → out_proj, forward and backward.
"""
import math

import torch
import torch.nn as nn

from .. import _autograd as A
from .. import _enc
from .activations import Swish

__all__ = ["RelPosEncXL", "RelPosMHAXL", "PositionalwiseFeedForward", "MultiheadAttention"]

# head size limit of the fused self-attention kernels (csrc/attention.hip);
# wider heads take the xattn core (dh <= 256), as any cross-attention does
FUSED_DH_MAX = 128


class RelPosEncXL(nn.Module):
    """attention.py:312-359.  The (1, 2T-1, d) table depends only on T and d;
    it is built once per (T, device, dtype) on the host from the registered
    inv_freq buffer and cached (the bf16 encoder path takes the bf16 table, so
    no step casts it)."""

    def __init__(self, emb_dim):
        super().__init__()
        self.emb_dim = emb_dim
        inv_freq = torch.exp(torch.arange(0, self.emb_dim, 2, dtype=torch.float32)
                             * -(math.log(10000.0) / self.emb_dim))
        self.register_buffer("inv_freq", inv_freq)
        self._cache = {}

    def table(self, seq_len, device, dtype=torch.float32):
        key = (seq_len, str(device), dtype, self.inv_freq.data_ptr())
        pe = self._cache.get(key)
        if pe is None:
            inv = self.inv_freq.detach().to("cpu", torch.float32)
            pos = torch.arange(0, seq_len, dtype=torch.float32).unsqueeze(-1)
            pe_half = torch.zeros(seq_len, self.emb_dim, dtype=torch.float32)
            pe_half[:, 0::2] = torch.sin(pos * inv)
            pe_half[:, 1::2] = torch.cos(pos * inv)  # cos(-x) == cos(x): past/future equal
            pe = torch.cat([torch.flip(pe_half, (0,)), pe_half[1:]], dim=0).unsqueeze(0)
            pe = pe.to(device=device, dtype=dtype)  # bf16: round-to-nearest-even, as the cast kernel
            if len(self._cache) >= 8:
                self._cache.clear()
            self._cache[key] = pe
        return pe

    def forward(self, x: torch.Tensor):
        return self.table(x.size(1), x.device, torch.float32 if x.dtype == torch.bfloat16 else x.dtype)


class RelPosMHAXL(nn.Module):
    """attention.py:362-639: self-attention on the fused rel-pos flash
    kernels; query != key / value (and q_len != k_len) on cross_forward."""

    def __init__(self, embed_dim, num_heads, dropout=0.0, vbias=False, vdim=None, mask_pos_future=False):
        super().__init__()
        self.embed_dim = embed_dim
        self.vdim = vdim if vdim is not None else embed_dim
        self._qkv_same_embed_dim = self.vdim == embed_dim
        self.mask_pos_future = mask_pos_future
        self.vbias = vbias
        self.num_heads = num_heads
        self.dropout = dropout
        self.head_dim = embed_dim // num_heads
        self.vhead_dim = self.vdim // num_heads
        assert self.head_dim * num_heads == self.embed_dim, "embed_dim must be divisible by num_heads"
        assert self.vhead_dim * num_heads == self.vdim, "vdim must be divisible by num_heads"
        if self._qkv_same_embed_dim is False:
            self.qk_proj_weight = nn.Parameter(torch.empty(2 * embed_dim, embed_dim))
            self.v_proj_weight = nn.Parameter(torch.empty(self.vdim, embed_dim))
        else:
            self.in_proj_weight = nn.Parameter(torch.empty(3 * embed_dim, embed_dim))
        if vbias:
            self.value_bias_weight = nn.Parameter(torch.empty(self.vdim))
        else:
            self.vbias = None
        self.dropout_att = nn.Dropout(dropout)
        self.out_proj = nn.Linear(self.vdim, embed_dim)
        self.linear_pos = nn.Linear(embed_dim, embed_dim, bias=False)
        self.pos_bias_u = nn.Parameter(torch.empty(self.head_dim, self.num_heads))
        self.pos_bias_v = nn.Parameter(torch.empty(self.head_dim, self.num_heads))
        if next(self.parameters()).dtype == torch.float16:
            self.attn_fill_value = -65000
        else:
            self.attn_fill_value = -float("inf")
        self._reset_parameters()
        self.scale = 1 / math.sqrt(self.embed_dim)
        self._wc = _enc.WeightCache()

    def _reset_parameters(self):
        if self._qkv_same_embed_dim:
            torch.nn.init.xavier_uniform_(self.in_proj_weight)
        else:
            torch.nn.init.xavier_uniform_(self.qk_proj_weight)
            torch.nn.init.xavier_uniform_(self.v_proj_weight)
        if self.vbias is not None:
            torch.nn.init.constant_(self.value_bias_weight, 0.0)
        torch.nn.init.xavier_uniform_(self.pos_bias_u)
        torch.nn.init.xavier_uniform_(self.pos_bias_v)

    def kernel_weights(self, dtype):
        """(in_proj, linear_pos, out_proj) weights in the compute dtype."""
        ps = [self.in_proj_weight, self.linear_pos.weight, self.out_proj.weight]
        if dtype == torch.float32:
            return tuple(p.detach() for p in ps)
        return self._wc.get("bf16", ps, lambda: tuple(_enc.cast_bf16(p.detach().contiguous()) for p in ps))

    def in_proj_bias(self):
        """vbias=True (attention.py:576-579): value + value_bias_weight per
        head, as a bias of the in_proj GEMM in the head-interleaved [q|k|v]
        layout (zeros for q and k).  Built from the parameter with torch ops
        (a 3·d vector), so its gradient reaches value_bias_weight.  None
        without vbias."""
        if self.vbias is None:
            return None
        H, dh = self.num_heads, self.head_dim
        vb = self.value_bias_weight.view(H, 1, dh)
        z = torch.zeros(H, 2, dh, device=vb.device, dtype=vb.dtype)
        return torch.cat([z, vb], dim=1).reshape(3 * H * dh)

    def fused_in_proj(self, dtype):
        """The bf16 in_proj weight when a producer kernel can apply it on chip
        (sbk_ffn_proj: no in_proj bias, 3·d columns in 256-column blocks), else None."""
        if dtype != torch.bfloat16 or self.vbias is not None or not self._qkv_same_embed_dim:
            return None
        w_in = self.kernel_weights(dtype)[0]
        return w_in if _enc.ffn_proj_supported(self.embed_dim, 256, w_in.shape[0]) else None

    def attend_heads(self, x2d, B, T, pos_embs, kpm_u8, dtype, need_weights, pk=None, qkv=None, am=None):
        """attend without the output projection: (o (B*T, d) in dtype, attn,
        (o, out_proj weight, bias)) for a consumer that applies out_proj
        itself (sbk_conv_module_pre)."""
        w_in, w_pos, w_out = self.kernel_weights(dtype)
        if qkv is None:
            ib = self.in_proj_bias()
            qkv = _enc.gemm(x2d, w_in, bias=None if ib is None else ib.detach(), out_dtype=dtype)
        if pk is None:
            pos = pos_embs.reshape(-1, self.embed_dim)
            if pos.dtype != dtype:
                pos = _enc.cast_bf16(pos.float().contiguous()) if dtype == torch.bfloat16 else pos.float()
            pk = _enc.gemm(pos.contiguous(), w_pos, out_dtype=dtype)
        o, probs = _enc.relpos_attention(qkv, pk, self.pos_bias_u.detach(), self.pos_bias_v.detach(), kpm_u8, B, T,
                                         self.num_heads, self.head_dim, self.scale, need_weights, am=am)
        return o, probs, (o, w_out, self.out_proj.bias.detach())

    def attend(self, x2d, B, T, pos_embs, kpm_u8, dtype, need_weights, residual=None, post_ln=None, pk=None,
               qkv=None, am=None):
        """Core used by the fused Conformer layer: x2d (B*T, d) in `dtype`
        (or qkv = x2d · in_proj^T already computed by the producer kernel).
        Returns (out (B*T, d) fp32 [+ residual], attn or None); with post_ln =
        (w, b, eps) also u = LN(out) in `dtype` (fused into the output
        projection when d_model == 256): (out, attn, u)."""
        w_in, w_pos, w_out = self.kernel_weights(dtype)
        if qkv is None:
            ib = self.in_proj_bias()
            qkv = _enc.gemm(x2d, w_in, bias=None if ib is None else ib.detach(), out_dtype=dtype)
        if pk is None:  # the encoder passes its one stacked linear_pos GEMM's slice
            pos = pos_embs.reshape(-1, self.embed_dim)
            if pos.dtype != dtype:
                pos = _enc.cast_bf16(pos.float().contiguous()) if dtype == torch.bfloat16 else pos.float()
            pk = _enc.gemm(pos.contiguous(), w_pos, out_dtype=dtype)
        o, probs = _enc.relpos_attention(qkv, pk, self.pos_bias_u.detach(), self.pos_bias_v.detach(), kpm_u8, B, T,
                                         self.num_heads, self.head_dim, self.scale, need_weights, am=am)
        bias = self.out_proj.bias.detach()
        if post_ln is not None:
            if _enc.gemm_ln_supported(self.embed_dim) and _enc.USE_GEMM_LN:
                out, u = _enc.gemm_ln(o, w_out, post_ln, bias=bias, res=residual, u_dtype=dtype)
            else:
                out = _enc.gemm(o, w_out, bias=bias, res=residual, out_dtype=torch.float32)
                u, _ = _enc.layernorm(out, *post_ln, out1_dtype=dtype)
            return out, probs, u
        out = _enc.gemm(o, w_out, bias=bias, res=residual, out_dtype=torch.float32)
        return out, probs

    def train_attend(self, x2d, B, T, pos, kpm_u8, dtype, residual=None, am=None):
        """Differentiable attention block (training path): x2d (B*T, d) →
        (residual + out_proj(attn(x2d)) fp32, attention probabilities after dropout)."""
        qkv = A.linear(x2d, self.in_proj_weight, self.in_proj_bias(), dtype, self._wc, "t_in", out_dtype=dtype)
        pk = A.linear(pos.reshape(-1, self.embed_dim), self.linear_pos.weight, None, dtype, self._wc, "t_pos",
                      out_dtype=dtype)
        p = self.dropout_att.p if self.training else 0.0
        o, attn = A.RelPosAttentionFn.apply(qkv, pk, self.pos_bias_u, self.pos_bias_v, kpm_u8, B, T,
                                            self.num_heads, self.head_dim, self.scale, float(p), am)
        out = A.linear(o, self.out_proj.weight, self.out_proj.bias, dtype, self._wc, "t_out", res=residual)
        return out, attn

    def cross_forward(self, query, key, value, pos_embs, key_padding_mask=None, attn_mask=None, self_att=False):
        """attention.py:554-639 for query != key / value: separate q / k / v
        projections on the MFMA GEMM (the row chunks of in_proj_weight,
        :555-564; vbias as the v projection's bias, :576-579), linear_pos, the
        cross-length rel-pos core (csrc/xattn.hip: rel_shift of the
        (q_len, 2*k_len-1) band incl. mask_pos_future) and out_proj, each
        differentiable.  self_att: the self-attention projection layout
        instead (:546-553: in_proj rows per head [q_h | k_h | v_h]), for
        heads wider than the fused kernels take.  Returns (out (B, Lq, E),
        attention weights)."""
        B, Lq, E = query.shape
        Lk = key.shape[1]
        if value.shape[:2] != key.shape[:2]:
            raise ValueError(f"key {tuple(key.shape)} and value {tuple(value.shape)} lengths differ")
        dtype = _enc.compute_dtype()
        H, dh = self.num_heads, self.head_dim
        if self_att:
            w3 = self.in_proj_weight.view(H, 3, dh, E)
            wq, wk, wv = (w3[:, i].reshape(H * dh, E) for i in range(3))
        else:
            wq, wk, wv = self.in_proj_weight.chunk(3, dim=0)
        vb = self.value_bias_weight if self.vbias is not None else None
        if self_att:
            # kernel copies of the per-head slices, cached against in_proj_weight
            # itself (the slices are fresh tensors every call)
            def lin(x, i, w, b):
                wk_ = self._wc.get(("s", i, dtype), [self.in_proj_weight],
                                   lambda: A.kernel_weight(w.detach().contiguous(), dtype, _enc.WeightCache(), "k"))
                return A.LinearFn.apply(A.to_dtype(x, dtype), w, b, wk_, dtype, None, 1.0, None)
            q = lin(query.reshape(B * Lq, E), 0, wq, None)
            k = lin(key.reshape(B * Lk, E), 1, wk, None)
            v = lin(value.reshape(B * Lk, E), 2, wv, vb)
        else:
            q = A.linear(query.reshape(B * Lq, E), wq, None, dtype, self._wc, "x_q", out_dtype=dtype)
            k = A.linear(key.reshape(B * Lk, E), wk, None, dtype, self._wc, "x_k", out_dtype=dtype)
            v = A.linear(value.reshape(B * Lk, E), wv, vb, dtype, self._wc, "x_v", out_dtype=dtype)
        pk = A.linear(pos_embs.reshape(-1, E), self.linear_pos.weight, None, dtype, self._wc, "x_pos",
                      out_dtype=dtype)
        kpm = key_padding_mask.to(query.device, torch.uint8).contiguous() if key_padding_mask is not None else None
        am = _enc.attn_mask_arg(attn_mask, B, Lq, H, query.device, Lk=Lk)
        p = self.dropout_att.p if self.training else 0.0
        o, attn = A.RelPosCrossAttnFn.apply(q, k, v, pk, self.pos_bias_u, self.pos_bias_v, kpm, am, B, Lq, Lk, H, dh,
                                            self.scale, bool(self.mask_pos_future), float(p))
        out = A.linear(o, self.out_proj.weight, self.out_proj.bias, dtype, self._wc, "x_out")
        if p == 0:
            attn = attn.clone()  # without dropout the weights are the softmax saved for backward: the caller's copy
        return out.view(B, Lq, E), attn

    def forward(self, query, key, value, pos_embs, key_padding_mask=None, attn_mask=None,
                return_attn_weights=True):
        """attention.py:485-639.  Self-attention (query, key and value
        identical, every Conformer call site) runs the fused kernels;
        anything else — key or value != query, q_len != k_len, or heads
        wider than FUSED_DH_MAX — takes cross_forward.  attn_mask: (Lq, Lk) or (B*H, Lq, Lk), bool (True =
        masked) or additive float (:598-611)."""
        if not self._qkv_same_embed_dim:
            raise NotImplementedError  # the reference raises too (attention.py:566)
        same = ((query is key or (query.shape == key.shape and torch.equal(query, key)))
                and (key is value or (key.shape == value.shape and torch.equal(key, value))))
        if not same or self.head_dim > FUSED_DH_MAX:
            out, attn = self.cross_forward(query, key, value, pos_embs, key_padding_mask, attn_mask, self_att=same)
            return (out, attn) if return_attn_weights else out
        B, T, d = query.shape
        dtype = _enc.compute_dtype()
        x2d = query.reshape(B * T, d)
        kpm = key_padding_mask.to(torch.uint8).contiguous() if key_padding_mask is not None else None
        am = _enc.attn_mask_arg(attn_mask, B, T, self.num_heads, query.device)
        if A.needs_grad(self, query) or (self.training and self.dropout > 0):
            out, attn = self.train_attend(x2d.float(), B, T, pos_embs.float(), kpm, dtype, am=am)
        else:
            x2d = _enc.to_compute(x2d, dtype)
            out, attn = self.attend(x2d, B, T, pos_embs, kpm, dtype, return_attn_weights, am=am)
        out = out.view(B, T, d)
        if return_attn_weights:
            return out, attn
        return out


class PositionalwiseFeedForward(nn.Module):
    """attention.py:781-839: Linear → activation → Dropout → Linear, the
    activation fused into the first GEMM's epilogue."""

    _deff = None  # zero-padded shadow copies (Conformer._PaddedEncoder): LN statistics over this many columns

    def __init__(self, d_ffn, input_shape=None, input_size=None, dropout=0.0, activation=nn.ReLU):
        super().__init__()
        if input_shape is None and input_size is None:
            raise ValueError("Expected one of input_shape or input_size")
        if input_size is None:
            input_size = input_shape[-1]
        self.ffn = nn.Sequential(nn.Linear(input_size, d_ffn), activation(), nn.Dropout(dropout),
                                 nn.Linear(d_ffn, input_size))
        self._wc = _enc.WeightCache()

    def act_name(self):
        a = self.ffn[1]
        if isinstance(a, Swish) or type(a).__name__ == "Swish":
            if getattr(a, "beta", 1) != 1:
                raise NotImplementedError("Swish(beta != 1) is not fused")
            return "swish", 0.0
        if isinstance(a, nn.ReLU):
            return "relu", 0.0
        if isinstance(a, nn.LeakyReLU):
            return "leaky_relu", a.negative_slope
        if isinstance(a, nn.GELU):
            return "gelu", 0.0
        raise NotImplementedError(f"activation {type(a).__name__} is not fused")

    def kernel_weights(self, dtype):
        ps = [self.ffn[0].weight, self.ffn[3].weight]
        if dtype == torch.float32:
            return tuple(p.detach() for p in ps)
        return self._wc.get("bf16", ps, lambda: tuple(_enc.cast_bf16(p.detach().contiguous()) for p in ps))

    def run(self, u2d, dtype, residual=None, alpha=1.0):
        """u2d (M, d) in dtype → residual + alpha * FFN(u2d) (fp32)."""
        w1, w2 = self.kernel_weights(dtype)
        act, slope = self.act_name()
        h = _enc.gemm(u2d, w1, bias=self.ffn[0].bias.detach(), act=act, slope=slope, out_dtype=dtype)
        return _enc.gemm(h, w2, bias=self.ffn[3].bias.detach(), res=residual, alpha=alpha, out_dtype=torch.float32)

    def train_run(self, u2d, dtype, residual=None, alpha=1.0, out_p=0.0):
        """Differentiable FFN (training path): residual + alpha * Dropout(out_p)(FFN(u2d))."""
        act, slope = self.act_name()
        if act == "relu":
            act, slope = "leaky_relu", 0.0  # ReLU = LeakyReLU(0), same backward
        if act not in ("swish", "leaky_relu", "gelu"):
            raise NotImplementedError(f"activation {act} has no backward kernel yet")
        l1, l2 = self.ffn[0], self.ffn[3]
        h = A.linear(u2d, l1.weight, l1.bias, dtype, self._wc, "t1", out_dtype=dtype)
        h = A.act(h, act, slope)
        h = A.dropout(h, self.ffn[2].p, self.training)
        if out_p == 0:
            return A.linear(h, l2.weight, l2.bias, dtype, self._wc, "t2", res=residual, alpha=alpha)
        y = A.linear(h, l2.weight, l2.bias, dtype, self._wc, "t2")
        return A.DropAddFn.apply(y, residual, float(alpha), None, float(out_p), torch.float32)

    def fusable(self, dtype):
        """True when the whole LN→FFN→residual block can run as one kernel."""
        return (dtype == torch.bfloat16 and self.act_name()[0] != "glu"
                and _enc.ffn_supported(self.ffn[0].in_features, self.ffn[0].out_features))

    def run_fused(self, x, ln0, alpha, post_ln=None, next_ln=None, next_dtype=torch.bfloat16, out=None):
        """x (M, d) fp32 → (post_ln(x + alpha * FFN(LN0(x))), next_ln(...) or None),
        one kernel (bf16 MFMA, hidden activation kept on chip)."""
        w1, w2 = self.kernel_weights(torch.bfloat16)
        act, slope = self.act_name()
        b1, b2 = (lin.bias.detach() if lin.bias is not None else torch.zeros(lin.out_features, device=x.device)
                  for lin in (self.ffn[0], self.ffn[3]))
        return _enc.ffn(x, ln0, w1, b1, act, slope, w2, b2, alpha,
                        post_ln=post_ln, next_ln=next_ln, next_dtype=next_dtype, out=out, deff=self._deff)

    def chain_block(self, ln0, alpha, post_ln=None):
        """This block's parameters for _enc.ffn_chain: (ln0, w1, b1, w2, b2,
        alpha, post_ln) in the fused kernel's formats."""
        w1, w2 = self.kernel_weights(torch.bfloat16)
        b1, b2 = (lin.bias.detach() if lin.bias is not None else torch.zeros(lin.out_features, device=w1.device)
                  for lin in (self.ffn[0], self.ffn[3]))
        return (ln0, w1, b1, w2, b2, alpha, post_ln)

    def run_fused_proj(self, x, ln0, alpha, next_ln, wp, post_ln=None):
        """run_fused with the next block's input projection on chip: returns
        (out fp32, next_ln(out) · wp^T bf16)."""
        w1, w2 = self.kernel_weights(torch.bfloat16)
        act, slope = self.act_name()
        b1, b2 = (lin.bias.detach() if lin.bias is not None else torch.zeros(lin.out_features, device=x.device)
                  for lin in (self.ffn[0], self.ffn[3]))
        return _enc.ffn_proj(x, ln0, w1, b1, act, slope, w2, b2, alpha, next_ln, wp, post_ln=post_ln,
                             deff=self._deff)

    def forward(self, x):
        shp = x.shape
        dtype = _enc.compute_dtype()
        u = x.reshape(-1, shp[-1])
        if A.needs_grad(self, x) or (self.training and self.ffn[2].p > 0):
            return self.train_run(A.to_dtype(u, dtype), dtype).view(*shp[:-1], -1)
        u = _enc.to_compute(u, dtype)
        return self.run(u, dtype).view(*shp[:-1], -1)


class MultiheadAttention(nn.Module):
    """attention.py:642-778: the wrapper of torch.nn.MultiheadAttention
    (state_dict keys att.in_proj_weight / att.in_proj_bias /
    att.out_proj.{weight,bias}, or att.{q,k,v}_proj_weight with kdim / vdim).
    Inference self-attention without attn_mask (query is key is value, the
    TransformerEncoderLayer case) runs as one in_proj GEMM (rows permuted per
    head to [q_h | k_h | v_h]) → the fused attention kernel (scores·1/√d_head,
    key padding mask, softmax, P·V) → out_proj GEMM.  Everything else —
    cross-attention (key / value ≠ query, S ≠ L), attn_mask (2-D or
    (B·H, L, S), bool / byte / additive), pos_embs (added to attn_mask,
    :756-761), a float key_padding_mask, training with attention dropout, or
    gradients — runs the differentiable path: q / k / v projections on the
    MFMA GEMM, the attention core of csrc/xattn.hip (its positional band and
    biases zero), out_proj.  Returns (output (B, L, E), head-averaged
    weights (B, L, S)) like the reference."""

    def __init__(self, nhead, d_model, dropout=0.0, bias=True, add_bias_kv=False, add_zero_attn=False, kdim=None,
                 vdim=None):
        super().__init__()
        self.att = nn.MultiheadAttention(embed_dim=d_model, num_heads=nhead, dropout=dropout, bias=bias,
                                         add_bias_kv=add_bias_kv, add_zero_attn=add_zero_attn, kdim=kdim, vdim=vdim)
        self.nhead = nhead
        self.d_model = d_model
        self._wc = _enc.WeightCache()
        self._zeros = {}

    def _check(self):
        a = self.att
        if not a._qkv_same_embed_dim or a.bias_k is not None or a.add_zero_attn or a.in_proj_bias is None:
            raise NotImplementedError("MultiheadAttention: only the default projection layout (bias, no bias_kv, "
                                      "no zero_attn, kdim = vdim = d_model) is on the HIP path")

    def qkv_weights(self, mode):
        """in_proj rows permuted to the kernel's per-head [q_h | k_h | v_h]
        layout, in the compute mode (torch.float32 | torch.bfloat16 | "mx");
        returns (weight, bias fp32)."""
        a = self.att
        ps = [a.in_proj_weight, a.in_proj_bias]

        def make():
            E, H = self.d_model, self.nhead
            dh = E // H
            idx = torch.arange(3 * E, device=a.in_proj_weight.device).view(3, H, dh).transpose(0, 1).reshape(-1)
            w = a.in_proj_weight.detach()[idx].contiguous()
            b = a.in_proj_bias.detach()[idx].contiguous().float()
            return _mode_weight(w, mode), b
        return self._wc.get(("qkv", str(mode)), ps, make)

    def out_weights(self, mode):
        w = self.att.out_proj.weight
        return self._wc.get(("out", str(mode)), [w], lambda: _mode_weight(w.detach().contiguous(), mode))

    def zero_band(self, T, dev, dtype):
        """(2T-1, E) zeros for the positional term + zero u/v biases (H, dh)."""
        key = (T, str(dev), dtype)
        z = self._zeros.get(key)
        if z is None:
            E, H = self.d_model, self.nhead
            z = (torch.zeros(2 * T - 1, E, device=dev, dtype=dtype), torch.zeros(E // H, H, device=dev))
            self._zeros = {key: z}
        return z

    def attend(self, qkv, B, T, kpm_u8, need_weights):
        """qkv (B*T, 3E) per-head layout (bf16 or fp32) → (o (B*T, E), probs (B, H, T, T) or None)."""
        E, H = self.d_model, self.nhead
        dh = E // H
        if not need_weights and _enc.mha_fast_ok(qkv, T, dh):
            # band-free kernel: no zero positional band through the MFMAs
            return _enc.mha_attention(qkv, kpm_u8, B, T, H, dh, 1.0 / math.sqrt(dh)), None
        band, zb = self.zero_band(T, qkv.device, qkv.dtype)
        return _enc.relpos_attention(qkv, band, zb, zb, kpm_u8, B, T, H, dh, 1.0 / math.sqrt(dh),
                                     need_probs=need_weights)

    def general_forward(self, query, key, value, attn_mask=None, key_padding_mask=None, pos_embs=None):
        """The differentiable path (see the class docstring).  Returns
        (out (B, L, E), weights (B, L, S) averaged over heads)."""
        a = self.att
        if a.bias_k is not None or a.add_zero_attn:
            raise NotImplementedError("MultiheadAttention: add_bias_kv / add_zero_attn are not on the HIP path")
        B, L, E = query.shape
        S = key.shape[1]
        if value.shape[:2] != key.shape[:2]:
            raise ValueError(f"key {tuple(key.shape)} and value {tuple(value.shape)} lengths differ")
        H = self.nhead
        dh = E // H
        dtype = _enc.compute_dtype()
        if a._qkv_same_embed_dim:
            wq, wk, wv = a.in_proj_weight.chunk(3, dim=0)
        else:
            wq, wk, wv = a.q_proj_weight, a.k_proj_weight, a.v_proj_weight
        bq = bk = bv = None
        if a.in_proj_bias is not None:
            bq, bk, bv = a.in_proj_bias.chunk(3, dim=0)
        q = A.linear(query.reshape(B * L, -1), wq, bq, dtype, self._wc, "g_q", out_dtype=dtype)
        k = A.linear(key.reshape(B * S, -1), wk, bk, dtype, self._wc, "g_k", out_dtype=dtype)
        v = A.linear(value.reshape(B * S, -1), wv, bv, dtype, self._wc, "g_v", out_dtype=dtype)
        # attn_mask (+ pos_embs) and a float key padding mask as one additive
        # fp32 mask; bool / byte masks: True (non-zero) = masked
        if pos_embs is not None:
            # attention.py:756-761, in place on the caller's mask as there (a
            # mask shared by a stack of layers accumulates every layer's add;
            # a bool / byte mask raises, as in the reference)
            if attn_mask is not None:
                attn_mask += pos_embs
            else:
                attn_mask = pos_embs
        m = attn_mask
        if m is not None and m.dim() == 3 and m.shape[-1] == 1:
            m = m.reshape(m.shape[0], m.shape[1])  # (L, S, 1) pos_embs
        if m is not None and m.dtype == torch.uint8:
            m = m.bool()
        kpm = None
        if key_padding_mask is not None:
            if key_padding_mask.dtype in (torch.bool, torch.uint8):
                kpm = key_padding_mask.to(query.device, torch.uint8).contiguous()
            else:  # additive (B, S): folded into a (B*H, L, S) mask
                add = key_padding_mask.to(query.device, torch.float32).view(B, 1, 1, S).expand(B, H, L, S)
                if m is None:
                    m = add.reshape(B * H, L, S)
                else:
                    mf = (torch.zeros(m.shape, device=query.device).masked_fill(m.to(query.device), -float("inf"))
                          if m.dtype == torch.bool else m.to(query.device, torch.float32))
                    mf = mf.view(1, 1, L, S) if mf.dim() == 2 else mf.view(-1, H, L, S)
                    m = (mf + add).reshape(B * H, L, S)
        am = _enc.attn_mask_arg(m, B, L, H, query.device, Lk=S)
        p = a.dropout if self.training else 0.0
        # the xattn core without a positional band: plain scaled dot-product attention
        o, attn = A.RelPosCrossAttnFn.apply(q, k, v, None, None, None, kpm, am, B, L, S, H, dh, 1.0 / math.sqrt(dh),
                                            False, float(p))
        out = A.linear(o, a.out_proj.weight, a.out_proj.bias, dtype, self._wc, "g_out")
        return out.view(B, L, E), attn.mean(dim=1)

    def forward(self, query, key, value, attn_mask=None, key_padding_mask=None, return_attn_weights=True,
                pos_embs=None):
        fast = (query is key and key is value and attn_mask is None and pos_embs is None
                and (key_padding_mask is None or key_padding_mask.dtype in (torch.bool, torch.uint8))
                and not A.needs_grad(self, query) and not (self.training and self.att.dropout > 0)
                and self.att._qkv_same_embed_dim and self.att.bias_k is None and not self.att.add_zero_attn
                and self.att.in_proj_bias is not None and self.d_model // self.nhead <= FUSED_DH_MAX)
        if not fast:
            out, w = self.general_forward(query, key, value, attn_mask, key_padding_mask, pos_embs)
            return (out, w) if return_attn_weights else out
        self._check()
        B, T, E = query.shape
        mode = _enc.compute_dtype()
        x2d = _enc.to_compute(query.reshape(B * T, E), mode)
        w_in, b_in = self.qkv_weights(mode)
        qkv = _enc.gemm(x2d, w_in, bias=b_in, out_dtype=mode)
        kpm = key_padding_mask.to(torch.uint8).contiguous() if key_padding_mask is not None else None
        o, probs = self.attend(qkv, B, T, kpm, bool(return_attn_weights))
        out = _enc.gemm(o, self.out_weights(mode), bias=self.att.out_proj.bias.detach().float(),
                        out_dtype=torch.float32).view(B, T, E)
        if return_attn_weights:
            return out, probs.mean(dim=1)
        return out


def _mode_weight(w, mode):
    """A weight in compute mode: fp32 as is, bf16 cast, or "mx" (MXFP8 q, scales)."""
    if mode == "mx":
        from .. import _w2v
        return _w2v.mx_quant(w.float().contiguous())
    if mode == torch.bfloat16:
        return _enc.cast_bf16(w.float().contiguous())
    return w.float().contiguous()
