"""Fused transducer head: joint → output projection →
log-softmax → RNN-T loss without the (B, T, U+1, V) logits.

The LibriSpeech transducer recipe computes

    z      = Transducer_joint(tn.unsqueeze(2), pn.unsqueeze(1))   # (B, T, U+1, J)
    logits = transducer_lin(z)                                    # (B, T, U+1, V)
    loss   = transducer_loss(logits, targets, wav_lens, token_lens, blank)

(speechbrain/nnet/transducer/transducer_joint.py:57-95, speechbrain/nnet/
losses.py:27-85, speechbrain/nnet/loss/transducer_loss.py:31-293).  At config
4 (B=32, T=376, U+1=65, V=1000) the fp32 logits and their gradient are
3.13 GB each.  `transducer_head_loss(tn, pn, weight, ...)` computes the same
loss and the gradients wrt tn, pn and weight from csrc/thead.hip:

  forward   sbk_thead_fwd      z generated on chip, S = z·Wᵀ (bf16 MFMA,
                               fp32), online log-sum-exp, blank / label
                               log-probs  →  sbk_rnnt_lattice (α, β, loss)
  backward  sbk_thead_dlogits  S recomputed → dS = ∂L/∂logits in bf16
            sbk_gemm           dZ = dS·W
            sbk_joint_bwd      dTN (sum over U), dPN (sum over T)
            sbk_thead_wgrad    dW = dSᵀ·z (z regenerated)

so the only (rows × V) tensor is the transient bf16 dS of the backward.
Numerics: the bf16-autocast recipe's (z and W in bf16, fp32 accumulation);
the logits are not rounded to bf16 before the log-softmax.  Without bf16
autocast (the fp32 compute dtype) the head runs the materialised chain on
the fp32 kernels instead — sbk_joint_fwd → exact-f32 MFMA Linear → the HIP
RNN-T loss — so an fp32 step never computes in bf16 behind the caller's back.
"""
import torch
import torch.nn as nn

from ... import _autograd as A
from ... import _enc
from ..._lib import check, custom_op, lib, ptr, require_device, stream_of
from ..linear import Linear

__all__ = ["transducer_head_loss", "TransducerHeadLinear"]

_RED = {"mean": 0, "sum": 1, "none": 2}
_ACT = {nn.Identity: 0, nn.LeakyReLU: 3, nn.ReLU: 6}  # (Tanh: the materialised Transducer_joint path)


def _padded_bf16(w):
    """(V, J) fp32 -> (Vp, J) bf16, rows >= V zero (the head's column tiles)."""
    V, J = w.shape
    Vp = int(lib().sbk_thead_vpad(V))
    out = torch.zeros(Vp, J, device=w.device, dtype=torch.bfloat16)
    out[:V] = _enc.cast_bf16(w)
    return out


@custom_op("sbk::thead_loss", mutates_args=())
def thead_loss(tn: torch.Tensor, pn: torch.Tensor, w: torch.Tensor, labels: torch.Tensor, Tl: torch.Tensor,
               Ul: torch.Tensor, blank: int, reduction: int, loss_mode: int, act: int,
               slope: float) -> tuple[torch.Tensor, torch.Tensor]:
    """tn (B, T, J), pn (B, U1, J), w (V, J) fp32 → (loss, RNN-T workspace)."""
    B, T, J = tn.shape
    U1, V = pn.shape[1], w.shape[0]
    L = lib()
    n = B * T * U1
    ws = torch.empty(int(L.sbk_rnnt_workspace_floats(B, T, U1)), device=tn.device, dtype=torch.float32)
    out = torch.empty(B if reduction == 2 else (), device=tn.device, dtype=torch.float32)
    wb = _padded_bf16(w)
    s = stream_of(tn)
    check(L.sbk_thead_fwd(ptr(tn), ptr(pn), ptr(wb), ptr(labels), B, T, U1, J, V, int(blank), int(act), float(slope),
                          ptr(ws[2 * n:]), ptr(ws), ptr(ws[n:]), s), "sbk_thead_fwd")
    check(L.sbk_rnnt_lattice(ptr(Tl), ptr(Ul), B, T, U1, int(loss_mode), int(reduction), ptr(ws), ptr(out), s),
          "sbk_rnnt_lattice")
    return out, ws


@thead_loss.register_fake
def _(tn, pn, w, labels, Tl, Ul, blank, reduction, loss_mode, act, slope):
    B, T, _ = tn.shape
    U1 = pn.shape[1]
    return tn.new_empty(B if reduction == 2 else ()), tn.new_empty(7 * B * T * U1 + 2 * B)


@custom_op("sbk::thead_grad", mutates_args=())
def thead_grad(tn: torch.Tensor, pn: torch.Tensor, w: torch.Tensor, labels: torch.Tensor, Tl: torch.Tensor,
               ws: torch.Tensor, go: torch.Tensor, blank: int, act: int,
               slope: float) -> tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
    """(dtn, dpn, dw) from the forward's workspace; rows scaled by go (one
    value, or one per utterance)."""
    B, T, J = tn.shape
    U1, V = pn.shape[1], w.shape[0]
    L = lib()
    n = B * T * U1
    Vp = int(L.sbk_thead_vpad(V))
    s = stream_of(tn)
    wb = _padded_bf16(w)
    ds = torch.empty(n, Vp, device=tn.device, dtype=torch.bfloat16)
    check(L.sbk_thead_dlogits(ptr(tn), ptr(pn), ptr(wb), ptr(labels), B, T, U1, J, V, int(blank), int(act),
                              float(slope), ptr(ws[2 * n:]), ptr(ws[5 * n:]), ptr(ws[6 * n:]), ptr(go),
                              int(go.numel() > 1), ptr(ds), s), "sbk_thead_dlogits")
    # dZ = dS · W: W^T zero-padded to Vp columns is the (N, K) operand
    dz = _enc.gemm(ds, wb.t().contiguous(), out_dtype=torch.bfloat16)
    dtn = torch.empty_like(tn)
    dpn = torch.empty_like(pn)
    jws = torch.empty(int(L.sbk_joint_bwd_workspace_floats(B, T, U1, J)), device=tn.device, dtype=torch.float32)
    check(L.sbk_joint_bwd(ptr(tn), ptr(pn), ptr(dz), 1, B, T, U1, J, int(act), float(slope), ptr(dtn), ptr(dpn),
                          ptr(jws), s), "sbk_joint_bwd")
    del dz
    dw = torch.zeros(V, J, device=tn.device, dtype=torch.float32)
    check(L.sbk_thead_wgrad(ptr(ds), ptr(tn), ptr(pn), ptr(Tl), B, T, U1, J, V, int(act), float(slope), ptr(dw), s),
          "sbk_thead_wgrad")
    return dtn, dpn, dw


@thead_grad.register_fake
def _(tn, pn, w, labels, Tl, ws, go, blank, act, slope):
    return torch.empty_like(tn), torch.empty_like(pn), torch.empty_like(w)


def _setup(ctx, inputs, output):
    tn, pn, w, labels, Tl, _, blank, reduction, loss_mode, act, slope = inputs
    ctx.save_for_backward(tn, pn, w, labels, Tl, output[1])
    ctx.a = (blank, act, slope)
    # torchaudio semantics: d(mean)/d(loss_b) = 1/B (as sbk::rnnt)
    ctx.scale = 1.0 / tn.shape[0] if (loss_mode == 1 and reduction == 0) else 1.0


def _backward(ctx, grad_loss, grad_ws):
    tn, pn, w, labels, Tl, ws = ctx.saved_tensors
    go = (grad_loss.detach().to(torch.float32).reshape(-1) * ctx.scale).contiguous()
    dtn, dpn, dw = thead_grad(tn, pn, w, labels, Tl, ws, go, *ctx.a)
    return dtn, dpn, dw, None, None, None, None, None, None, None, None


thead_loss.register_autograd(_backward, setup_context=_setup)


def _act_of(nonlinearity):
    code = _ACT.get(type(nonlinearity))
    if code is None:
        raise NotImplementedError(f"joint nonlinearity {type(nonlinearity).__name__} has no HIP kernel")
    slope = float(getattr(nonlinearity, "negative_slope", 0.0)) if code == 3 else 0.0
    if slope > 1.0:
        raise NotImplementedError("the fused head's kernels take LeakyReLU slopes <= 1")
    return code, slope


def transducer_head_loss(tn, pn, weight, targets, input_lens, target_lens, blank_index, reduction="mean",
                         use_torchaudio=True, nonlinearity=None):
    """transducer_loss(Linear(Transducer_joint(tn, pn), weight), targets, ...)
    (losses.py:27-85 semantics: relative lengths rounded against T and the
    target width; use_torchaudio selects -log P / mean over the batch) with
    the joint, projection and log-softmax fused.
    tn (B, T, J) or (B, T, 1, J); pn (B, U+1, J) or (B, 1, U+1, J); weight
    (V, J) — the bias-free output Linear's weight; nonlinearity the joint's
    module (default LeakyReLU, the recipe's)."""
    if reduction not in _RED:
        raise Exception("Unexpected reduction {}".format(reduction))
    if tn.dim() == 4:
        tn = tn[:, :, 0, :]
    if pn.dim() == 4:
        pn = pn[:, 0, :, :]
    require_device(tn, pn, weight, targets)
    act, slope = _act_of(nonlinearity if nonlinearity is not None else nn.LeakyReLU())
    if _enc.compute_dtype() == torch.float32:
        return _materialised_fp32(tn, pn, weight, targets, input_lens, target_lens, blank_index, reduction,
                                  use_torchaudio, act, slope)
    B, T, J = tn.shape
    U1 = pn.shape[1]
    in_lens = (input_lens * T).round().int()
    tg_lens = (target_lens * targets.shape[1]).round().int()
    lab = targets.to(device=tn.device, dtype=torch.int32)
    if lab.shape[1] < U1 - 1:
        lab = torch.nn.functional.pad(lab, (0, U1 - 1 - lab.shape[1]))
    lab = lab[:, : U1 - 1].contiguous()
    Tl = in_lens.to(device=tn.device, dtype=torch.int32).contiguous()
    Ul = tg_lens.to(device=tn.device, dtype=torch.int32).contiguous()
    out, _ = thead_loss(tn.float().contiguous(), pn.float().contiguous(), weight.float().contiguous(), lab, Tl, Ul,
                        int(blank_index), _RED[reduction], 1 if use_torchaudio else 0, act, slope)
    return out


def _materialised_fp32(tn, pn, weight, targets, input_lens, target_lens, blank_index, reduction, use_torchaudio,
                       act, slope):
    """fp32 compute dtype: Transducer_joint → Linear → transducer_loss as the
    recipe runs them (transducer_joint.py:57-95, linear.py:15-76,
    losses.py:27-85), every op an fp32 HIP kernel with its own backward."""
    from ..losses import transducer_loss
    B, T, J = tn.shape
    U1 = pn.shape[1]
    z = A.JointFn.apply(A.to_dtype(tn.float(), torch.float32), A.to_dtype(pn.float(), torch.float32), act, slope,
                        torch.float32)
    logits = A.LinearFn.apply(z.view(B * T * U1, J), weight, None, weight.detach().float().contiguous(),
                              torch.float32, None, 1.0, None)
    return transducer_loss(logits.view(B, T, U1, -1), targets, input_lens, target_lens, blank_index, reduction,
                           use_torchaudio=use_torchaudio)


class TransducerHeadLinear(Linear):
    """The recipe's output projection (speechbrain.nnet.linear.Linear,
    J -> V, bias=False; same constructor, state_dict keys `w.weight` and
    seeded init) whose forward also takes the joint inputs and returns the
    fused transducer loss:

        lin(z)                                        -> logits (as Linear)
        lin(tn, pn, targets, input_lens, target_lens) -> loss, no logits

    The loss goes through the module's own forward, so a DDP-wrapped head
    all-reduces its weight gradient like any other module."""

    def __init__(self, n_neurons, input_shape=None, input_size=None, bias=False, combine_dims=False,
                 nonlinearity=None, blank_index=0, reduction="mean", use_torchaudio=True):
        super().__init__(n_neurons, input_shape=input_shape, input_size=input_size, bias=bias,
                         combine_dims=combine_dims)
        self.nonlinearity = nonlinearity if nonlinearity is not None else nn.LeakyReLU()
        self.blank_index = blank_index
        self.reduction = reduction
        self.use_torchaudio = use_torchaudio

    def forward(self, x, pn=None, targets=None, input_lens=None, target_lens=None):
        if pn is None:
            return super().forward(x)
        if self.w.bias is not None:
            raise NotImplementedError("the fused head takes a bias-free output projection (the recipe's)")
        return transducer_head_loss(x, pn, self.w.weight, targets, input_lens, target_lens, self.blank_index,
                                    self.reduction, self.use_torchaudio, self.nonlinearity)
