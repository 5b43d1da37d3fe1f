"""Drop-in for speechbrain.nnet.loss.transducer_loss (Transducer,
TransducerLoss; transducer_loss.py:239-351) on HIP kernels
(speechbrain_amd/csrc/rnnt.hip) instead of Numba CUDA.

Semantics kept from the reference:
  * loss per utterance = -(α[T-1,U] + lp[T-1,U,∅]) / T (time-normalised);
    reductions mean | sum | none, anything else raises Exception;
  * gradients are the UN-normalised ∂(-log P)/∂lp, multiplied by
    grad_output in backward (so "mean" does not divide by B).
Deviation: the reference TransducerLoss.forward compares torch.device
objects with the string "cuda" and therefore always raises ValueError; this
module accepts ROCm tensors (and raises for CPU tensors: no CPU fallback).
"""
import torch
from torch.autograd import Function
from torch.nn import Module

from ..._lib import check, lib, ptr, require_device, stream_of

_RED = {"mean": 0, "sum": 1, "none": 2}


def _prep(x, labels, T, U):
    require_device(x, labels)
    if x.dtype != torch.float32:
        raise TypeError("transducer loss kernels take fp32 logits / log-probs")
    x = x.detach().contiguous()
    B, maxT, U1, V = x.shape
    lab = labels.to(device=x.device, dtype=torch.int32)
    if lab.shape[1] < U1 - 1:
        lab = torch.nn.functional.pad(lab, (0, U1 - 1 - lab.shape[1]))
    lab = lab[:, : U1 - 1].contiguous()
    Tl = torch.as_tensor(T).to(device=x.device, dtype=torch.int32).contiguous()
    Ul = torch.as_tensor(U).to(device=x.device, dtype=torch.int32).contiguous()
    return x, lab, Tl, Ul, B, maxT, U1, V


def rnnt_forward(x, labels, T, U, blank, reduction, is_logits, loss_mode):
    """Runs the forward kernels; returns (loss, ctx tuple for the backward)."""
    if reduction not in _RED:
        raise Exception("Unexpected reduction {}".format(reduction))
    x, lab, Tl, Ul, B, maxT, U1, V = _prep(x, labels, T, U)
    L = lib()
    ws = torch.empty(int(L.sbk_rnnt_workspace_floats(B, maxT, U1)), device=x.device, dtype=torch.float32)
    out = torch.empty(B if reduction == "none" else 1, device=x.device, dtype=torch.float32)
    check(L.sbk_rnnt_forward(ptr(x), ptr(lab), ptr(Tl), ptr(Ul), B, maxT, U1, V, int(blank), int(is_logits),
                             int(loss_mode), _RED[reduction], ptr(ws), ptr(out), stream_of(x)), "sbk_rnnt_forward")
    loss = out if reduction == "none" else out[0]
    return loss, (x, lab, ws, B, maxT, U1, V, int(blank))


def rnnt_backward(saved, grad_output, mode, extra_scale=1.0):
    x, lab, ws, B, maxT, U1, V, blank = saved
    go = grad_output.detach().to(device=x.device, dtype=torch.float32).reshape(-1) * extra_scale
    per_b = int(go.numel() > 1)
    go = go.contiguous()
    grad = torch.empty_like(x)
    check(lib().sbk_rnnt_backward(ptr(x), ptr(lab), B, maxT, U1, V, blank, mode, ptr(ws), ptr(go), per_b,
                                  ptr(grad), stream_of(x)), "sbk_rnnt_backward")
    return grad


class Transducer(Function):
    """Transducer.apply(log_probs, labels, T, U, blank, reduction)
    (transducer_loss.py:239-293): log_probs (B, maxT, maxU+1, V)."""

    @staticmethod
    def forward(ctx, log_probs, labels, T, U, blank, reduction):
        loss, saved = rnnt_forward(log_probs, labels, T, U, blank, reduction, is_logits=0, loss_mode=0)
        ctx.saved = saved
        return loss

    @staticmethod
    def backward(ctx, grad_output):
        return rnnt_backward(ctx.saved, grad_output, mode=0), None, None, None, None, None


class TransducerLogits(Function):
    """Fused log_softmax + Transducer (losses.py:79-85): the gradient wrt the
    logits is g - softmax·Σg in one pass, no (B,T,U,V) log-prob tensor."""

    @staticmethod
    def forward(ctx, logits, labels, T, U, blank, reduction, loss_mode=0):
        loss, saved = rnnt_forward(logits, labels, T, U, blank, reduction, is_logits=1, loss_mode=loss_mode)
        ctx.saved = saved
        ctx.scale = 1.0
        if loss_mode == 1 and reduction == "mean":
            ctx.scale = 1.0 / saved[3]  # standard semantics: d(mean)/d(loss_b) = 1/B
        return loss

    @staticmethod
    def backward(ctx, grad_output):
        return rnnt_backward(ctx.saved, grad_output, mode=1, extra_scale=ctx.scale), None, None, None, None, None, None


class TransducerLoss(Module):
    """transducer_loss.py:296-351."""

    def __init__(self, blank=0, reduction="mean"):
        super().__init__()
        self.blank = blank
        self.reduction = reduction
        self.loss = Transducer.apply

    def forward(self, logits, labels, T, U):
        for t in (logits, labels, T, U):
            if not (isinstance(t, torch.Tensor) and t.device.type == "cuda"):
                raise ValueError(f"Found inputs tensors to be on {[logits.device, labels.device, T.device, U.device]}"
                                 " while needed to be on a 'cuda' device to use the transducer loss.")
        return TransducerLogits.apply(logits, labels, T, U, self.blank, self.reduction, 0)
