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
from torch.nn import Module

from ..._lib import check, custom_op, lib, ptr, require_device, stream_of

_RED = {"mean": 0, "sum": 1, "none": 2}


@custom_op("sbk::rnnt", mutates_args=())
def rnnt(x: torch.Tensor, labels: torch.Tensor, Tl: torch.Tensor, Ul: torch.Tensor, blank: int, reduction: int,
         is_logits: bool, loss_mode: int) -> tuple[torch.Tensor, torch.Tensor]:
    """Forward kernels (gather [+ fused log-softmax], α/β lattice, sparse
    grads, reduction).  Returns (loss: () for mean/sum, (B,) for none;
    workspace kept for the backward)."""
    B, maxT, U1, V = x.shape
    L = lib()
    ws = torch.empty(int(L.sbk_rnnt_workspace_floats(B, maxT, U1)), device=x.device, dtype=torch.float32)
    out = torch.empty(B if reduction == 2 else (), device=x.device, dtype=torch.float32)
    check(L.sbk_rnnt_forward(ptr(x), ptr(labels), ptr(Tl), ptr(Ul), B, maxT, U1, V, int(blank), int(is_logits),
                             int(loss_mode), int(reduction), ptr(ws), ptr(out), stream_of(x)), "sbk_rnnt_forward")
    return out, ws


@rnnt.register_fake
def _(x, labels, Tl, Ul, blank, reduction, is_logits, loss_mode):
    B, maxT, U1, _ = x.shape
    return (x.new_empty(B if reduction == 2 else ()), x.new_empty(7 * B * maxT * U1 + 2 * B))


@custom_op("sbk::rnnt_grad", mutates_args=())
def rnnt_grad(x: torch.Tensor, labels: torch.Tensor, ws: torch.Tensor, go: torch.Tensor, blank: int,
              mode: int) -> torch.Tensor:
    """Dense (B, T, U1, V) gradient: mode 0 wrt log-probs, 1 wrt logits
    (through the log-softmax); rows scaled by go (one value or one per b)."""
    B, maxT, U1, V = x.shape
    grad = torch.empty_like(x)
    check(lib().sbk_rnnt_backward(ptr(x), ptr(labels), B, maxT, U1, V, blank, mode, ptr(ws), ptr(go),
                                  int(go.numel() > 1), ptr(grad), stream_of(x)), "sbk_rnnt_backward")
    return grad


@rnnt_grad.register_fake
def _(x, labels, ws, go, blank, mode):
    return torch.empty_like(x)


def _rnnt_setup(ctx, inputs, output):
    x, labels, _, _, blank, reduction, is_logits, loss_mode = inputs
    ctx.save_for_backward(x, labels, output[1])
    ctx.blank = blank
    ctx.mode = int(is_logits)
    # standard (torchaudio) semantics: d(mean)/d(loss_b) = 1/B; the Numba
    # semantics multiply by grad_output only (transducer_loss.py:289-293)
    ctx.scale = 1.0 / x.shape[0] if (loss_mode == 1 and reduction == 0) else 1.0


def _rnnt_backward(ctx, grad_loss, grad_ws):
    x, labels, ws = ctx.saved_tensors
    go = (grad_loss.detach().to(torch.float32).reshape(-1) * ctx.scale).contiguous()
    return rnnt_grad(x, labels, ws, go, ctx.blank, ctx.mode), None, None, None, None, None, None, None


rnnt.register_autograd(_rnnt_backward, setup_context=_rnnt_setup)


def rnnt_loss(x, labels, T, U, blank, reduction, is_logits, loss_mode):
    if reduction not in _RED:
        raise Exception("Unexpected reduction {}".format(reduction))
    require_device(x, labels)
    if x.dtype != torch.float32:
        raise TypeError("transducer loss kernels take fp32 logits / log-probs")
    x = x.contiguous()
    B, maxT, U1, V = x.shape
    lab = labels.to(device=x.device, dtype=torch.int32)
    if lab.shape[1] < U1 - 1:
        lab = torch.nn.functional.pad(lab, (0, U1 - 1 - lab.shape[1]))
    lab = lab[:, : U1 - 1].contiguous()
    Tl = torch.as_tensor(T).to(device=x.device, dtype=torch.int32).contiguous()
    Ul = torch.as_tensor(U).to(device=x.device, dtype=torch.int32).contiguous()
    return rnnt(x, lab, Tl, Ul, int(blank), _RED[reduction], bool(is_logits), int(loss_mode))[0]


class Transducer:
    """Transducer.apply(log_probs, labels, T, U, blank, reduction)
    (transducer_loss.py:239-293): log_probs (B, maxT, maxU+1, V).  The
    autograd.Function of the reference is the sbk::rnnt custom op's
    registered autograd here (traceable, capturable)."""

    @staticmethod
    def apply(log_probs, labels, T, U, blank, reduction):
        return rnnt_loss(log_probs, labels, T, U, blank, reduction, is_logits=False, loss_mode=0)


class TransducerLogits:
    """Fused log_softmax + Transducer (losses.py:79-85): the gradient wrt the
    logits is g - softmax·Σg in one pass, no (B,T,U,V) log-prob tensor."""

    @staticmethod
    def apply(logits, labels, T, U, blank, reduction, loss_mode=0):
        return rnnt_loss(logits, labels, T, U, blank, reduction, is_logits=True, loss_mode=loss_mode)


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
