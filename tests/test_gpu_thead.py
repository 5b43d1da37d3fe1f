"""Fused transducer head (csrc/thead.hip) vs the materialised chain and vs
the CPU RNN-T oracle (oracle/rnnt.py).  The fused kernels run under bf16
autocast (the recipe's precision); without autocast the head is the fp32
materialised chain on the exact-f32 kernels (test_head_fp32_is_materialised).

Reference path, at the same operand rounding (the bf16-autocast recipe: z and
W rounded to bf16, fp32 accumulation, fp32 logits): z = bf16(act(tn + pn)),
logits = z · bf16(W)ᵀ in fp32, then sbk::rnnt (TransducerLogits) — the HIP
loss pinned to the reference's known answer and the CPU oracle in
test_gpu_rnnt.py — with torch autograd for ∂/∂(tn, pn, W).
Tolerances: the loss differs only by fp32 summation order (1e-4 relative).
The fused backward rounds dS = ∂L/∂logits and dZ to bf16 (2^-9 relative
each) before the two gradient GEMMs, so gradients are compared normwise:
‖a − b‖ ≤ 1e-2 ‖b‖ (observed values printed)."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

import oracle.rnnt as OR

pytestmark = pytest.mark.gpu


def _materialised(tn, pn, w, targets, in_rel, tg_rel, blank, reduction, use_torchaudio, slope):
    from speechbrain_amd.nnet.losses import transducer_loss
    z = F.leaky_relu(tn.unsqueeze(2) + pn.unsqueeze(1), slope)
    z = z.to(torch.bfloat16).float()
    logits = z @ w.to(torch.bfloat16).float().t()
    return transducer_loss(logits, targets, in_rel, tg_rel, blank, reduction, use_torchaudio=use_torchaudio)


def _case(dev, B, T, U, J, V, seed):
    g = torch.Generator().manual_seed(seed)
    tn = torch.randn(B, T, J, generator=g)
    pn = torch.randn(B, U + 1, J, generator=g)
    w = torch.randn(V, J, generator=g) / J ** 0.5
    targets = torch.randint(1, V, (B, U), generator=g).int()
    Tb = torch.tensor([T - (3 * i) % max(T // 2, 1) for i in range(B)])
    Ub = torch.tensor([U - (2 * i) % max(U // 2, 1) for i in range(B)])
    return (tn.to(dev), pn.to(dev), w.to(dev), targets.to(dev), (Tb.float() / T).to(dev), (Ub.float() / U).to(dev))


def _nrel(a, b):
    return ((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-30)).item()


@pytest.mark.parametrize("B,T,U,J,V", [(3, 9, 5, 128, 70), (2, 40, 19, 1024, 1000), (4, 17, 64, 256, 129)])
@pytest.mark.parametrize("use_torchaudio,reduction", [(True, "mean"), (False, "mean"), (True, "none")])
def test_thead_vs_materialised(dev, B, T, U, J, V, use_torchaudio, reduction):
    from speechbrain_amd.nnet.loss.transducer_head import transducer_head_loss
    tn, pn, w, targets, in_rel, tg_rel = _case(dev, B, T, U, J, V, seed=B * 1000 + U)
    slope = 0.01
    leaves = [t.clone().requires_grad_() for t in (tn, pn, w)]
    ref = _materialised(*leaves, targets, in_rel, tg_rel, 0, reduction, use_torchaudio, slope)
    ref.sum().backward()
    fl = [t.clone().requires_grad_() for t in (tn, pn, w)]
    with torch.autocast("cuda", dtype=torch.bfloat16):
        out = transducer_head_loss(*fl, targets, in_rel, tg_rel, 0, reduction, use_torchaudio,
                                   torch.nn.LeakyReLU(slope))
    out.sum().backward()
    assert out.shape == ref.shape
    assert torch.allclose(out, ref, rtol=1e-4, atol=1e-5), (out, ref)
    for name, a, b in zip(("dtn", "dpn", "dW"), fl, leaves):
        e = _nrel(a.grad, b.grad)
        print(f"{name}: normwise rel err {e:.2e}")
        assert e <= 1e-2, f"{name}: {e}"


def test_thead_full_c4(dev):
    """Config-4 shapes (B=32, T=376, U+1=65, J=1024, V=1000): the loss and
    the gradients against the materialised path (3.1 GB of fp32 logits on
    the reference side; the fused side's largest tensor is the bf16 dS)."""
    from speechbrain_amd.nnet.loss.transducer_head import transducer_head_loss
    B, T, U, J, V = 32, 376, 64, 1024, 1000
    tn, pn, w, targets, in_rel, tg_rel = _case(dev, B, T, U, J, V, seed=7)
    tn, pn = tn * 0.5, pn * 0.5
    fl = [t.clone().requires_grad_() for t in (tn, pn, w)]
    torch.cuda.reset_peak_memory_stats(dev)
    base = torch.cuda.memory_allocated(dev)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        out = transducer_head_loss(*fl, targets, in_rel, tg_rel, 0, "mean", True)
    out.backward()
    peak_fused = torch.cuda.max_memory_allocated(dev) - base
    leaves = [t.clone().requires_grad_() for t in (tn, pn, w)]
    ref = _materialised(*leaves, targets, in_rel, tg_rel, 0, "mean", True, 0.01)
    ref.backward()
    assert torch.isfinite(out) and abs(out.item() - ref.item()) <= 1e-4 * abs(ref.item()), (out.item(), ref.item())
    for name, a, b in zip(("dtn", "dpn", "dW"), fl, leaves):
        e = _nrel(a.grad, b.grad)
        print(f"{name}: normwise rel err {e:.2e}")
        assert e <= 1e-2, f"{name}: {e}"
    rows = B * T * (U + 1)
    print(f"fused peak {peak_fused / 2**30:.2f} GiB vs fp32 logits alone {rows * V * 4 / 2**30:.2f} GiB")
    assert peak_fused < 2 * rows * V * 4


def test_head_linear_module(dev):
    """TransducerHeadLinear: forward(z) is the recipe's Linear; forward(tn,
    pn, targets, lens) is the fused loss, and seeded construction draws the
    same weights as Linear (checkpoint keys w.weight)."""
    from speechbrain_amd.nnet.linear import Linear
    from speechbrain_amd.nnet.loss.transducer_head import TransducerHeadLinear
    torch.manual_seed(3)
    ref = Linear(input_size=128, n_neurons=70, bias=False).to(dev)
    torch.manual_seed(3)
    head = TransducerHeadLinear(input_size=128, n_neurons=70, bias=False).to(dev)
    assert list(head.state_dict()) == list(ref.state_dict()) == ["w.weight"]
    assert torch.equal(head.w.weight, ref.w.weight)
    tn, pn, _, targets, in_rel, tg_rel = _case(dev, 3, 9, 5, 128, 70, seed=5)
    with torch.no_grad():
        z = F.leaky_relu(tn.unsqueeze(2) + pn.unsqueeze(1), 0.01)
        assert torch.equal(head(z), ref(z))
        with torch.autocast("cuda", dtype=torch.bfloat16):
            loss = head(tn, pn, targets, in_rel, tg_rel)
        want = _materialised(tn, pn, head.w.weight, targets, in_rel, tg_rel, 0, "mean", True, 0.01)
    assert torch.allclose(loss, want, rtol=1e-4, atol=1e-5), (loss, want)


def _oracle_head(tn, pn, w, targets, in_rel, tg_rel, blank, use_torchaudio, slope):
    """The recipe's head on the fused kernels' operand rounding — z =
    bf16(LeakyReLU(tn + pn)), logits = z · bf16(W)^T (float64) — then the RNN-T
    oracle (transducer_loss.py:31-236 restated, float64): per-utterance loss
    and d/d(logits) (log-softmax chained), then the chain rule to tn, pn, W
    in float64.  Returns (loss (mean reduction), dtn, dpn, dW)."""
    tn, pn, w = (t.detach().cpu().double() for t in (tn, pn, w))
    pre = tn[:, :, None, :] + pn[:, None, :, :]
    z = F.leaky_relu(pre, slope).to(torch.bfloat16).double()
    wb = w.to(torch.bfloat16).double()
    logits = (z @ wb.t()).numpy()
    tg = targets.cpu().numpy()
    loss_b, g = OR.transducer_loss(logits, tg, in_rel.cpu().numpy(), tg_rel.cpu().numpy(), blank, "none",
                                   dtype=np.float64)
    B, T = tn.shape[:2]
    Tabs = np.round(in_rel.cpu().numpy() * T).astype(np.int64)
    if use_torchaudio:  # -log P per utterance, mean over the batch, gradients / B
        loss = float((loss_b * Tabs).mean())
        g = g / B
    else:  # time-normalised loss, un-normalised gradients (the Numba quirks)
        loss = float(loss_b.mean())
    g = torch.from_numpy(g)
    dz = g @ wb
    da = dz * torch.where(pre >= 0, 1.0, slope)
    return loss, da.sum(2), da.sum(1), g.reshape(-1, g.shape[-1]).t() @ z.reshape(-1, z.shape[-1])


@pytest.mark.parametrize("B,T,U,J,V", [(2, 7, 4, 128, 37), (3, 11, 6, 256, 129)])
@pytest.mark.parametrize("use_torchaudio", [True, False])
def test_thead_vs_oracle_rnnt(dev, B, T, U, J, V, use_torchaudio):
    """transducer_head_loss (bf16 autocast: thead fwd / dlogits / wgrad
    kernels, the HIP lattice) against oracle/rnnt.py directly, not through
    the materialised HIP chain.  Loss: 1e-4 relative (fp32 summation order
    only).  Gradients: the fused backward rounds dS = dL/dlogits and dZ to
    bf16 (relative step 2^-8 each) before the two gradient GEMMs, so they are
    compared normwise at 1e-2 (observed values printed)."""
    from speechbrain_amd.nnet.loss.transducer_head import transducer_head_loss
    tn, pn, w, targets, in_rel, tg_rel = _case(dev, B, T, U, J, V, seed=B * 100 + U)
    slope = 0.01
    fl = [t.clone().requires_grad_() for t in (tn, pn, w)]
    with torch.autocast("cuda", dtype=torch.bfloat16):
        out = transducer_head_loss(*fl, targets, in_rel, tg_rel, 0, "mean", use_torchaudio,
                                   torch.nn.LeakyReLU(slope))
    out.backward()
    loss, dtn, dpn, dw = _oracle_head(tn, pn, w, targets, in_rel, tg_rel, 0, use_torchaudio, slope)
    assert abs(out.item() - loss) <= 1e-4 * abs(loss), (out.item(), loss)
    for name, a, b in zip(("dtn", "dpn", "dW"), fl, (dtn, dpn, dw)):
        e = _nrel(a.grad.cpu().double(), b)
        print(f"{name}: normwise rel err vs oracle {e:.2e}")
        assert e <= 1e-2, f"{name}: {e}"


@pytest.mark.parametrize("use_torchaudio", [True, False])
def test_head_fp32_is_materialised(dev, use_torchaudio):
    """Without bf16 autocast the head computes in fp32: the
    joint → exact-f32 Linear → HIP RNN-T chain, equal to the unrounded
    materialised chain and to the float64 oracle without bf16 rounding."""
    from speechbrain_amd.nnet.loss.transducer_head import transducer_head_loss
    from speechbrain_amd.nnet.losses import transducer_loss
    tn, pn, w, targets, in_rel, tg_rel = _case(dev, 3, 11, 6, 256, 129, seed=17)
    fl = [t.clone().requires_grad_() for t in (tn, pn, w)]
    out = transducer_head_loss(*fl, targets, in_rel, tg_rel, 0, "mean", use_torchaudio)
    out.backward()
    leaves = [t.clone().requires_grad_() for t in (tn, pn, w)]
    z = F.leaky_relu(leaves[0].unsqueeze(2) + leaves[1].unsqueeze(1), 0.01)
    ref = transducer_loss(z @ leaves[2].t(), targets, in_rel, tg_rel, 0, "mean", use_torchaudio=use_torchaudio)
    ref.backward()
    assert abs(out.item() - ref.item()) <= 1e-4 * abs(ref.item())
    for name, a, b in zip(("dtn", "dpn", "dW"), fl, leaves):
        assert _nrel(a.grad, b.grad) <= 1e-4, name
