"""HIP RNN-T loss vs the reference's known answer and the CPU oracle."""
import numpy as np
import pytest
import torch

from conftest import assert_close
import oracle.rnnt as OR

pytestmark = pytest.mark.gpu

KAT = [[[[0.1, 0.6, 0.1, 0.1, 0.1], [0.1, 0.1, 0.6, 0.1, 0.1], [0.1, 0.1, 0.2, 0.8, 0.1]],
        [[0.1, 0.6, 0.1, 0.1, 0.1], [0.1, 0.1, 0.2, 0.1, 0.1], [0.7, 0.1, 0.2, 0.1, 0.1]]]]


def test_known_answer(dev):
    """tests/unittests/test_losses.py:109-152 (exact float equality)."""
    from speechbrain_amd.nnet.losses import transducer_loss
    leaf = torch.tensor(KAT, device=dev).requires_grad_()
    log_probs = leaf.log_softmax(dim=-1)
    targets = torch.tensor([[1, 2]], device=dev).int()
    out = transducer_loss(log_probs, targets, torch.tensor([1.0], device=dev), torch.tensor([1.0], device=dev),
                          blank_index=0, use_torchaudio=False)
    out.backward()
    assert abs(out.item() - 2.247833251953125) < 1e-6
    assert out.item() == 2.247833251953125
    # gradient wrt the leaf vs the oracle chained through both log_softmaxes
    lp = torch.tensor(KAT).log_softmax(-1)
    _, g_logit = OR.transducer_loss(lp.numpy(), np.array([[1, 2]]), np.array([1.0]), np.array([1.0]), 0)
    lp_cpu = torch.tensor(KAT, requires_grad=True)
    torch.autograd.backward(lp_cpu.log_softmax(-1), torch.from_numpy(g_logit))
    assert_close(leaf.grad, lp_cpu.grad, rtol=1e-5, name="kat grad")


def _case(seed, B=3, T=9, U=4, V=7):
    rng = np.random.default_rng(seed)
    logits = rng.standard_normal((B, T, U + 1, V)).astype(np.float32)
    labels = rng.integers(1, V, (B, U)).astype(np.int32)
    Tl = np.array([T, T - 2, 3][:B], np.int32)
    Ul = np.array([U, 2, U - 1][:B], np.int32)
    return logits, labels, Tl, Ul


@pytest.mark.parametrize("reduction", ["mean", "sum", "none"])
def test_transducer_apply_vs_oracle(dev, reduction):
    from speechbrain_amd.nnet.loss.transducer_loss import Transducer
    for seed in range(3):
        logits, labels, Tl, Ul = _case(seed)
        lp = OR.log_softmax(logits.astype(np.float64)).astype(np.float32)
        ref_loss, ref_g, ref_a, ref_b = OR.transducer_forward(lp, labels, Tl, Ul, 0, reduction)
        x = torch.from_numpy(lp).to(dev).requires_grad_()
        loss = Transducer.apply(x, torch.from_numpy(labels).to(dev), torch.from_numpy(Tl).to(dev),
                                torch.from_numpy(Ul).to(dev), 0, reduction)
        assert_close(loss, np.asarray(ref_loss), rtol=1e-6, name="loss")
        go = torch.ones_like(loss) if reduction != "none" else torch.arange(1, 4, device=dev, dtype=torch.float32)
        loss.backward(go)
        scale = go.cpu().numpy().reshape(-1, 1, 1, 1) if reduction == "none" else 1.0
        assert_close(x.grad, ref_g * scale, rtol=1e-6, name="grad")


def test_invalid_reduction_raises(dev):
    from speechbrain_amd.nnet.loss.transducer_loss import Transducer
    logits, labels, Tl, Ul = _case(0)
    with pytest.raises(Exception, match="Unexpected reduction"):
        Transducer.apply(torch.from_numpy(logits).to(dev), torch.from_numpy(labels).to(dev),
                         torch.from_numpy(Tl).to(dev), torch.from_numpy(Ul).to(dev), 0, "batchmean")


def test_fused_logits_path_vs_oracle(dev):
    """transducer_loss(use_torchaudio=False): loss and d loss / d logits."""
    from speechbrain_amd.nnet.losses import transducer_loss
    for seed in range(3):
        logits, labels, Tl, Ul = _case(10 + seed, B=3, T=12, U=5, V=11)
        T, U = logits.shape[1], labels.shape[1]
        rel_T = Tl / T
        rel_U = Ul / U
        ref_loss, ref_g = OR.transducer_loss(logits, labels, rel_T, rel_U, 0, "mean")
        x = torch.from_numpy(logits).to(dev).requires_grad_()
        loss = transducer_loss(x, torch.from_numpy(labels).to(dev), torch.from_numpy(rel_T).float().to(dev),
                               torch.from_numpy(rel_U).float().to(dev), 0, use_torchaudio=False)
        loss.backward()
        assert_close(loss, np.asarray(ref_loss), rtol=1e-6, name="loss")
        assert_close(x.grad, ref_g, rtol=1e-5, name="grad")


def test_torchaudio_mode_semantics(dev):
    """use_torchaudio=True: -log P (brute force), mean over batch, grad / B."""
    from speechbrain_amd.nnet.losses import transducer_loss
    logits, labels, Tl, Ul = _case(21, B=2, T=5, U=3, V=6)
    Tl = np.array([5, 4], np.int32)
    Ul = np.array([3, 2], np.int32)
    x = torch.from_numpy(logits).to(dev).requires_grad_()
    loss = transducer_loss(x, torch.from_numpy(labels).to(dev), torch.from_numpy(Tl / 5).float().to(dev),
                           torch.from_numpy(Ul / 3).float().to(dev), 0, use_torchaudio=True)
    lp = OR.log_softmax(logits.astype(np.float64))
    nll = [OR.brute_force_nll(lp[b], labels[b], Tl[b], Ul[b], 0) for b in range(2)]
    assert abs(loss.item() - np.mean(nll)) < 1e-4
    loss.backward()
    # finite difference on one logit (float64 brute force)
    eps = 1e-3
    lp2 = logits.astype(np.float64).copy()
    lp2[0, 1, 1, 2] += eps
    nll2 = OR.brute_force_nll(OR.log_softmax(lp2)[0], labels[0], Tl[0], Ul[0], 0)
    fd = (nll2 - nll[0]) / eps / 2
    assert abs(fd - x.grad[0, 1, 1, 2].item()) < 1e-3


def test_full_size_config4(dev):
    """BASELINE config 4 shapes: B=32, T=376, U+1=65, V=1000 (3.1 GB logits).
    Checks 2 utterances against the oracle and size-independent properties."""
    from speechbrain_amd.nnet.losses import transducer_loss
    B, T, U, V = 32, 376, 64, 1000
    g = torch.Generator(device=dev).manual_seed(0)
    logits = torch.randn(B, T, U + 1, V, device=dev, generator=g)
    rng = np.random.default_rng(0)
    labels = torch.from_numpy(rng.integers(1, V, (B, U)).astype(np.int32)).to(dev)
    ulen = rng.integers(40, 65, B)
    rel_U = torch.from_numpy(ulen / U).float().to(dev)
    rel_T = torch.ones(B, device=dev)
    x = logits.requires_grad_()
    loss = transducer_loss(x, labels, rel_T, rel_U, 0, reduction="none", use_torchaudio=False)
    loss.sum().backward()
    assert torch.isfinite(loss).all() and torch.isfinite(x.grad).all()
    # each logits-gradient row sums to zero (softmax Jacobian property)
    rs = x.grad.sum(-1)
    assert rs.abs().max().item() < 1e-4
    for b in (0, 17):
        lg = logits[b:b + 1].detach().cpu().numpy()
        lab = labels[b:b + 1].cpu().numpy()
        ref_loss, ref_g = OR.transducer_loss(lg, lab, np.array([1.0]), np.array([ulen[b] / U]), 0, "none")
        assert_close(loss[b:b + 1], np.asarray(ref_loss), rtol=1e-5, name=f"loss{b}")
        # Gradients are -exp(α + β + lp - log P) with α, β ~ -3e3 at T=376,
        # V=1000: one f32 ulp of those sums is ~2.4e-4, so 1-ulp differences in
        # the per-cell log-probs (GPU f32 log-softmax vs the oracle's f64 one)
        # move a gradient by that much relative; small cases are checked at
        # 1e-5..1e-6 above.
        assert_close(x.grad[b:b + 1, :, :ulen[b] + 1], ref_g[:, :, :ulen[b] + 1], rtol=5e-4, name=f"grad{b}")


def _fd_nll(lp, labels, Tl, Ul, b, idx, eps=1e-4):
    """Central difference of the brute-force -log P (float64) of utterance b
    wrt one log-prob entry (entries perturbed as free inputs)."""
    a = lp[b].copy()
    a[idx] += eps
    hi = OR.brute_force_nll(a, labels[b], Tl[b], Ul[b], 0)
    a[idx] -= 2 * eps
    lo = OR.brute_force_nll(a, labels[b], Tl[b], Ul[b], 0)
    return (hi - lo) / (2 * eps)


def test_numba_mode_grads_vs_finite_differences(dev):
    """Transducer.apply gradients (the reference's cu_kernel_compute_grad
    contract, transducer_loss.py:183-236: un-normalised d(-log P)/d lp, not
    divided by T or B) against central differences of the brute-force path
    sum — independent of the oracle's α/β gradient restatement.  Every lattice
    cell's blank and label entry of both utterances is checked, plus entries
    that must get exactly zero gradient (other vocab, cells outside T_b/U_b)."""
    from speechbrain_amd.nnet.loss.transducer_loss import Transducer
    logits, labels, Tl, Ul = _case(33, B=2, T=5, U=3, V=6)
    Tl = np.array([5, 4], np.int32)
    Ul = np.array([3, 2], np.int32)
    lp = OR.log_softmax(logits.astype(np.float64))
    x = torch.from_numpy(lp.astype(np.float32)).to(dev).requires_grad_()
    loss = Transducer.apply(x, torch.from_numpy(labels).to(dev), torch.from_numpy(Tl).to(dev),
                            torch.from_numpy(Ul).to(dev), 0, "sum")
    loss.backward()
    g = x.grad.cpu().numpy().astype(np.float64)
    checked = 0
    for b in range(2):
        for t in range(Tl[b]):
            for u in range(Ul[b] + 1):
                entries = [0] + ([int(labels[b, u])] if u < Ul[b] else [])
                for v in entries:
                    fd = _fd_nll(lp, labels, Tl, Ul, b, (t, u, v))
                    assert abs(g[b, t, u, v] - fd) <= 2e-5 * max(1.0, abs(fd)), (b, t, u, v, g[b, t, u, v], fd)
                    checked += 1
                others = [v for v in range(6) if v not in entries]
                assert np.all(g[b, t, u, others] == 0.0)
        assert np.all(g[b, Tl[b]:] == 0.0) and np.all(g[b, :, Ul[b] + 1:] == 0.0)
    assert checked > 40
    # the loss itself: -log P / T_b summed (Numba semantics)
    nll = [OR.brute_force_nll(lp[b], labels[b], Tl[b], Ul[b], 0) for b in range(2)]
    assert abs(loss.item() - sum(n / t for n, t in zip(nll, Tl))) < 1e-5


def test_numba_mode_logit_grads_vs_finite_differences(dev):
    """transducer_loss(use_torchaudio=False) gradient wrt the logits (the
    wrapper's log_softmax chained, losses.py:79-85) against central
    differences of brute-force -log P over perturbed logits."""
    from speechbrain_amd.nnet.losses import transducer_loss
    logits, labels, _, _ = _case(34, B=1, T=4, U=2, V=5)
    x = torch.from_numpy(logits).to(dev).requires_grad_()
    loss = transducer_loss(x, torch.from_numpy(labels).to(dev), torch.ones(1, device=dev),
                           torch.ones(1, device=dev), 0, use_torchaudio=False)
    loss.backward()
    g = x.grad.cpu().numpy()
    eps = 1e-4
    base = logits.astype(np.float64)
    for t in range(4):
        for u in range(3):
            for v in range(5):
                a = base.copy()
                a[0, t, u, v] += eps
                hi = OR.brute_force_nll(OR.log_softmax(a)[0], labels[0], 4, 2, 0)
                a[0, t, u, v] -= 2 * eps
                lo = OR.brute_force_nll(OR.log_softmax(a)[0], labels[0], 4, 2, 0)
                fd = (hi - lo) / (2 * eps)
                assert abs(g[0, t, u, v] - fd) <= 2e-5 * max(1.0, abs(fd)), (t, u, v, g[0, t, u, v], fd)


def test_invalid_lengths_and_labels_give_nan_not_corruption(dev):
    """lengths outside the lattice (U_b > U1-1, T_b > maxT, T_b = 0)
    or labels outside [0, V) poison that utterance's loss with NaN; the other
    utterances of the batch are unaffected (no write outside a slab)."""
    from speechbrain_amd.nnet.loss.transducer_loss import Transducer
    logits, labels, Tl, Ul = _case(40, B=3, T=6, U=3, V=5)
    lp = OR.log_softmax(logits.astype(np.float64)).astype(np.float32)
    good_loss, _, _, _ = OR.transducer_forward(lp, labels, Tl, Ul, 0, "none")
    for bad in ("U", "T", "T0", "label"):
        Tb, Ub, lab = Tl.copy(), Ul.copy(), labels.copy()
        if bad == "U":
            Ub[1] = 9
        elif bad == "T":
            Tb[1] = 7
        elif bad == "T0":
            Tb[1] = 0
        else:
            lab[1, 0] = 5
        out = Transducer.apply(torch.from_numpy(lp).to(dev), torch.from_numpy(lab).to(dev),
                               torch.from_numpy(Tb).to(dev), torch.from_numpy(Ub).to(dev), 0, "none").cpu().numpy()
        assert np.isnan(out[1]), (bad, out)
        assert_close(out[[0, 2]], np.asarray(good_loss)[[0, 2]], rtol=1e-6, name=bad)
