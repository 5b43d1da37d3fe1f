"""CPU restatement of the SpeechBrain Numba RNN-T loss (test infrastructure).

Restates speechbrain/nnet/loss/transducer_loss.py:
  cu_kernel_forward      :31-106   α lattice, log_p = (α[T-1,U] + lp[T-1,U,∅]) / T
  cu_kernel_backward     :109-180  β lattice, log_p_beta = β[0,0] / T
  cu_kernel_compute_grad :183-236  ∂(-log P)/∂lp at blank and label entries
  Transducer.forward     :252-287  reductions mean|sum|none of -log_p
and speechbrain/nnet/losses.py:27-85 (transducer_loss: relative → absolute
lengths by round(rel·dim), log_softmax, Transducer.apply).

numba is not installed here, so parity is pinned by the reference's
known-answer test (tests/unittests/test_losses.py:109-152, loss
2.247833251953125) and by brute-force path enumeration (`brute_force_nll`).
"""
import itertools
import math

import numpy as np


def _lae(a, b, dt):
    """logaddexp as the reference writes it: max + log1p(exp(-|a-b|))."""
    m = max(a, b)
    return dt(m + dt(math.log1p(math.exp(-abs(a - b)))))


def alpha_beta(lp, labels, T, U, blank, dtype=np.float32):
    """lp: (B, maxT, maxU, V) log-probs; labels (B, maxU-1) ints; T, U (B,)
    ints (U = label count).  Returns alpha, beta (B, maxT, maxU) with zeros
    outside the valid lattice, exactly as the reference leaves them."""
    dt = np.dtype(dtype).type
    lp = np.asarray(lp, dtype=dtype)
    B, maxT, maxU, _ = lp.shape
    alpha = np.zeros((B, maxT, maxU), dtype)
    beta = np.zeros((B, maxT, maxU), dtype)
    for b in range(B):
        Tb, Ub = int(T[b]), int(U[b])
        y = [int(v) for v in labels[b]]
        for t in range(Tb):
            for u in range(Ub + 1):
                if t == 0 and u == 0:
                    continue
                if u == 0:
                    alpha[b, t, 0] = dt(alpha[b, t - 1, 0] + lp[b, t - 1, 0, blank])
                elif t == 0:
                    alpha[b, 0, u] = dt(alpha[b, 0, u - 1] + lp[b, 0, u - 1, y[u - 1]])
                else:
                    emit = dt(alpha[b, t, u - 1] + lp[b, t, u - 1, y[u - 1]])
                    no_emit = dt(alpha[b, t - 1, u] + lp[b, t - 1, u, blank])
                    alpha[b, t, u] = _lae(no_emit, emit, dt)
        for t in range(Tb - 1, -1, -1):
            for u in range(Ub, -1, -1):
                if u == Ub:
                    if t == Tb - 1:
                        beta[b, t, u] = lp[b, t, u, blank]
                    else:
                        beta[b, t, u] = dt(beta[b, t + 1, u] + lp[b, t, u, blank])
                elif t == Tb - 1:
                    beta[b, t, u] = dt(beta[b, t, u + 1] + lp[b, t, u, y[u]])
                else:
                    emit = dt(beta[b, t, u + 1] + lp[b, t, u, y[u]])
                    no_emit = dt(beta[b, t + 1, u] + lp[b, t, u, blank])
                    beta[b, t, u] = _lae(no_emit, emit, dt)
    return alpha, beta


def log_p_alpha(lp, alpha, T, U, blank, dtype=np.float32):
    """transducer_loss.py:101-106: (α[T-1,U] + lp[T-1,U,∅]) / T."""
    dt = np.dtype(dtype).type
    out = np.zeros(len(T), dtype)
    for b in range(len(T)):
        Tb, Ub = int(T[b]), int(U[b])
        out[b] = dt(dt(alpha[b, Tb - 1, Ub] + lp[b, Tb - 1, Ub, blank]) / dt(Tb))
    return out


def grads_wrt_logprobs(lp, labels, alpha, beta, T, U, blank, dtype=np.float32):
    """transducer_loss.py:183-236: dense (B,maxT,maxU,V), zero except the
    blank and label entries; NOT divided by T (quirk kept)."""
    dt = np.dtype(dtype).type
    lp = np.asarray(lp, dtype=dtype)
    g = np.zeros(lp.shape, dtype)
    for b in range(lp.shape[0]):
        Tb, Ub = int(T[b]), int(U[b])
        lpz = beta[b, 0, 0]
        g[b, Tb - 1, Ub, blank] = -dt(math.exp(dt(dt(alpha[b, Tb - 1, Ub] + lp[b, Tb - 1, Ub, blank]) - lpz)))
        for t in range(Tb - 1):
            for u in range(Ub + 1):
                s = dt(dt(alpha[b, t, u] + beta[b, t + 1, u]) + lp[b, t, u, blank])
                g[b, t, u, blank] = -dt(math.exp(dt(s - lpz)))
        for t in range(Tb):
            for u in range(Ub):
                l = int(labels[b][u])
                s = dt(dt(alpha[b, t, u] + beta[b, t, u + 1]) + lp[b, t, u, l])
                g[b, t, u, l] = -dt(math.exp(dt(s - lpz)))
    return g


def transducer_forward(lp, labels, T, U, blank=0, reduction="mean", dtype=np.float32):
    """Transducer.forward (transducer_loss.py:252-287) → (loss, grads)."""
    alpha, beta = alpha_beta(lp, labels, T, U, blank, dtype)
    lpa = log_p_alpha(np.asarray(lp, dtype), alpha, T, U, blank, dtype)
    grads = grads_wrt_logprobs(lp, labels, alpha, beta, T, U, blank, dtype)
    if reduction == "mean":
        loss = -lpa.mean(dtype=dtype)
    elif reduction == "sum":
        loss = -lpa.sum(dtype=dtype)
    elif reduction == "none":
        loss = -lpa
    else:
        raise Exception("Unexpected reduction {}".format(reduction))
    return loss, grads, alpha, beta


def log_softmax(x, axis=-1):
    x = np.asarray(x)
    m = x.max(axis=axis, keepdims=True)
    return x - m - np.log(np.exp(x - m).sum(axis=axis, keepdims=True))


def transducer_loss(logits, targets, input_lens, target_lens, blank_index,
                    reduction="mean", dtype=np.float32):
    """losses.py:27-85 with use_torchaudio=False → (loss, d loss/d logits).

    The gradient wrt logits chains the reference's log_softmax backward:
    g_logit = g_lp - softmax · Σ_v g_lp (g_lp scaled by d(loss)/d(-log_p) =
    1 for mean and sum, exactly as Transducer.backward multiplies by
    grad_output=1)."""
    logits = np.asarray(logits, dtype)
    Tabs = np.round(np.asarray(input_lens) * logits.shape[1]).astype(np.int32)
    Uabs = np.round(np.asarray(target_lens) * np.asarray(targets).shape[1]).astype(np.int32)
    lp = log_softmax(logits.astype(np.float64)).astype(dtype)
    loss, g_lp, _, _ = transducer_forward(lp, targets, Tabs, Uabs, blank_index, reduction, dtype)
    p = np.exp(lp.astype(np.float64))
    g_logit = (g_lp - p * g_lp.sum(-1, keepdims=True)).astype(dtype)
    return loss, g_logit


def brute_force_nll(lp, labels, T, U, blank):
    """-log Σ over all monotone alignments (float64), independent of the
    lattice recursion: an alignment is a choice of which of the T+U steps
    are label emissions (the final step is always the blank at (T-1, U))."""
    lp = np.asarray(lp, np.float64)
    y = [int(v) for v in labels[:U]]
    total = []
    steps = T - 1 + U  # moves before the final blank
    for emit_pos in itertools.combinations(range(steps), U):
        t = u = 0
        s = 0.0
        ep = set(emit_pos)
        for k in range(steps):
            if k in ep:
                s += lp[t, u, y[u]]
                u += 1
            else:
                s += lp[t, u, blank]
                t += 1
        s += lp[T - 1, U, blank]
        total.append(s)
    m = max(total)
    return -(m + math.log(sum(math.exp(v - m) for v in total)))
