"""Decoder-shaped MultiheadAttention timing (the general path that
TransformerASR's decoder self- / cross-attention takes): the drop-in
(speechbrain_amd.nnet.attention.MultiheadAttention, q / k / v projections on
sbk_gemm + the xattn core in its no-position mode + out_proj) against
torch.nn.MultiheadAttention with the same weights — the call the reference
makes (attention.py:642-779) — forward, and forward + backward.

Shapes: the LibriSpeech transformer.yaml decoder (d_model 512, nhead 4), B =
32 utterances, 64 target tokens, 376 encoder frames (C3's 15 s); the self-
attention with the causal lookahead mask, the cross-attention unmasked with
a key padding mask.  fp32, and bf16 autocast.
usage: python scripts/mha_decoder_timing.py"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timeit(fn, n=20, w=5):
    for _ in range(w):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / n * 1e6


def main():
    from speechbrain_amd.nnet.attention import MultiheadAttention
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    B, L, S, E, H = 32, 64, 376, 512, 4
    mha = MultiheadAttention(H, E).to(dev).train(False)
    ref = mha.att  # the wrapped torch.nn.MultiheadAttention: same weights
    causal = torch.triu(torch.ones(L, L, dtype=torch.bool, device=dev), diagonal=1)
    kpm = torch.arange(S, device=dev)[None, :] >= torch.randint(S // 2, S + 1, (B,), device=dev)[:, None]
    kpm[:, 0] = False
    cases = {
        "self  (L=S=64, causal)": dict(q=(B, L), kv=(B, L), attn_mask=causal, kpm=None),
        "cross (L=64, S=376, kpm)": dict(q=(B, L), kv=(B, S), attn_mask=None, kpm=kpm),
    }
    print(f"B={B} E={E} H={H}; us per call (mean of 20)")
    print(f"{'case':28s} {'dtype':6s} {'pass':8s} {'drop-in':>9s} {'torch MHA':>10s} {'ratio':>6s}")
    for name, c in cases.items():
        for dt in ("fp32", "bf16"):
            xq = torch.randn(*c["q"], E, device=dev)
            xkv = xq if c["kv"] == c["q"] else torch.randn(*c["kv"], E, device=dev)
            ctx = (lambda: torch.autocast("cuda", dtype=torch.bfloat16)) if dt == "bf16" else \
                (lambda: torch.autocast("cuda", enabled=False))

            def ours(grad):
                q = xq.clone().requires_grad_(grad)
                kv = q if xkv is xq else xkv.clone().requires_grad_(grad)
                with ctx():
                    out, _ = mha(q, kv, kv, attn_mask=c["attn_mask"], key_padding_mask=c["kpm"])
                if grad:
                    out.float().sum().backward()

            def theirs(grad):
                q = xq.clone().requires_grad_(grad)
                kv = q if xkv is xq else xkv.clone().requires_grad_(grad)
                with ctx():
                    out, _ = ref(q.transpose(0, 1), kv.transpose(0, 1), kv.transpose(0, 1), attn_mask=c["attn_mask"],
                                 key_padding_mask=c["kpm"])
                if grad:
                    out.float().sum().backward()

            for grad in (False, True):
                with torch.set_grad_enabled(grad):
                    a = timeit(lambda: ours(grad))
                    b = timeit(lambda: theirs(grad))
                print(f"{name:28s} {dt:6s} {'fwd+bwd' if grad else 'fwd':8s} {a:9.1f} {b:10.1f} {a / b:6.2f}")


if __name__ == "__main__":
    main()
