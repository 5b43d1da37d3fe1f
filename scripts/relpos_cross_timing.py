"""RelPosMHAXL cross-attention timing (query != key/value: a Conformer
TransformerASR decoder's cross-attention, Transformer.py:549-556): B = 32,
64 tokens, 376 encoder frames, d 256, 4 heads; forward and forward +
backward, fp32 and bf16 autocast.  usage: python scripts/relpos_cross_timing.py"""
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
    from speechbrain_amd.nnet.attention import RelPosEncXL, RelPosMHAXL
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    B, L, S, E, H = 32, 64, 376, 256, 4
    m = RelPosMHAXL(E, num_heads=H, dropout=0.0).to(dev).eval()
    pe = RelPosEncXL(E).to(dev)
    xq = torch.randn(B, L, E, device=dev)
    xkv = torch.randn(B, S, E, device=dev)
    kpm = torch.arange(S, device=dev)[None, :] >= torch.randint(S // 2, S + 1, (B,), device=dev)[:, None]
    kpm[:, 0] = False
    pos = pe(xkv)
    print(f"B={B} Lq={L} Lk={S} E={E} H={H}; us per call (mean of 20)")
    for dt in ("fp32", "bf16"):
        for grad in (False, True):
            def run():
                q = xq.clone().requires_grad_(grad)
                kv = xkv.clone().requires_grad_(grad)
                with torch.autocast("cuda", dtype=torch.bfloat16, enabled=dt == "bf16"):
                    out, _ = m(q, kv, kv, pos_embs=pos, key_padding_mask=kpm)
                if grad:
                    out.float().sum().backward()
            with torch.set_grad_enabled(grad):
                print(f"{dt:5s} {'fwd+bwd' if grad else 'fwd':8s} {timeit(run):9.1f}")


if __name__ == "__main__":
    main()
