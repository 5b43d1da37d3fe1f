"""One decoder-shaped cross-attention forward (+ backward) through the
MultiheadAttention drop-in, for rocprofv3 kernel stats (see
scripts/mha_decoder_timing.py for the shapes).  usage: [bf16] [bwd]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from speechbrain_amd.nnet.attention import MultiheadAttention
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    B, L, S, E, H = 32, 64, 376, 512, 4
    mha = MultiheadAttention(H, E).to(dev).train(False)
    kpm = torch.arange(S, device=dev)[None, :] >= torch.randint(S // 2, S + 1, (B,), device=dev)[:, None]
    kpm[:, 0] = False
    bf16, bwd = "bf16" in sys.argv, "bwd" in sys.argv
    xq = torch.randn(B, L, E, device=dev)
    xkv = torch.randn(B, S, E, device=dev)
    for _ in range(10):
        q = xq.clone().requires_grad_(bwd)
        kv = xkv.clone().requires_grad_(bwd)
        with torch.set_grad_enabled(bwd), torch.autocast("cuda", dtype=torch.bfloat16, enabled=bf16):
            out, _ = mha(q, kv, kv, key_padding_mask=kpm)
        if bwd:
            out.float().sum().backward()
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
