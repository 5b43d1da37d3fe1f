"""Does a chain launch that fills only a quarter of the CUs (63 workgroups of
48 rows) overlap with the conv module + attention of another half batch on a
second stream?  Device time per iteration by graph replay: each alone, then
both forked onto two streams in one graph.  (The premise of a 96-row chain
tile that halves the weight stream per row: worth building only if the idle
CUs can be filled.)  GPU box, not the product."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from speechbrain_amd import _enc  # noqa: E402
from speechbrain_amd.lobes.models.transformer.Conformer import ConvolutionModule  # noqa: E402

bf = torch.bfloat16
dev = torch.device("cuda")
torch.manual_seed(0)
D, H, NP = 256, 1024, 768


def ln():
    return (1 + 0.1 * torch.randn(D, device=dev), 0.1 * torch.randn(D, device=dev), 1e-5)


def blk():
    return (ln(), (torch.randn(H, D, device=dev) / 16).to(bf), 0.1 * torch.randn(H, device=dev),
            (torch.randn(D, H, device=dev) / 32).to(bf), 0.1 * torch.randn(D, device=dev), 0.5)


a, b = blk() + (ln(),), blk() + (None,)
nxt = ln()
wp = (torch.randn(NP, D, device=dev) / 16).to(bf)
xq = torch.randn(3008, D, device=dev)   # 63 chain workgroups
xh = torch.randn(6016, D, device=dev)   # 126
xf = torch.randn(12032, D, device=dev)  # 251

Bh, T = 16, 376
cm = ConvolutionModule(D, 31).to(dev).eval()
xc = torch.randn(Bh * T, D, device=dev)
pre = ((torch.randn(Bh * T, D, device=dev) * 0.5).to(bf), (torch.randn(D, D, device=dev) / 16).to(bf),
       torch.zeros(D, device=dev))
qkv = torch.randn(Bh * T, 3 * D, device=dev).to(bf)
pk = torch.randn(2 * T - 1, D, device=dev).to(bf)
u = torch.randn(D, device=dev)
v = torch.randn(D, device=dev)


def chain(x):
    return lambda: _enc.ffn_chain(x, a, b, "swish", 0.0, nxt, wp)


def conv_attn():
    cm.run_fused(xc, Bh, T, None, pre=pre)
    _enc.relpos_attention(qkv, pk, u, v, None, Bh, T, 4, 64, 1 / 16.0)


s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()


def both():
    cur = torch.cuda.current_stream()
    s1.wait_stream(cur)
    s2.wait_stream(cur)
    with torch.cuda.stream(s1):
        chain(xq)()
    with torch.cuda.stream(s2):
        conv_attn()
    cur.wait_stream(s1)
    cur.wait_stream(s2)


def graph_time(fn, reps=20):
    with torch.no_grad():
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            fn()
        torch.cuda.current_stream().wait_stream(s)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for _ in range(reps):
                fn()
        g.replay()
        torch.cuda.synchronize()
        best = 1e9
        for _ in range(5):
            t0 = time.perf_counter()
            g.replay()
            torch.cuda.synchronize()
            best = min(best, (time.perf_counter() - t0) / reps * 1e6)
    return best


if __name__ == "__main__":
    for name, fn in (("chain 251 WG (full batch)", chain(xf)), ("chain 126 WG", chain(xh)),
                     ("chain 63 WG", chain(xq)), ("conv + attention, half batch", conv_attn),
                     ("chain 63 WG || conv + attention (two streams)", both)):
        print(f"{name:48s} {graph_time(fn):8.1f} us", flush=True)
