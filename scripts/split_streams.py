"""Experiment: the config-3 step at B=32 on one stream vs the same 32
utterances as two B=16 halves on two streams inside one HIP graph (kernel
phases of the two halves overlap).  usage: python scripts/split_streams.py"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

dev = torch.device("cuda")
fbank, cnn, tr = bench.build_model(256, dev)
g = torch.Generator().manual_seed(1234)
wav = (0.1 * torch.randn(32, 240000, generator=g)).to(dev)
wl = torch.ones(32, device=dev)


def timed(run, n=40):
    for _ in range(5):
        run()
    torch.cuda.synchronize()
    best = 1e9
    for _ in range(3):
        t0 = time.perf_counter()
        for _ in range(n):
            run()
        torch.cuda.synchronize()
        best = min(best, (time.perf_counter() - t0) / n * 1e3)
    return best


one = bench.capture(bench.make_step(fbank, cnn, tr, wav, wl), False)
print(f"B=32 one stream: {timed(one):.4f} ms")
for parts in (2, 4):
    n = 32 // parts
    steps = [bench.make_step(fbank, cnn, tr, wav[i * n:(i + 1) * n].contiguous(), wl[i * n:(i + 1) * n].contiguous())
             for i in range(parts)]
    streams = [torch.cuda.Stream() for _ in range(parts)]
    outs = []

    def split():
        cur = torch.cuda.current_stream()
        res = []
        for s, st in zip(streams, steps):
            s.wait_stream(cur)
            with torch.cuda.stream(s):
                res.append(st())
        for s in streams:
            cur.wait_stream(s)
        return res

    ref = [o.float() for o in split()]
    run = bench.capture(split, False)
    print(f"B=32 as {parts} x B={n} on {parts} streams: {timed(run):.4f} ms")
