"""(Round-3 record; the SIDE_STREAM switch it toggled was removed with the
rejected variant.)  A/B of TransformerASR.encode's side stream (positional keys + key mask
beside the src Linear): graph replays of the bench's config-3 step with the
switch on and off, alternating, same process and box."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import speechbrain_amd.lobes.models.transformer.TransformerASR as TA  # noqa: E402

dev = torch.device("cuda")
fb, cnn, tr = bench.build_model(256, dev)
g = torch.Generator().manual_seed(0)
wav = (0.1 * torch.randn(32, 240000, generator=g)).to(dev)
wl = torch.ones(32, device=dev)
runs = {}
for flag in (True, False):
    TA.SIDE_STREAM = flag
    step = bench.make_step(fb, cnn, tr, wav, wl)
    for _ in range(3):
        step()
    torch.cuda.synchronize()
    gr = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gr):
        out = step()
    runs[flag] = (gr, out)
ref = None
res = {True: [], False: []}
for rep in range(6):
    for flag in (True, False):
        gr, out = runs[flag]
        for _ in range(3):
            gr.replay()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            gr.replay()
        e1.record()
        torch.cuda.synchronize()
        res[flag].append(e0.elapsed_time(e1) / 20)
print("side stream on : ms/step", sorted(res[True]))
print("side stream off: ms/step", sorted(res[False]))
a, b = runs[True][1], runs[False][1]
print("outputs identical:", bool(torch.equal(a, b)))
