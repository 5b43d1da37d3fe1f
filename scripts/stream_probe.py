"""Driver of scripts/stream_probe.hip (never the product): per-CU L2 -> LDS
weight-stream rate of the layer-chain ring, by ring depth / tile size / what
the waves do per step.  Prints per-variant µs per launch, GB/s per CU, cycles
per 32 KB step (from s_memtime) and the in-kernel clock.
usage: hipcc -O3 --offload-arch=gfx950 -shared -fPIC -o gpurun_probe_stream.so scripts/stream_probe.hip &&
       python scripts/stream_probe.py"""
import ctypes
import os

import numpy as np
import torch

lib = ctypes.CDLL(os.path.abspath(os.environ.get("PROBE_LIB", "gpurun_probe_stream.so")))
dev = torch.device("cuda")
STEP_BYTES_CU = 32768  # the chain's per-step weight bytes per CU
TOTAL = 76 * STEP_BYTES_CU  # the chain's 2.43 MB per launch
BUF = 4 << 20  # the strided layouts span up to 2.62 MB (checked below)
w = torch.randint(0, 1 << 14, (BUF // 2,), dtype=torch.int16, device=dev)
grid = 256
out = torch.empty(grid * 512, device=dev)
clk = torch.zeros(grid * 2, dtype=torch.int64, device=dev)
s = torch.cuda.current_stream().cuda_stream
names = {0: "dma", 1: "dma+frag", 3: "dma+frag+hid", 5: "dma+frag+mfma", 7: "dma+frag+hid+mfma"}
cases = [(ns, gl, m, 0) for ns, gl in ((2, 4), (4, 4), (2, 8)) for m in (0, 1, 3, 5, 7)]
cases += [(ns, 4, m, ldb) for ns in (2, 4) for ldb in (512, 2048) for m in (0, 7)]
for ns, gl, mode, ldb in cases:
    steps = TOTAL // (8 * gl * 1024)
    if ldb:
        cpm = ldb // 128
        span = (-(-steps // cpm)) * gl * 64 * ldb
    else:
        span = steps * 8 * gl * 1024
    assert span <= BUF, (ns, gl, ldb, span)
    if True:
        args = (ns, gl, mode, ldb, ctypes.c_void_p(w.data_ptr()), steps, ctypes.c_void_p(out.data_ptr()),
                ctypes.c_void_p(clk.data_ptr()), grid, ctypes.c_void_p(s))
        for _ in range(3):
            assert lib.stream_probe(*args) == 0
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        n = 20
        e0.record()
        for _ in range(n):
            lib.stream_probe(*args)
        e1.record()
        torch.cuda.synchronize()
        us = 1000 * e0.elapsed_time(e1) / n
        c = clk.view(grid, 2).cpu().numpy().astype(np.float64)
        cyc = np.median(c[:, 0])
        ghz = np.median(c[:, 0] / c[:, 1]) * 0.1
        print(f"NS={ns} tile={8 * gl}KB ld={ldb:4d} {names[mode]:>18}: {us:7.2f} us/launch  {TOTAL / us / 1e3:6.1f} GB/s/CU  "
              f"{cyc / (TOTAL / STEP_BYTES_CU):6.0f} cyc/32KB  clock {ghz:.2f} GHz", flush=True)
