"""Per-launch time of the layer-chain FFN kernel (sbk_ffn_chain: FFN2 + norm2
of layer i, FFN1 + norm1 + in_proj of layer i+1; M = 12032, config 3) for one
library build, by HIP-graph replay; A/B of probe builds (never the product).
usage: python scripts/chain_time.py [lib.so ...]   (no argument: the product library)"""
import os
import subprocess
import sys

if len(sys.argv) > 1 and sys.argv[1] != "--one":
    for lib in sys.argv[1:]:
        env = dict(os.environ, SBK_PROBE_LIB=lib)
        r = subprocess.run([sys.executable, __file__, "--one"], env=env, capture_output=True, text=True, timeout=120)
        print(f"{os.path.basename(lib):32s} {r.stdout.strip() or r.stderr.strip()[-600:]}", flush=True)
    sys.exit(0)

import torch  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import speechbrain_amd._lib as _L  # noqa: E402
if os.environ.get("SBK_PROBE_LIB"):
    _L.LIB_PATH = os.path.abspath(os.environ["SBK_PROBE_LIB"])
from speechbrain_amd import _enc  # noqa: E402

dev = torch.device("cuda")
D, H, M = 256, 1024, 12032
g = torch.Generator(device=dev).manual_seed(0)


def blk():
    w1 = _enc.cast_bf16((torch.randn(H, D, device=dev, generator=g) / 16).contiguous())
    w2 = _enc.cast_bf16((torch.randn(D, H, device=dev, generator=g) / 32).contiguous())
    ln = (torch.ones(D, device=dev), torch.zeros(D, device=dev), 1e-5)
    return ln, w1, torch.zeros(H, device=dev), w2, torch.zeros(D, device=dev), 0.5


la = blk() + (((torch.ones(D, device=dev), torch.zeros(D, device=dev), 1e-5)),)
lb = blk() + (None,)
wp = _enc.cast_bf16((torch.randn(3 * D, D, device=dev, generator=g) / 16).contiguous())
nl = (torch.ones(D, device=dev), torch.zeros(D, device=dev), 1e-5)
x = torch.randn(M, D, device=dev, generator=g)


def fn():
    return _enc.ffn_chain(x, la, lb, "swish", 0.0, nl, wp)


for _ in range(3):
    out = fn()
torch.cuda.synchronize()
s = torch.cuda.Stream()
s.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(s):
    fn()
torch.cuda.current_stream().wait_stream(s)
reps = 30
gr = torch.cuda.CUDAGraph()
with torch.cuda.graph(gr):
    for _ in range(reps):
        fn()
gr.replay()
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(5):
    gr.replay()
e1.record()
torch.cuda.synchronize()
us = e0.elapsed_time(e1) / (5 * reps) * 1000.0
o = out if isinstance(out, torch.Tensor) else out[-1]
print(f"{us:7.2f} us/launch  {2.49e6 * M / us / 1e6:6.0f} TF/s  checksum {float(o.double().abs().sum()):.6e}")
