"""Per-launch time of the fused conv module as the config-3 step runs it
(sbk_conv_module_pre: MHSA out_proj + residual + the whole convolution
module, B = 32, T = 376, d = 256, k = 31) for one library build, by HIP-graph
replay; A/B of probe builds (never the product).
usage: python scripts/conv_time.py [lib.so ...]   (no argument: the product library)"""
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
B, T, D, K = 32, 376, 256, 31
g = torch.Generator(device=dev).manual_seed(0)
bf = torch.bfloat16
x = torch.randn(B * T, D, device=dev, generator=g)
o = torch.randn(B * T, D, device=dev, generator=g).to(bf)
wo = (torch.randn(D, D, device=dev, generator=g) / 16).to(bf)
bo = torch.zeros(D, device=dev)
ln = (torch.ones(D, device=dev), torch.zeros(D, device=dev), 1e-5)
w1p = (torch.randn(2 * D, D, device=dev, generator=g) / 16).to(bf)
b1p = torch.zeros(2 * D, device=dev)
wc = torch.randn(K, D, device=dev, generator=g) / 8
w2 = (torch.randn(D, D, device=dev, generator=g) / 16).to(bf)
b2 = torch.zeros(D, device=dev)


def fn():
    return _enc.conv_module(x, B, T, ln, w1p, b1p, wc, None, False, ln, w2, b2, None, pre=(o, wo, bo))


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
print(f"{us:7.2f} us/launch  checksum {float(out.double().abs().sum()):.6e}")
