"""Per-call time of sbk_specaugment at config 2 (32 x 1501 x 240, recipe draws
of seed 1234, mean fill) for one library build, by HIP-graph replay; A/B of
probe builds (never the product).
usage: python scripts/sa_time.py [lib.so ...]   (no argument: the product library)"""
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
from speechbrain_amd.lobes.augment import SpecAugment  # noqa: E402

dev = torch.device("cuda")
N, T, F = 32, 1501, 240
x = torch.randn(N, T, F, device=dev) * 10 - 40
sa = SpecAugment(time_warp=True, time_warp_window=5, time_warp_mode="bicubic", freq_mask=True,
                 freq_mask_width=(0, 30), n_freq_mask=2, time_mask=True, time_mask_width=(0, 40), n_time_mask=2,
                 replace_with_zero=False)
torch.manual_seed(1234)
c, w, fm, tm = sa.draws(N, T, F)
fm_d, tm_d = fm.to(dev), tm.to(dev)


def fn():
    torch.ops.sbk.specaugment_(x, N, T, F, c, w, fm_d, tm_d, True, -1, 0)


for _ in range(3):
    fn()
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
print(f"{us:7.2f} us/call  (c={c} w={w})  {2 * 4.0 * N * T * F / us / 1e3:.0f} GB/s algorithmic")
