"""Front-end probe (GPU box, not part of the product): the fused two-block
ConvolutionFrontEnd on (32, 1501, 80) bf16, timed."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import speechbrain_amd._lib as _L  # noqa: E402
if os.environ.get("SBK_PROBE_LIB"):
    _L.LIB_PATH = os.path.abspath(os.environ["SBK_PROBE_LIB"])  # probe builds of the kernel (not product)
from speechbrain_amd.lobes.models.convolution import ConvolutionFrontEnd  # noqa: E402
from scripts.kbench import timeit  # noqa: E402

dev = torch.device("cuda")
cnn = ConvolutionFrontEnd(input_shape=(8, 10, 80), num_blocks=2, num_layers_per_block=1, out_channels=(64, 32),
                          kernel_sizes=(3, 3), strides=(2, 2), residuals=(False, False)).to(dev).eval()
x = torch.randn(32, 1501, 80, device=dev)
with torch.no_grad(), torch.autocast("cuda", dtype=torch.bfloat16):
    us = timeit(lambda: cnn.run(x, torch.bfloat16), reps=20)
print(f"frontend fused: {us:.1f}us", flush=True)

if os.environ.get("SBK_PROBE_TL"):
    import ctypes
    import numpy as np
    torch.cuda.synchronize()
    buf = (ctypes.c_ulonglong * (12 * 16))()
    assert ctypes.CDLL(_L.LIB_PATH).sbk_probe_fe_tl(buf) == 0
    tl = np.array(buf, dtype=np.int64).reshape(12, 16)
    for w in range(12):
        r = tl[w]
        # persistent kernel (marks of workgroup 100's last tile): 0 tile top, 1 after the xs barrier,
        # 2 block-1 MFMA + LN statistics, 3 block-1 writes, 12 block 2 (+ next-tile fetch issue), 13 epilogue
        print(f"w{w}: xs-stage {r[1]-r[0]} block1 mfma+stats {r[2]-r[1]} block1 writes {r[3]-r[2]} "
              f"block2 {r[12]-r[3]} epi {r[13]-r[12]} total {r[13]-r[0]}; kernel (all tiles) {r[15]-r[14]}")
