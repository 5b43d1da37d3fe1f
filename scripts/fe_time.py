"""Per-launch time of the Fbank spectrum kernel (fb._deferred, B = 32 x 15 s)
for one library build; A/B of kernel variants built by probe_build.sh.
usage: python scripts/fe_time.py [lib.so ...]   (no argument: the product library)"""
import os
import subprocess
import sys

if len(sys.argv) > 2 or (len(sys.argv) == 2 and sys.argv[1] != "--one"):
    for lib in sys.argv[1:]:
        env = dict(os.environ, SBK_PROBE_LIB=lib)
        r = subprocess.run([sys.executable, __file__, "--one"], env=env, capture_output=True, text=True, timeout=120)
        print(lib, r.stdout.strip() or r.stderr.strip()[-400:])
    sys.exit(0)

import torch  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import speechbrain_amd._lib as _L  # noqa: E402
if os.environ.get("SBK_PROBE_LIB"):
    _L.LIB_PATH = os.path.abspath(os.environ["SBK_PROBE_LIB"])
from speechbrain_amd.lobes.features import Fbank  # noqa: E402

dev = torch.device("cuda")
fb = Fbank(n_mels=80).to(dev)
g = torch.Generator().manual_seed(0)
wav = (0.1 * torch.randn(32, 240000, generator=g)).to(dev)
ref = None
for _ in range(3):
    out, _sm = fb._deferred(wav)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(50):
    fb._deferred(wav)
e1.record()
torch.cuda.synchronize()
print(f"{1000 * e0.elapsed_time(e1) / 50:.2f} us  checksum {float(out.double().sum()):.6f}")
