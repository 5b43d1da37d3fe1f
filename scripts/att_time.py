import os, sys, torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import speechbrain_amd._lib as _L
if os.environ.get("SBK_PROBE_LIB"):
    _L.LIB_PATH = os.path.abspath(os.environ["SBK_PROBE_LIB"])
from speechbrain_amd import _enc
dev = torch.device("cuda")
B, T, H, dh = 32, 376, 4, 64
d = H * dh
qkv = torch.randn(B * T, 3 * d, device=dev).to(torch.bfloat16)
pk = torch.randn(2 * T - 1, d, device=dev).to(torch.bfloat16)
u = torch.randn(H * dh, device=dev); v = torch.randn(H * dh, device=dev)
kpm = torch.zeros(B, T, dtype=torch.uint8, device=dev)
ref = None
for _ in range(5):
    o, _ = _enc.relpos_attention(qkv, pk, u, v, kpm, B, T, H, dh, 1 / 16.0)
torch.cuda.synchronize()
s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
best = 1e9
for rep in range(5):
    s.record()
    for _ in range(100):
        _enc.relpos_attention(qkv, pk, u, v, kpm, B, T, H, dh, 1 / 16.0)
    e.record(); torch.cuda.synchronize()
    best = min(best, s.elapsed_time(e) / 100 * 1e3)
print(os.environ.get("SBK_PROBE_LIB", "product"), f"best-of-5 avg {best:.2f} us per launch")
