"""Joint-output projection GEMM at C4 shapes: sbk_gemm (MFMA kernel) vs
torch.mm (hipBLASLt), bf16 operands, fp32 out.  M = 32*376*65, N = 1000, K = 1024."""
import time
import torch
from speechbrain_amd import _enc

M, N, K = 32 * 376 * 65, 1000, 1024
a = torch.randn(M, K, device="cuda").to(torch.bfloat16)
w = (torch.randn(N, K, device="cuda") / 32).to(torch.bfloat16)


def t(fn, n=5):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / n


fl = 2.0 * M * N * K
for tile in (2, 1, 3, 7, 11, 12, 19, 21):
    try:
        s = t(lambda: _enc.gemm(a, w, tile=tile))
        print(f"sbk_gemm tile {tile}: {s*1e3:.3f} ms  {fl/s/1e12:.1f} TF/s", flush=True)
    except Exception as e:
        print("tile", tile, "failed", e)
for name, fn in [("sbk_gemm f32out", lambda: _enc.gemm(a, w)),
                 ("torch.mm bf16out", lambda: torch.mm(a, w.t())),
                 ("torch.mm f32out", lambda: torch.mm(a, w.t(), out_dtype=torch.float32) if hasattr(torch.mm, "__call__") else None)]:
    try:
        s = t(fn)
        print(f"{name}: {s*1e3:.3f} ms  {fl/s/1e12:.1f} TF/s", flush=True)
    except Exception as e:
        print(name, "failed", e)
g = torch.randn(M, N, device="cuda").to(torch.bfloat16)
for name, fn in [("dgrad g@w", lambda: torch.mm(g, w)), ("wgrad g^T@a", lambda: torch.mm(g.t(), a))]:
    s = t(fn)
    print(f"{name}: {s*1e3:.3f} ms  {fl/s/1e12:.1f} TF/s", flush=True)
