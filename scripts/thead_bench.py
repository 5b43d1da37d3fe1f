"""Transducer-head timing at config-4 shapes (GPU box, not the product):
the fused path's kernels one by one and end to end, against the
materialised chain (joint -> logits GEMM -> rnnt with fused log-softmax ->
dense grad -> dZ / dW GEMMs -> joint backward).
    python scripts/thead_bench.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import speechbrain_amd._lib as _L  # noqa: E402
if os.environ.get("SBK_PROBE_LIB"):
    _L.LIB_PATH = os.path.abspath(os.environ["SBK_PROBE_LIB"])  # probe builds (not product)
from speechbrain_amd import _enc  # noqa: E402
from speechbrain_amd._lib import lib, ptr, stream_of  # noqa: E402

dev = torch.device("cuda")
B, T, U1, J, V = 32, 376, 65, 1024, 1000
n = B * T * U1
L = lib()


def ev_time(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1000.0


g = torch.Generator().manual_seed(0)
tn = (0.5 * torch.randn(B, T, J, generator=g)).to(dev)
pn = (0.5 * torch.randn(B, U1, J, generator=g)).to(dev)
w = (torch.randn(V, J, generator=g) / J ** 0.5).to(dev)
from speechbrain_amd.nnet.loss.transducer_head import _padded_bf16  # noqa: E402
wb = _padded_bf16(w)
labels = torch.randint(1, V, (B, U1 - 1), generator=g).int().to(dev)
Tl = torch.full((B,), T, dtype=torch.int32, device=dev)
Ul = torch.randint(40, U1, (B,), generator=g).int().to(dev)
ws = torch.empty(int(L.sbk_rnnt_workspace_floats(B, T, U1)), device=dev)
out = torch.empty((), device=dev)
s = stream_of(tn)
Vp = int(L.sbk_thead_vpad(V))
go = torch.full((1,), 1.0 / B, device=dev)
ds = torch.empty(n, Vp, device=dev, dtype=torch.bfloat16)
wt = wb.t().contiguous()
dtn, dpn = torch.empty_like(tn), torch.empty_like(pn)
jws = torch.empty(int(L.sbk_joint_bwd_workspace_floats(B, T, U1, J)), device=dev)
dw = torch.zeros(V, J, device=dev)

fl = 2.0 * n * J * V
res = {}
res["thead_fwd"] = ev_time(lambda: L.sbk_thead_fwd(ptr(tn), ptr(pn), ptr(wb), ptr(labels), B, T, U1, J, V, 0, 3,
                                                   0.01, ptr(ws[2 * n:]), ptr(ws), ptr(ws[n:]), s))
res["lattice"] = ev_time(lambda: L.sbk_rnnt_lattice(ptr(Tl), ptr(Ul), B, T, U1, 1, 0, ptr(ws), ptr(out), s))
res["thead_dlogits"] = ev_time(lambda: L.sbk_thead_dlogits(ptr(tn), ptr(pn), ptr(wb), ptr(labels), B, T, U1, J, V, 0,
                                                           3, 0.01, ptr(ws[2 * n:]), ptr(ws[5 * n:]), ptr(ws[6 * n:]),
                                                           ptr(go), 0, ptr(ds), s))
dz = _enc.gemm(ds, wt, out_dtype=torch.bfloat16)
res["dz_gemm"] = ev_time(lambda: _enc.gemm(ds, wt, out_dtype=torch.bfloat16))
res["joint_bwd"] = ev_time(lambda: L.sbk_joint_bwd(ptr(tn), ptr(pn), ptr(dz), 1, B, T, U1, J, 3, 0.01, ptr(dtn),
                                                   ptr(dpn), ptr(jws), s))
res["thead_wgrad"] = ev_time(lambda: L.sbk_thead_wgrad(ptr(ds), ptr(tn), ptr(pn), ptr(Tl), B, T, U1, J, V, 3, 0.01,
                                                       ptr(dw), s))
for k, v in res.items():
    extra = f"  {fl / v / 1e6:.0f} TF/s" if k in ("thead_fwd", "thead_dlogits", "dz_gemm", "thead_wgrad") else ""
    print(f"{k:14s} {v:9.1f} us{extra}", flush=True)
print(f"fused total {sum(res.values()) / 1000:.2f} ms", flush=True)
del dz

# materialised chain (the r01 training path)
from speechbrain_amd.nnet.loss.transducer_head import transducer_head_loss  # noqa: E402
from speechbrain_amd.nnet.losses import transducer_loss  # noqa: E402
import speechbrain_amd._autograd as A  # noqa: E402

tg = labels.clone()
in_rel = torch.ones(B, device=dev)
tg_rel = Ul.float() / (U1 - 1)


def fused():
    a = [t.detach().requires_grad_() for t in (tn, pn, w)]
    transducer_head_loss(*a, tg, in_rel, tg_rel, 0, "mean", True).backward()


def materialised():
    a = [t.detach().requires_grad_() for t in (tn, pn, w)]
    with torch.autocast("cuda", dtype=torch.bfloat16):
        z = A.JointFn.apply(a[0], a[1], 3, 0.01, torch.bfloat16)
        logits = torch.nn.functional.linear(z, a[2])
    transducer_loss(logits.float(), tg, in_rel, tg_rel, 0, "mean", use_torchaudio=True).backward()


torch.cuda.reset_peak_memory_stats()
base = torch.cuda.memory_allocated()
t_f = ev_time(fused, reps=3)
pk_f = (torch.cuda.max_memory_allocated() - base) / 2 ** 30
torch.cuda.reset_peak_memory_stats()
t_m = ev_time(materialised, reps=3)
pk_m = (torch.cuda.max_memory_allocated() - base) / 2 ** 30
print(f"end to end: fused {t_f / 1000:.2f} ms (peak +{pk_f:.2f} GiB) | materialised {t_m / 1000:.2f} ms "
      f"(peak +{pk_m:.2f} GiB)", flush=True)
