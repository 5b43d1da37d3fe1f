"""Which op of the config-4 training step is not row-independent?  Single
process: gradients of the full 4-utterance batch vs the two halves
accumulated (no DDP), per tensor; plus the GRU prediction net's outputs on a
half batch vs the full batch (fp32 and bf16 autocast)."""
import sys
import os

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import torch
import test_gpu_ddp as T

dev = torch.device("cuda:0")
for fused in (True, False):
    ro = {"device": str(dev), "auto_mix_prec": "bf16" if fused else False, "max_grad_norm": 0.0}
    full = T._brain(dev, fused, ro)
    T._run(full, dev, 1, steps=1)
    half = T._brain(dev, fused, dict(ro, grad_accumulation_factor=2))
    b = T._batch(dev, 0)
    half.fit_batch([t[0:2] for t in b])
    half.fit_batch([t[2:4] for t in b])
    rows = []
    for k, ref in full.grads.items():
        e = ((half.grads[k].double() - ref.double()).norm() / ref.double().norm().clamp_min(1e-30)).item()
        rows.append((e, k))
    rows.sort()
    print("fused" if fused else "fp32", "worst full-vs-halves:", rows[-6:])
    gru = full.modules.dec
    x = torch.randn(4, 9, 999, device=dev)
    with torch.autocast("cuda", dtype=torch.bfloat16, enabled=fused):
        y4, _ = gru(x)
        y2, _ = gru(x[:2])
    print("GRU half vs full max abs diff:", (y4[:2].float() - y2.float()).abs().max().item())
