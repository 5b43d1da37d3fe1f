"""Brain's fp16 mixed-precision step (the reference's --auto_mix_prec,
speechbrain/core.py:558, :905-919: torch.cuda.amp.autocast + GradScaler
scale / unscale_ / step / update) over the config-4 module set at reduced
size (ConvolutionFrontEnd + 2-layer Conformer + TN / PN + GRU + the
transducer head).  The speechbrain_amd modules compute in fp32 under fp16
autocast (no fp16 kernels); the library GRU runs in fp16.  So the fp16
step's unscaled gradients equal the fp32 step's up to the GRU's fp16
rounding (normwise 2e-2 per tensor; measured values printed), the scaler
really scales (its scale grows from 2^16), and the loss matches."""
import pytest
import torch

pytestmark = pytest.mark.gpu

B, SECONDS, UMAX = 2, 2.0, 6


def _batch(dev):
    import bench_train as BT
    g = torch.Generator().manual_seed(7)
    wavs = 0.1 * torch.randn(B, int(BT.SR * SECONDS), generator=g)
    U = torch.tensor([6, 4])
    tokens = torch.randint(1, BT.V, (B, UMAX), generator=g)
    tokens[torch.arange(UMAX)[None, :] >= U[:, None]] = 0
    return [t.to(dev) for t in (wavs, torch.tensor([1.0, 0.8]), torch.nn.functional.pad(tokens, (1, 0)), tokens,
                                U.float() / UMAX)]


def _run(dev, amp):
    import bench_train as BT

    class GradBrain(BT.brain_class(False)):
        grads = None

        def compute_forward(self, batch, stage):
            hp = self.hparams
            self.hparams = {"compute_features": hp["compute_features"], "normalize": lambda f, l, epoch: f,
                            "augmentation": lambda f: f}
            try:
                return super().compute_forward(batch, stage)
            finally:
                self.hparams = hp

        def check_gradients(self, loss):
            self.grads = {n: p.grad.detach().float().clone() for n, p in self.modules.named_parameters()
                          if p.grad is not None}
            return super().check_gradients(loss)

    mods, hp = BT.build_modules(layers=2, dropout=0.0, fused_head=False)
    hp = {k: (v.to(dev) if hasattr(v, "to") else v) for k, v in hp.items()}
    b = GradBrain(modules=mods, opt_class=lambda p: torch.optim.SGD(p, lr=1e-4), hparams=hp,
                  run_opts={"device": str(dev), "auto_mix_prec": amp, "max_grad_norm": 0.0})
    for m in b.modules.values():
        m.train()
    loss = b.fit_batch(_batch(dev))
    return b, float(loss)


def test_brain_fp16_amp_step_matches_fp32(dev):
    b16, l16 = _run(dev, "fp16")
    b32, l32 = _run(dev, False)
    assert b16.scaler is not None and b16.scaler.get_scale() >= 65536.0
    assert abs(l16 - l32) <= 1e-2 * abs(l32), (l16, l32)
    assert set(b16.grads) == set(b32.grads) and len(b16.grads) > 50
    worst = []
    for k, g32 in b32.grads.items():
        g16 = b16.grads[k]
        assert torch.isfinite(g16).all(), k
        e = ((g16.double() - g32.double()).norm() / g32.double().norm().clamp_min(1e-30)).item()
        worst.append((e, k))
    worst.sort()
    print("\nfp16 AMP vs fp32, worst gradients:", worst[-3:], "loss", l16, l32)
    assert worst[-1][0] <= 2e-2, worst[-3:]
