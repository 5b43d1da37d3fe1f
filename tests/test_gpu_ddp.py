"""Brain DDP over the real modules on the GPU:
speechbrain/core.py:1238-1264 (_wrap_distributed), :1362-1392 (no_sync),
:882-932 (fit_batch), speechbrain/utils/distributed.py:107-172.

Two ranks are spawned on the one GPU of the box (gloo over device tensors:
RCCL refuses two ranks on one device) and run Brain.fit_batch over the config-4
module set at reduced size — ConvolutionFrontEnd(64, 32) + a 2-layer
Conformer (d = 256) + TN / PN projections + GRU prediction net + the
transducer head (fused TransducerHeadLinear under bf16 autocast, the fp32
materialised chain without) — so the custom autograd Functions, the fused
head's weight gradient and gradient_as_bucket_view buckets all pass through
DDP.  Each rank takes half of a 4-utterance batch; with accumulation 2 the
first micro-batch runs under no_sync.

Checks (after two optimizer steps): both ranks end with bit-identical
parameters, and the all-reduced gradients of the last step equal a
single-process run on the concatenated batches.  Every
per-row computation of the path is independent of the other rows of the
batch, so the two differ only in the fp32 summation order of the weight /
bias reductions (split-K atomics): normwise 1e-4 per tensor."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

B_ALL, SECONDS, UMAX = 4, 2.0, 8


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _batch(dev, micro):
    import bench_train as BT
    g = torch.Generator().manual_seed(100 + micro)
    wavs = 0.1 * torch.randn(B_ALL, int(BT.SR * SECONDS), generator=g)
    wav_lens = torch.tensor([1.0, 0.8, 0.9, 0.7])
    U = torch.tensor([8, 5, 7, 6])
    tokens = torch.randint(1, BT.V, (B_ALL, UMAX), generator=g)
    tokens[torch.arange(UMAX)[None, :] >= U[:, None]] = 0
    tokens_bos = torch.nn.functional.pad(tokens, (1, 0))
    return [t.to(dev) for t in (wavs, wav_lens, tokens_bos, tokens, U.float() / UMAX)]


def _brain(dev, fused, run_opts):
    """bench_train's transducer Brain without InputNormalization / SpecAugment
    (host-random and batch-statistics dependent: not comparable across
    batch splits), dropout 0, plain SGD; check_gradients snapshots the
    (all-reduced) gradients before clipping."""
    import bench_train as BT

    base = BT.brain_class(fused)

    class DDPTestBrain(base):
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
            self.grads = {}
            for mname, m in self.modules.items():
                inner = m.module if hasattr(m, "module") else m
                for n, p in inner.named_parameters():
                    if p.grad is not None:
                        self.grads[f"{mname}.{n}"] = p.grad.detach().float().cpu().clone()
            return super().check_gradients(loss)

    mods, hp = BT.build_modules(layers=2, dropout=0.0, fused_head=fused)
    hp = {k: (v.to(dev) if hasattr(v, "to") else v) for k, v in hp.items()}
    b = DDPTestBrain(modules=mods, opt_class=lambda p: torch.optim.SGD(p, lr=0.05), hparams=hp, run_opts=run_opts)
    for m in b.modules.values():
        m.train()
    return b


def _params(brain):
    out = {}
    for mname, m in brain.modules.items():
        inner = m.module if hasattr(m, "module") else m
        for n, p in inner.named_parameters():
            out[f"{mname}.{n}"] = p.detach().float().cpu().clone()
    return out


def _run(brain, dev, accum, half=None, steps=2):
    """`steps` optimizer steps of `accum` micro-batches (a second step also
    catches parameters that never receive a gradient: DDP without
    find_unused_parameters raises on the next forward)."""
    for micro in range(steps * accum):
        batch = _batch(dev, micro)
        if half is not None:
            batch = [t[half] for t in batch]
        brain.fit_batch(batch)


def _worker(rank, world, port, out, fused, accum):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    if root not in sys.path:
        sys.path.insert(0, root)
    import torch.distributed as dist
    from speechbrain_amd.utils.distributed import ddp_init_group
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    run_opts = {"device": str(dev), "distributed_launch": True, "distributed_backend": "gloo", "local_rank": 0,
                "auto_mix_prec": "bf16" if fused else False, "max_grad_norm": 0.0, "grad_accumulation_factor": accum}
    ddp_init_group(run_opts)
    brain = _brain(dev, fused, run_opts)
    assert all(hasattr(m, "require_backward_grad_sync") for m in brain.modules.values()
               if any(p.requires_grad for p in m.parameters()))
    per = B_ALL // world
    _run(brain, dev, accum, slice(rank * per, (rank + 1) * per))
    torch.cuda.synchronize()
    out[rank] = (_params(brain), brain.grads)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("fused,accum", [(True, 1), (True, 2), (False, 1)])
def test_brain_ddp_real_modules(dev, fused, accum):
    world = 2
    ctx = mp.get_context("spawn")
    mgr = ctx.Manager()
    out = mgr.dict()
    mp.start_processes(_worker, args=(world, _free_port(), out, fused, accum), nprocs=world, join=True,
                       start_method="spawn")
    (p0, g0), (p1, g1) = out[0], out[1]
    assert set(p0) == set(p1) and set(g0) == set(g1)
    for k in p0:
        assert torch.equal(p0[k], p1[k]), f"ranks differ: {k}"
    run_opts = {"device": str(dev), "auto_mix_prec": "bf16" if fused else False, "max_grad_norm": 0.0,
                "grad_accumulation_factor": accum}
    single = _brain(dev, fused, run_opts)
    _run(single, dev, accum)
    gs, ps = single.grads, _params(single)
    assert set(gs) == set(g0), set(gs) ^ set(g0)
    assert len(gs) > 50
    worst = []
    for k, ref in gs.items():
        e = ((g0[k].double() - ref.double()).norm() / ref.double().norm().clamp_min(1e-30)).item()
        worst.append((e, k))
        assert e <= 1e-4, f"{k}: DDP vs single-process gradient {e:.2e}"
    print("worst DDP-vs-single gradients:", sorted(worst)[-4:])
    for k in ps:
        d = (p0[k] - ps[k]).abs().max().item()
        assert d <= 1e-4 * max(ps[k].abs().max().item(), 1e-3), f"{k}: parameters {d:.2e}"
