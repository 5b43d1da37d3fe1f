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

Checks (two optimizer steps, SGD lr 1e-4; gradients recorded at each step):
  * both ranks end with bit-identical parameters;
  * the all-reduced gradients equal one process accumulating the same
    per-rank micro-batches (grad_accumulation_factor = ranks x accum).  Step 1
    starts from identical parameters, so only the order of the final fp32
    sums differs: normwise 1e-5 per tensor in bf16 (5e-4 for the library
    GRU, whose bf16 solver is chosen per process); 1e-4 in fp32, whose
    weight-gradient GEMMs split K over fp32 atomics (a rerun of the same
    process differs by up to 2e-5).  Step 2 starts from parameters that
    differ in the last fp32 bit: 5e-4 in bf16 (measured up to 2.1e-4, the
    first ConvBlock's weight, a sum over every (frame, bin) position) for
    every gradient except the rel-pos biases and linear_pos, batch
    sums cancelling to ~1e-3 of their terms that amplify flipped bf16
    roundings of their inputs (5e-3; measured 6.5e-5 .. 2.3e-3); 1e-3 in
    fp32, where those gradients measured 2.9e-4;
  * a single-process run on the concatenated batch: in bf16 a gradient that
    is reduced over the batch INSIDE the step and stored in bf16 — the shared
    positional projection p_k's (a bf16 activation under autocast, as in the
    reference) — is rounded once per batch split, bounded by the bf16 step
    2^-8 (normwise 1e-2; measured 8.5e-3 for linear_pos.weight); in fp32 the
    rel-pos bias / linear_pos gradients are batch sums that cancel to ~1e-3
    of their terms, 1e-3 (measured 3e-4)."""
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
        grads = None  # one {name: gradient} per optimizer step

        def compute_forward(self, batch, stage):
            hp = self.hparams
            self.hparams = {"compute_features": hp["compute_features"], "normalize": lambda f, l, epoch: f,
                            "augmentation": lambda f: f}
            try:
                return super().compute_forward(batch, stage)
            finally:
                self.hparams = hp

        def check_gradients(self, loss):
            g = {}
            for mname, m in self.modules.items():
                inner = m.module if hasattr(m, "module") else m
                for n, p in inner.named_parameters():
                    if p.grad is not None:
                        g[f"{mname}.{n}"] = p.grad.detach().float().cpu().clone()
            self.grads = (self.grads or []) + [g]
            return super().check_gradients(loss)

    mods, hp = BT.build_modules(layers=2, dropout=0.0, fused_head=fused)
    hp = {k: (v.to(dev) if hasattr(v, "to") else v) for k, v in hp.items()}
    b = DDPTestBrain(modules=mods, opt_class=lambda p: torch.optim.SGD(p, lr=1e-4), hparams=hp, run_opts=run_opts)
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


def _run(brain, dev, accum, half=None, steps=2, split=None):
    """`steps` optimizer steps of `accum` micro-batches (a second step also
    catches parameters that never receive a gradient: DDP without
    find_unused_parameters raises on the next forward).  split = world: the
    single-process reference of a DDP run — every micro-batch cut into the
    ranks' parts, fed one after another (grad_accumulation_factor = world x
    accum)."""
    for micro in range(steps * accum):
        batch = _batch(dev, micro)
        if half is not None:
            batch = [t[half] for t in batch]
        if split:
            per = B_ALL // split
            for r in range(split):
                brain.fit_batch([t[r * per:(r + 1) * per] for t in batch])
        else:
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
    assert set(p0) == set(p1) and len(g0) == len(g1) == 2
    for a, b in zip(g0, g1):  # the all-reduced gradients are the same on both ranks
        assert set(a) == set(b) and all(torch.equal(a[k], b[k]) for k in a)
    for k in p0:
        assert torch.equal(p0[k], p1[k]), f"ranks differ: {k}"
    def single_run(accum_factor, split):
        ro = {"device": str(dev), "auto_mix_prec": "bf16" if fused else False, "max_grad_norm": 0.0,
              "grad_accumulation_factor": accum_factor}
        b = _brain(dev, fused, ro)
        _run(b, dev, accum, split=split)
        return b.grads, _params(b)

    def rel(a, b):
        return ((a.double() - b.double()).norm() / b.double().norm().clamp_min(1e-30)).item()

    # gradients that are batch sums cancelling to ~1e-3 of their terms (the
    # rel-pos biases, the shared positional projection): they amplify
    # last-bit differences of their inputs, and only they get `loose`
    cancelling = ("pos_bias_u", "pos_bias_v", "linear_pos")

    def compare(ref_grads, ref_params, tols, what, loose=None):
        assert len(ref_grads) == len(g0) == 2
        for step, (gs, gr, tol0) in enumerate(zip(g0, ref_grads, tols)):
            assert set(gr) == set(gs), set(gr) ^ set(gs)
            assert len(gr) > 50
            worst = sorted((rel(gs[k], gr[k]), k) for k in gr)
            print(f"step {step + 1} worst DDP vs {what}:", worst[-3:])
            # the library GRU (MIOpen, bf16 under autocast) picks its solver per
            # process: its bf16 gradients differ across processes at the bf16
            # rounding level (measured 9.4e-5) though a rerun in one process is
            # bit-stable
            def tol_of(k):
                tol = tol0
                if loose is not None and loose[step] is not None and any(c in k for c in cancelling):
                    tol = loose[step]
                return max(tol, 5e-4) if fused and k.startswith("dec.") else tol
            bad = [(e, k, tol_of(k)) for e, k in worst if e > tol_of(k)]
            assert not bad, f"step {step + 1}: DDP vs {what}: gradients beyond their bound: {bad}"
        for k in ref_params:
            d = (p0[k] - ref_params[k]).abs().max().item()
            assert d <= 1e-4 * max(ref_params[k].abs().max().item(), 1e-3), f"{k}: parameters {d:.2e}"

    # the same per-rank micro-batches accumulated in one process
    ga, pa = single_run(world * accum, world)
    gb, _ = single_run(world * accum, world)
    print("single-process rerun noise, step 1 / 2:",
          [max(rel(x[k], y[k]) for k in x) for x, y in zip(ga, gb)])
    # step 1 starts from identical parameters: only the order of the final
    # fp32 sums differs (plus, fp32, the split-K atomics of the weight-gradient
    # GEMMs).  Step 2 starts from parameters that differ in the last fp32 bit,
    # which the bf16 casts turn into occasional flipped bf16 roundings; the
    # rel-pos bias and linear_pos gradients are batch sums that cancel to
    # ~1e-3 of their terms and amplify those flips (as in the concatenated-
    # batch comparison below): measured 6.5e-5 .. 2.3e-3 from one Fbank
    # kernel's rounding to the next, while a single-process rerun is
    # bit-stable (~5e-8)
    compare(ga, pa, (1e-5, 5e-4) if fused else (1e-4, 1e-3), "single-process accumulation of the ranks' micro-batches",
            loose=(None, 5e-3) if fused else None)
    # the concatenated batch: the bf16 batch-reduced p_k gradient as above
    # (1e-2); fp32, the rel-pos bias and linear_pos gradients are batch sums
    # that cancel to ~1e-3 of their terms, so 2+2 vs 4-row ordering shows at
    # ~3e-4 normwise
    compare(*single_run(accum, None), (1e-2, 1e-2) if fused else (1e-3, 1e-3), "single-process concatenated batch")
