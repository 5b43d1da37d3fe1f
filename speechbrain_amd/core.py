"""The Brain training step of the hot path:
speechbrain/core.py:882-932 (fit_batch), :951-994 (check_gradients),
:1238-1264 (_wrap_distributed), :1362-1392 (no_sync) and
speechbrain/utils/distributed.py:107-172 (ddp_init_group, here
utils/distributed.py).

Only the per-batch step is here — no data loaders, checkpointer, epoch loop
or logging (those stay the reference's; its Brain drives these modules
unchanged).  MI355X choices:
  * one process per GPU, DDP over RCCL (backend "nccl") with the gradient
    all-reduce overlapped with the backward; buckets of `bucket_cap_mb`
    (default 64 MB: the ~80 MB of Conformer-Transducer gradients go out in
    two large ring all-reduces over xGMI instead of four 25 MB ones);
    `gradient_as_bucket_view` so gradients live in the buckets (no copy);
  * mixed precision is bf16 autocast (same exponent range as fp32, so no
    GradScaler).  The reference's `--auto_mix_prec` (True) means fp16
    autocast + GradScaler; here True selects bf16 and says so in the log,
    and "fp16" is the reference's step exactly (fp16 autocast, GradScaler
    scale / unscale_ / step / update) with these modules computing in fp32
    (no fp16 kernels; _enc.compute_dtype) and library ops in fp16;
  * everything the modules compute runs on libsbk.so HIP kernels.
"""
import contextlib
import logging

import torch
from torch.nn.parallel import DistributedDataParallel as DDP

logger = logging.getLogger(__name__)


class Stage:
    """core.py:52-57."""
    TRAIN = 1
    VALID = 2
    TEST = 3


class Brain:
    """Per-batch training step of speechbrain.core.Brain.

    modules: dict of nn.Modules; opt_class: callable(params) -> optimizer;
    run_opts: device, distributed_launch, distributed_backend,
    auto_mix_prec (False | True/"bf16" | "fp16" + GradScaler), max_grad_norm (5.0),
    grad_accumulation_factor (1), nonfinite_patience (3),
    find_unused_parameters (False), bucket_cap_mb (64).
    """

    def __init__(self, modules=None, opt_class=None, hparams=None, run_opts=None):
        run_opts = dict(run_opts or {})
        self.device = run_opts.get("device", "cuda:0")
        self.distributed_launch = bool(run_opts.get("distributed_launch", False))
        self.distributed_backend = run_opts.get("distributed_backend", "nccl")
        amp = run_opts.get("auto_mix_prec", False)
        if amp is True:
            logger.warning("auto_mix_prec=True runs bf16 autocast on MI355X (the reference uses fp16 + GradScaler; "
                           "auto_mix_prec='fp16' runs that)")
        if amp == torch.float16:
            amp = "fp16"
        self.amp_dtype = {False: None, None: None, True: torch.bfloat16, "bf16": torch.bfloat16,
                          "fp16": torch.float16}[amp]
        # core.py:558 (GradScaler for the fp16 step)
        self.scaler = torch.amp.GradScaler("cuda") if self.amp_dtype == torch.float16 else None
        self.max_grad_norm = float(run_opts.get("max_grad_norm", 5.0))
        self.grad_accumulation_factor = int(run_opts.get("grad_accumulation_factor", 1))
        self.nonfinite_patience = int(run_opts.get("nonfinite_patience", 3))
        self.find_unused_parameters = bool(run_opts.get("find_unused_parameters", False))
        self.bucket_cap_mb = float(run_opts.get("bucket_cap_mb", 64))
        self.hparams = hparams
        self.opt_class = opt_class
        self.modules = torch.nn.ModuleDict(modules or {}).to(self.device)
        self.step = 0
        self.optimizer_step = 0
        self.nonfinite_count = 0
        self._wrap_distributed()
        self.optimizer = None
        if opt_class is not None:
            self.init_optimizers()

    # ------------------------------------------------------------------ setup
    def _wrap_distributed(self):
        """core.py:1238-1264: DDP around every module that has trainable parameters."""
        if not self.distributed_launch:
            return
        for name, module in self.modules.items():
            if any(p.requires_grad for p in module.parameters()):
                module = torch.nn.SyncBatchNorm.convert_sync_batchnorm(module)
                ids = None if self.distributed_backend == "gloo" else [torch.device(self.device)]
                self.modules[name] = DDP(module, device_ids=ids, find_unused_parameters=self.find_unused_parameters,
                                         bucket_cap_mb=self.bucket_cap_mb, gradient_as_bucket_view=True)

    def init_optimizers(self):
        self.optimizer = self.opt_class(self.modules.parameters())

    def zero_grad(self, set_to_none=False):
        """core.py:848-856 (zeros by default, as the reference)."""
        self.optimizer.zero_grad(set_to_none)

    @contextlib.contextmanager
    def no_sync(self, use=True):
        """core.py:1362-1392: suspend the DDP all-reduce of every module
        (gradient accumulation steps)."""
        if not use:
            yield
            return
        old = []
        for module in self.modules.values():
            if not hasattr(module, "require_backward_grad_sync"):
                break
            old.append(module.require_backward_grad_sync)
            module.require_backward_grad_sync = False
        try:
            yield
        finally:
            for module, value in zip(self.modules.values(), old):
                module.require_backward_grad_sync = value

    # ------------------------------------------------------------------- step
    def compute_forward(self, batch, stage):
        raise NotImplementedError

    def compute_objectives(self, predictions, batch, stage):
        raise NotImplementedError

    def on_fit_batch_end(self, batch, outputs, loss, should_step):
        pass

    def _autocast(self):
        if self.amp_dtype is None:
            return contextlib.nullcontext()
        return torch.autocast("cuda", dtype=self.amp_dtype)

    def fit_batch(self, batch):
        """core.py:882-932: forward, objective, backward (DDP all-reduce
        overlapped), gradient check + clip, optimizer step, zero_grad."""
        self.step += 1
        should_step = self.step % self.grad_accumulation_factor == 0
        with self._autocast():
            outputs = self.compute_forward(batch, Stage.TRAIN)
            loss = self.compute_objectives(outputs, batch, Stage.TRAIN)
        if self.scaler is not None:  # core.py:906-919: the fp16 step
            with self.no_sync(not should_step):
                self.scaler.scale(loss / self.grad_accumulation_factor).backward()
            if should_step:
                self.scaler.unscale_(self.optimizer)
                if self.check_gradients(loss):
                    self.scaler.step(self.optimizer)
                self.scaler.update()
                self.zero_grad()
                self.optimizer_step += 1
        else:
            with self.no_sync(not should_step):
                (loss / self.grad_accumulation_factor).backward()
            if should_step:
                if self.check_gradients(loss):
                    self.optimizer.step()
                self.zero_grad()
                self.optimizer_step += 1
        self.on_fit_batch_end(batch, outputs, loss, should_step)
        return loss.detach()

    def check_gradients(self, loss):
        """core.py:951-994: skip the step on a non-finite loss (up to
        nonfinite_patience times), then clip the global gradient norm."""
        if not torch.isfinite(loss):
            self.nonfinite_count += 1
            logger.warning(f"Loss is {loss}.")
            if self.nonfinite_count > self.nonfinite_patience:
                raise ValueError("Loss is not finite and patience is exhausted. To debug, wrap `fit()` with "
                                 "autograd's `detect_anomaly()`")
            logger.warning("Patience not yet exhausted, ignoring this batch.")
            return False
        if self.max_grad_norm > 0.0:
            torch.nn.utils.clip_grad_norm_((p for p in self.modules.parameters()), self.max_grad_norm)
        return True

    def evaluate_batch(self, batch, stage):
        """core.py:996-1021."""
        with torch.no_grad(), self._autocast():
            out = self.compute_forward(batch, stage=stage)
            loss = self.compute_objectives(out, batch, stage=stage)
        return loss.detach()
