"""speechbrain/utils/distributed.py:107-172 (ddp_init_group): one process per
GPU, rank/world from the torchrun environment, backend "nccl" (= RCCL over
xGMI on ROCm) or "gloo" (CPU tests)."""
import logging
import os

import torch

logger = logging.getLogger(__name__)


def ddp_init_group(run_opts):
    """Initialise the process group when run_opts["distributed_launch"] is set.
    Raises ValueError for the reference's error cases (missing local_rank /
    RANK, too few GPUs, unavailable or unknown backend)."""
    if not run_opts.get("distributed_launch"):
        logger.info("distributed_launch flag is disabled, this experiment will be executed without DDP.")
        return
    if "local_rank" not in run_opts:
        raise ValueError("To use DDP backend, start your script with torchrun and --distributed_launch")
    backend = run_opts.get("distributed_backend", "nccl")
    if backend != "gloo" and run_opts["local_rank"] + 1 > torch.cuda.device_count():
        raise ValueError("Killing process\nNot enough GPUs available!")
    if os.environ.get("RANK", "") == "":
        raise ValueError("To use DDP backend, start your script with torchrun (RANK is not set)")
    rank = int(os.environ["RANK"])
    available = {"nccl": torch.distributed.is_nccl_available, "gloo": torch.distributed.is_gloo_available,
                 "mpi": torch.distributed.is_mpi_available}
    if backend not in available:
        raise ValueError(backend + " communcation protocol doesn't exist.")
    if not available[backend]():
        raise ValueError(f"{backend.upper()} is not supported in your machine.")
    if backend == "nccl":
        torch.cuda.set_device(run_opts["local_rank"])
    torch.distributed.init_process_group(backend=backend, rank=rank)
