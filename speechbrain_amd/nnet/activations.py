"""Drop-in for speechbrain.nnet.activations.Swish (activations.py:111-142).

Inside the Conformer the Swish is fused into GEMM / depthwise-conv epilogues;
the standalone module runs the elementwise HIP kernel."""
import torch

from .._lib import check, lib, ptr, require_device, stream_of


class Swish(torch.nn.Module):
    """x * sigmoid(beta * x)."""

    def __init__(self, beta=1):
        super().__init__()
        self.beta = beta
        self.sigmoid = torch.nn.Sigmoid()

    def forward(self, x):
        require_device(x)
        x = x.float().contiguous()
        out = torch.empty_like(x)
        check(lib().sbk_swish(ptr(x), ptr(out), x.numel(), float(self.beta), stream_of(x)), "sbk_swish")
        return out
