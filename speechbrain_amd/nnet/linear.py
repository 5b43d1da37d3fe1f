"""Drop-in for speechbrain.nnet.linear.Linear (linear.py:15-76) on the MFMA GEMM
(state_dict keys: w.weight, w.bias)."""
import torch

from .. import _autograd as A
from .. import _enc


class Linear(torch.nn.Module):
    def __init__(self, n_neurons, input_shape=None, input_size=None, bias=True, combine_dims=False):
        super().__init__()
        self.combine_dims = combine_dims
        if input_shape is None and input_size is None:
            raise ValueError("Expected one of input_shape or input_size")
        if input_size is None:
            input_size = input_shape[-1]
            if len(input_shape) == 4 and self.combine_dims:
                input_size = input_shape[2] * input_shape[3]
        self.w = torch.nn.Linear(input_size, n_neurons, bias=bias)
        self._wc = _enc.WeightCache()

    def kernel_weight(self, dtype):
        if dtype == torch.float32:
            return self.w.weight.detach()
        return self._wc.get("bf16", [self.w.weight], lambda: _enc.cast_bf16(self.w.weight.detach().contiguous()))

    def forward(self, x):
        if x.ndim == 4 and self.combine_dims:
            x = x.reshape(x.shape[0], x.shape[1], x.shape[2] * x.shape[3])
        dtype = _enc.compute_dtype()
        shp = x.shape
        if A.needs_grad(self, x):
            y = A.linear(x.reshape(-1, shp[-1]), self.w.weight, self.w.bias, dtype, self._wc, "t_w")
            return y.view(*shp[:-1], -1)
        a = _enc.to_compute(x.reshape(-1, shp[-1]), dtype)
        b = self.w.bias.detach() if self.w.bias is not None else None
        return _enc.gemm(a, self.kernel_weight(dtype), bias=b).view(*shp[:-1], -1)
