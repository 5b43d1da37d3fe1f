"""Drop-in for the Conv2d wrapper of speechbrain.nnet.CNN (CNN.py:504-722):
same constructor and state_dict key (conv.weight / conv.bias).  Inside a
ConvBlock the convolution runs fused with its LayerNorm and LeakyReLU
(lobes.models.convolution); standalone, forward() is the reference's
(B, T, F[, C]) → (B, T', F', C_out) convolution (CNN.py:616-657) on the HIP
im2col kernel + the MFMA GEMM (_autograd.ConvBlockFn without norm and
activation, so it is differentiable), with the "same"/reflect padding
(get_padding_elem :1459-1481) or "valid"."""
import math

import torch
import torch.nn as nn

from .. import _autograd as A
from .. import _enc


def get_padding_elem(L_in: int, stride: int, kernel_size: int, dilation: int):
    """CNN.py:1459-1481."""
    if stride > 1:
        return [math.floor(kernel_size / 2), math.floor(kernel_size / 2)]
    L_out = math.floor((L_in - dilation * (kernel_size - 1) - 1) / stride) + 1
    return [math.floor((L_in - L_out) / 2), math.floor((L_in - L_out) / 2)]


class Conv2d(nn.Module):
    def __init__(self, out_channels, kernel_size, input_shape=None, in_channels=None, stride=(1, 1), dilation=(1, 1),
                 padding="same", groups=1, bias=True, padding_mode="reflect", skip_transpose=False, weight_norm=False,
                 conv_init=None):
        super().__init__()
        if isinstance(kernel_size, int):
            kernel_size = (kernel_size, kernel_size)
        if isinstance(stride, int):
            stride = (stride, stride)
        if isinstance(dilation, int):
            dilation = (dilation, dilation)
        self.kernel_size = kernel_size
        self.stride = stride
        self.dilation = dilation
        self.padding = padding
        self.padding_mode = padding_mode
        self.unsqueeze = False
        self.skip_transpose = skip_transpose
        if input_shape is None and in_channels is None:
            raise ValueError("Must provide one of input_shape or in_channels")
        if in_channels is None:
            in_channels = self._check_input(input_shape)
        self.in_channels = in_channels
        self.conv = nn.Conv2d(self.in_channels, out_channels, self.kernel_size, stride=self.stride, padding=0,
                              dilation=self.dilation, groups=groups, bias=bias)
        if conv_init == "kaiming":
            nn.init.kaiming_normal_(self.conv.weight)
        if weight_norm:
            raise NotImplementedError("weight_norm Conv2d is not on the accelerated path")
        self.groups = groups

    def _check_input(self, shape):
        if len(shape) == 3:
            self.unsqueeze = True
            in_channels = 1
        elif len(shape) == 4:
            in_channels = shape[3]
        else:
            raise ValueError("Expected 3d or 4d inputs. Got " + str(len(shape)))
        if not self.padding == "valid" and (self.kernel_size[0] % 2 == 0 or self.kernel_size[1] % 2 == 0):
            raise ValueError("The field kernel size must be an odd number. Got %s." % (self.kernel_size,))
        return in_channels

    def out_shape(self, shape):
        """(B, T, F[, C]) → (B, T', F', C_out) for the "same" geometry."""
        T, F = shape[1], shape[2]
        if self.padding == "same" and self.stride[0] > 1:
            Fo = (F - 1) // self.stride[0] + 1
            To = (T - 1) // self.stride[1] + 1
        elif self.padding == "same":
            Fo, To = F, T
        else:
            raise NotImplementedError("only padding='same' is on the accelerated path")
        return (shape[0], To, Fo, self.conv.out_channels)

    def fusable(self):
        return (self.kernel_size == (3, 3) and self.stride == (2, 2) and self.dilation == (1, 1)
                and self.padding == "same" and self.padding_mode == "reflect" and self.groups == 1
                and not self.skip_transpose)

    def forward(self, x):
        """CNN.py:616-657: x (B, T, F, C) — or (B, T, F) for a 3-D input_shape —
        → (B, T', F', C_out) ((B, T', F') when C_out = 1 and the input was 3-D,
        the reference's squeeze(1))."""
        if self.skip_transpose:
            raise NotImplementedError("Conv2d(skip_transpose=True): the accelerated path takes (B, T, F, C)")
        if self.groups != 1 or self.dilation != (1, 1):
            raise NotImplementedError("Conv2d: groups=1 and dilation 1 are on the accelerated path")
        (kf, kt), (sf, st) = self.kernel_size, self.stride
        if self.padding == "same":
            if self.padding_mode != "reflect":
                raise NotImplementedError("Conv2d 'same' padding: padding_mode='reflect' is on the accelerated path")
            # get_padding_elem: floor(k / 2) per side for stride > 1, (k - 1) / 2 at stride 1 (odd k)
            pt, pf = kt // 2 if st > 1 else (kt - 1) // 2, kf // 2 if sf > 1 else (kf - 1) // 2
        elif self.padding == "valid":
            pt = pf = 0
        else:
            raise NotImplementedError(f"Conv2d padding={self.padding!r}: 'same' (reflect) and 'valid' are on the "
                                      "accelerated path")
        squeeze = x.dim() == 3
        if squeeze:
            x = x.unsqueeze(-1)
        if x.shape[-1] != self.in_channels:
            raise ValueError(f"Conv2d: {x.shape[-1]} input channels, expected {self.in_channels}")
        if self.padding == "same" and (pt >= x.shape[1] or pf >= x.shape[2]):
            raise ValueError("Conv2d: reflect padding needs more frames / bins than the padding")
        dtype = _enc.compute_dtype()
        cv = self.conv
        xin = x if (x.dtype == dtype or self.in_channels == 1) else A.to_dtype(x, dtype)
        if xin.dtype not in (torch.float32, torch.bfloat16):
            xin = xin.float()
        y = A.ConvBlockFn.apply(xin, cv.weight, cv.bias, None, None, 1e-5, None, dtype, torch.float32,
                                (kt, kf, st, sf, pt, pf))
        if squeeze and y.shape[-1] == 1:
            y = y.squeeze(-1)
        return y
