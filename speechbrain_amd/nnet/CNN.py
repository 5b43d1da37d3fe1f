"""Drop-in for the Conv2d wrapper of speechbrain.nnet.CNN (CNN.py:504-722):
same constructor and state_dict key (conv.weight / conv.bias).  Inside a
ConvBlock the convolution runs fused with its LayerNorm and LeakyReLU
(lobes.models.convolution); standalone, forward() is the reference's
(B, T, F[, C]) → (B, T', F', C_out) convolution (CNN.py:616-657) on the HIP
im2col kernels + the MFMA GEMM, differentiable: "same" reflect with
dilation 1 on the ConvBlock path (_autograd.ConvBlockFn without norm and
activation); any other stride / dilation / groups / padding ("same" with
every padding_mode, "valid", "causal", get_padding_elem :1459-1481) and
skip_transpose on sbk_im2col_x / sbk_col2im_x (_autograd.Conv2dXFn)."""
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

    _MODES = {"reflect": 0, "constant": 1, "zeros": 1, "replicate": 2, "circular": 3}

    def _geometry(self, Ti, Fi):
        """Leading / trailing pads per axis and the pad mode of the reference's
        forward (CNN.py:624-640): "same" pads get_padding_elem per side with
        padding_mode (_manage_padding :659-691, whose L_in is the channel
        count — for stride 1 the pad is d (k - 1) / 2 whatever it is), "causal"
        zero-pads (k[0] - 1) · d[1] before the frequency axis (F.pad's last
        pair but one), "valid" none."""
        (kf, kt), (sf, st), (df, dt) = self.kernel_size, self.stride, self.dilation
        mode = 1
        pt0 = pt1 = pf0 = pf1 = 0
        if self.padding == "same":
            pt0 = pt1 = get_padding_elem(self.in_channels, st, kt, dt)[0]
            pf0 = pf1 = get_padding_elem(self.in_channels, sf, kf, df)[0]
            if self.padding_mode not in self._MODES:
                raise NotImplementedError(f"Conv2d padding_mode={self.padding_mode!r}")
            mode = self._MODES[self.padding_mode]
            if mode == 0 and (pt0 >= Ti or pf0 >= Fi):
                raise ValueError("Conv2d: reflect padding needs more frames / bins than the padding")
        elif self.padding == "causal":
            pf0 = (kf - 1) * dt
        elif self.padding != "valid":
            raise ValueError("Padding must be 'same','valid' or 'causal'. Got " + self.padding)
        To = (Ti + pt0 + pt1 - dt * (kt - 1) - 1) // st + 1
        Fo = (Fi + pf0 + pf1 - df * (kf - 1) - 1) // sf + 1
        if To <= 0 or Fo <= 0:
            raise ValueError(f"Conv2d: input ({Ti}, {Fi}) smaller than the dilated kernel")
        return (kt, kf, st, sf, dt, df, pt0, pf0, To, Fo, mode)

    def forward(self, x):
        """CNN.py:616-657: x (B, T, F, C) — or (B, T, F) for a 3-D input_shape,
        or with skip_transpose the torch layout (B, C, H, W) — → (B, T', F',
        C_out) ((B, T', F') when C_out = 1 and the input was 3-D, the
        reference's squeeze(1); (B, C_out, H', W') with skip_transpose).  Any
        stride, dilation, groups, padding ("same" with any padding_mode,
        "valid", "causal") on the HIP im2col kernels + the MFMA GEMM, per
        group."""
        if self.skip_transpose:
            # the conv's (kernel[0], kernel[1]) run over (H, W) = dims (2, 3):
            # as (B, W, H, C) that is this path's (B, T, F, C)
            sq = x.dim() == 3  # (B, H, W): the reference's unsqueeze(1) / squeeze(1)
            if sq:
                x = x.unsqueeze(1)
            y = self._conv(x.permute(0, 3, 2, 1)).permute(0, 3, 2, 1)
            return y.squeeze(1) if sq and y.shape[1] == 1 else y
        squeeze = x.dim() == 3
        if squeeze:
            x = x.unsqueeze(-1)
        y = self._conv(x)
        if squeeze and y.shape[-1] == 1:
            y = y.squeeze(-1)
        return y

    def _conv(self, x):
        if x.shape[-1] != self.in_channels:
            raise ValueError(f"Conv2d: {x.shape[-1]} input channels, expected {self.in_channels}")
        dtype = _enc.compute_dtype()
        cv = self.conv
        xin = x if (x.dtype == dtype or self.in_channels == 1) else A.to_dtype(x, dtype)
        if xin.dtype not in (torch.float32, torch.bfloat16):
            xin = xin.float()
        (kf, kt), (sf, st) = self.kernel_size, self.stride
        general = (self.groups != 1 or self.dilation != (1, 1) or self.padding != "same"
                   or self.padding_mode != "reflect")
        if not general:
            # "same" reflect, dilation 1: the ConvBlock path's kernels
            pt, pf = kt // 2 if st > 1 else (kt - 1) // 2, kf // 2 if sf > 1 else (kf - 1) // 2
            if pt >= x.shape[1] or pf >= x.shape[2]:
                raise ValueError("Conv2d: reflect padding needs more frames / bins than the padding")
            return A.ConvBlockFn.apply(xin, cv.weight, cv.bias, None, None, 1e-5, None, dtype, torch.float32,
                                       (kt, kf, st, sf, pt, pf))
        geom = self._geometry(x.shape[1], x.shape[2])
        G = self.groups
        if G == 1:
            return A.Conv2dXFn.apply(xin, cv.weight, cv.bias, dtype, torch.float32, geom)
        cig, cog = self.in_channels // G, cv.out_channels // G
        outs = []
        for gi in range(G):
            xg = xin[..., gi * cig:(gi + 1) * cig].contiguous()
            wg = cv.weight[gi * cog:(gi + 1) * cog]
            bg = cv.bias[gi * cog:(gi + 1) * cog] if cv.bias is not None else None
            outs.append(A.Conv2dXFn.apply(xg, wg, bg, dtype, torch.float32, geom))
        return torch.cat(outs, dim=-1)
