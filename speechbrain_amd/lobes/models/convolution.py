"""Drop-in for speechbrain.lobes.models.convolution (ConvolutionFrontEnd,
ConvBlock; convolution.py:12-175) with each block as ONE fused kernel:
reflect-padded 3x3 stride-2 Conv2d → LayerNorm over (freq, channels) →
LeakyReLU.  Cin = 1 runs on the VALU (9 taps), Cin % 8 == 0 as an implicit
GEMM on MFMA (bf16 under autocast, exact f32 otherwise).  State_dict keys
match the reference (convblock_i.convs.conv_0.conv.*, .norm_0.norm.*)."""
import torch
import torch.nn as nn

from ... import _autograd as A
from ... import _enc
from ...nnet.CNN import Conv2d
from ...nnet.normalization import LayerNorm

_f32 = torch.float32


class _Named(nn.Module):
    """Ordered container with explicit layer names (nnet/containers.py Sequential keys)."""

    def add(self, name, module):
        self.add_module(name, module)
        return module


class ConvBlock(nn.Module):
    def __init__(self, num_layers, out_channels, input_shape, kernel_size=3, stride=1, dilation=1, residual=False,
                 conv_module=Conv2d, activation=torch.nn.LeakyReLU, norm=None, dropout=0.1, conv_bias=True,
                 padding="same", conv_init=None):
        super().__init__()
        self.convs = _Named()
        shape = tuple(input_shape)
        for i in range(num_layers):
            conv = self.convs.add(f"conv_{i}", conv_module(out_channels=out_channels, kernel_size=kernel_size,
                                                             input_shape=shape,
                                                             stride=stride if i == num_layers - 1 else 1,
                                                             dilation=dilation, bias=conv_bias, padding=padding,
                                                             conv_init=conv_init))
            shape = conv.out_shape(shape)
            if norm is not None:
                self.convs.add(f"norm_{i}", norm(input_shape=shape))
            self.convs.add(f"act_{i}", activation())
            self.convs.add(f"dropout_{i}", torch.nn.Dropout(dropout))
        self.out_shape = shape
        self.num_layers = num_layers
        self.reduce_conv = None
        self.drop = None
        if residual:
            raise NotImplementedError("residual ConvBlock is not on the accelerated path")

    def _check(self):
        c = self.convs
        act = getattr(c, "act_0")
        norm = getattr(c, "norm_0", None)
        if (self.num_layers != 1 or not c.conv_0.fusable() or not isinstance(norm, LayerNorm)
                or not isinstance(act, nn.LeakyReLU)):
            raise NotImplementedError("fused ConvBlock supports 1 x (Conv2d k3 s2 reflect + LayerNorm + LeakyReLU)")

    def params(self):
        """(conv weight, bias, ln weight, ln bias, ln eps, leaky slope) of the fused block."""
        c = self.convs
        conv = c.conv_0.conv
        ln = c.norm_0.norm
        bias = conv.bias.detach() if conv.bias is not None else None
        return (conv.weight.detach().contiguous(), bias, ln.weight.detach(), ln.bias.detach(), ln.eps,
                c.act_0.negative_slope)

    def wperm(self, dtype):
        """Weights as (Cout, time, freq, Cin) in the compute dtype (implicit-GEMM B operand)."""
        conv = self.convs.conv_0.conv
        if not hasattr(self, "_wc"):
            self._wc = _enc.WeightCache()

        def make():
            w = conv.weight.detach().permute(0, 3, 2, 1).contiguous()  # (Cout, time, freq, Cin)
            return _enc.cast_bf16(w) if dtype == torch.bfloat16 else w
        return self._wc.get(("wperm", dtype), [conv.weight], make)

    def run(self, x, out_dtype):
        self._check()
        c = self.convs
        conv = c.conv_0.conv
        ln = c.norm_0.norm
        slope = c.act_0.negative_slope
        bias = conv.bias.detach() if conv.bias is not None else None
        if conv.in_channels == 1:
            if x.dim() == 4:
                x = x[..., 0]
            return _enc.conv_block_c1(x.float().contiguous(), conv.weight.detach().contiguous(), bias,
                                      ln.weight.detach(), ln.bias.detach(), ln.eps, slope, out_dtype)
        if x.dim() == 3:
            x = x.unsqueeze(-1)
        dtype = x.dtype if x.dtype == torch.bfloat16 else _f32
        wp = self.wperm(dtype)
        return _enc.conv_block_mfma(x.contiguous(), wp, bias, ln.weight.detach(), ln.bias.detach(), ln.eps, slope,
                                    out_dtype)

    def train_run(self, x, dtype, out_dtype):
        """Differentiable block (training path): im2col + MFMA GEMM + (freq x
        chan) LayerNorm + LeakyReLU (ConvBlockFn) + Dropout."""
        self._check()
        c = self.convs
        conv = c.conv_0.conv
        ln = c.norm_0.norm
        if x.dim() == 3:
            x = x.unsqueeze(-1)
        if x.dtype != dtype and conv.in_channels > 1:
            x = A.to_dtype(x, dtype)
        y = A.ConvBlockFn.apply(x, conv.weight, conv.bias, ln.weight, ln.bias, ln.eps, c.act_0.negative_slope, dtype,
                                out_dtype)
        return A.dropout(y, c.dropout_0.p, self.training)

    def wants_train_path(self, x):
        return A.needs_grad(self, x) or (self.training and self.convs.dropout_0.p > 0)

    def forward(self, x):
        if self.wants_train_path(x):
            return self.train_run(x, _enc.compute_dtype(), _f32)
        return self.run(x, _f32)


class ConvolutionFrontEnd(nn.Module):
    """convolution.py:12-84 (a Sequential of ConvBlocks)."""

    def __init__(self, input_shape, num_blocks=3, num_layers_per_block=5, out_channels=[128, 256, 512],
                 kernel_sizes=[3, 3, 3], strides=[1, 2, 2], dilations=[1, 1, 1], residuals=[True, True, True],
                 conv_module=Conv2d, activation=torch.nn.LeakyReLU, norm=LayerNorm, dropout=0.1, conv_bias=True,
                 padding="same", conv_init=None):
        super().__init__()
        shape = tuple(input_shape)
        self.block_names = []
        block_out_shapes = []
        for i in range(num_blocks):
            # The reference's Sequential infers each block's input shape by a
            # dummy forward through the previous blocks in training mode
            # (nnet/containers.py get_output_shape), whose Dropout layers draw
            # from the CPU generator.  Consume the same draws so that a seeded
            # construction gives bit-identical initial weights.
            if i > 0:
                with torch.no_grad():
                    for s in block_out_shapes:
                        torch.nn.functional.dropout(torch.zeros(s), dropout, True)
            blk = ConvBlock(num_layers=num_layers_per_block, out_channels=out_channels[i],
                            input_shape=shape, kernel_size=kernel_sizes[i], stride=strides[i],
                            dilation=dilations[i], residual=residuals[i], conv_module=conv_module,
                            activation=activation, norm=norm, dropout=dropout, conv_bias=conv_bias,
                            padding=padding, conv_init=conv_init)
            self.add_module(f"convblock_{i}", blk)
            self.block_names.append(f"convblock_{i}")
            shape = blk.out_shape
            block_out_shapes.append(shape)

    def _fusable2(self, x, dtype):
        if dtype != torch.bfloat16 or len(self.block_names) != 2 or x.dim() != 3:
            return False
        b1, b2 = (getattr(self, n) for n in self.block_names)
        for blk in (b1, b2):
            blk._check()
        c1, c2 = b1.convs.conv_0.conv, b2.convs.conv_0.conv
        return (c1.in_channels == 1 and c1.out_channels == 64 and c2.in_channels == 64
                and c2.out_channels % 16 == 0 and c2.out_channels <= 32 and (x.shape[2] - 1) // 2 + 1 <= 40)

    def run(self, x, last_dtype):
        """Intermediate block outputs in the compute dtype, the last in `last_dtype`."""
        dtype = _enc.compute_dtype()
        blocks = [getattr(self, n) for n in self.block_names]
        if any(b.wants_train_path(x) for b in blocks):
            n = len(blocks)
            for i, b in enumerate(blocks):
                x = b.train_run(x, dtype, last_dtype if i == n - 1 else dtype)
            return x
        if self._fusable2(x, dtype):
            # both blocks in one kernel: the block-1 activation stays in LDS
            b1, b2 = (getattr(self, n) for n in self.block_names)
            return _enc.conv_frontend2(x.float().contiguous(), b1.params(), b2.params(), b2.wperm(dtype),
                                       last_dtype)
        n = len(self.block_names)
        for i, name in enumerate(self.block_names):
            x = getattr(self, name).run(x, last_dtype if i == n - 1 else dtype)
        return x

    def forward(self, x):
        return self.run(x, _enc.compute_dtype())
