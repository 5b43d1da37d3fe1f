"""Drop-in for speechbrain.lobes.models.convolution (ConvolutionFrontEnd,
ConvBlock; convolution.py:12-175).

The recipe's blocks (one reflect-padded 3x3 stride-2 Conv2d → LayerNorm over
(freq, channels) → LeakyReLU each) run as ONE fused kernel per block — Cin = 1
on the VALU (9 taps), Cin % 8 == 0 as an implicit GEMM on MFMA — or both
blocks in one (frontend2).  Every other configuration the reference accepts
(num_layers_per_block > 1, residual blocks with their 1x1 reduce_conv +
norm, any odd kernel and stride, norm=None; the defaults
ConvolutionFrontEnd(input_shape) constructs) runs layer by layer on im2col +
MFMA GEMM + wide LayerNorm + LeakyReLU (_autograd.ConvBlockFn), with or
without gradients.  State_dict keys and seeded initial weights match the
reference (convblock_i.convs.conv_j.conv.*, .norm_j.norm.*,
.reduce_conv.conv.conv.*, .reduce_conv.norm.norm.*)."""
import torch
import torch.nn as nn

from ... import _autograd as A
from ... import _enc
from ... import ops
from ...nnet.CNN import Conv2d
from ...nnet.normalization import LayerNorm

_f32 = torch.float32


class _Named(nn.Module):
    """Ordered container with explicit layer names (nnet/containers.py Sequential keys)."""

    def add(self, name, module):
        self.add_module(name, module)
        return module


def _dummy_dropouts(shapes, p):
    """The CPU-generator draws of the reference Sequential's shape inference
    (nnet/containers.py get_output_shape: a forward of zeros through the
    layers built so far, in training mode): one dropout per shape, in order."""
    with torch.no_grad():
        for shp in shapes:
            torch.nn.functional.dropout(torch.zeros(shp), p, True)


class ConvBlock(nn.Module):
    def __init__(self, num_layers, out_channels, input_shape, kernel_size=3, stride=1, dilation=1, residual=False,
                 conv_module=Conv2d, activation=torch.nn.LeakyReLU, norm=None, dropout=0.1, conv_bias=True,
                 padding="same", conv_init=None):
        super().__init__()
        self.convs = _Named()
        shape = tuple(input_shape)
        layer_shapes = []  # each layer's output shape (its dropout's input)
        for i in range(num_layers):
            # the Sequential infers conv_i's and norm_i's input shapes by a
            # dummy forward through layers 0..i-1, whose dropouts draw
            _dummy_dropouts(layer_shapes, dropout)
            conv = self.convs.add(f"conv_{i}", conv_module(out_channels=out_channels, kernel_size=kernel_size,
                                                             input_shape=shape,
                                                             stride=stride if i == num_layers - 1 else 1,
                                                             dilation=dilation, bias=conv_bias, padding=padding,
                                                             conv_init=conv_init))
            shape = conv.out_shape(shape)
            if norm is not None:
                _dummy_dropouts(layer_shapes, dropout)
                self.convs.add(f"norm_{i}", norm(input_shape=shape))
            self.convs.add(f"act_{i}", activation())
            self.convs.add(f"dropout_{i}", torch.nn.Dropout(dropout))
            layer_shapes.append(shape)
        self.out_shape = shape
        self.num_layers = num_layers
        self.layer_shapes = layer_shapes
        self.reduce_conv = None
        self.drop = None
        if residual:
            # convolution.py:158-168: 1x1 conv with the block's stride + norm, added before a dropout
            self.reduce_conv = _Named()
            self.reduce_conv.add("conv", conv_module(out_channels=out_channels, kernel_size=1,
                                                     input_shape=tuple(input_shape), stride=stride))
            self.reduce_conv.add("norm", norm(input_shape=self.reduce_conv.conv.out_shape(tuple(input_shape))))
            self.drop = torch.nn.Dropout(dropout)

    def dummy_draw_shapes(self):
        """Shapes of the dropouts a forward of this block draws, in order
        (the ConvolutionFrontEnd's shape inference of the next block)."""
        return list(self.layer_shapes) + ([self.out_shape] if self.reduce_conv is not None else [])

    def _layer(self, i):
        c = self.convs
        return getattr(c, f"conv_{i}"), getattr(c, f"norm_{i}", None), getattr(c, f"act_{i}"), getattr(c, f"dropout_{i}")

    def _fusable(self):
        """The recipe's block: one k3 s2 reflect Conv2d + LayerNorm + LeakyReLU (fused kernels)."""
        if self.num_layers != 1 or self.reduce_conv is not None:
            return False
        conv, norm, act, _ = self._layer(0)
        return conv.fusable() and isinstance(norm, LayerNorm) and isinstance(act, nn.LeakyReLU)

    def _check(self):
        if not self._fusable():
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
        if not self._fusable():
            return self.general_run(x, _enc.compute_dtype(), out_dtype)
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

    @staticmethod
    def _conv_ln(x, conv, norm, slope, dtype, out_dtype):
        """Conv2d "same" reflect → [LayerNorm] → [LeakyReLU] (ConvBlockFn)."""
        cv = conv.conv
        if conv.padding != "same" or conv.padding_mode != "reflect" or conv.groups != 1 or conv.skip_transpose:
            raise NotImplementedError("ConvBlock convolutions: padding='same', reflect, groups=1")
        if conv.dilation != (1, 1):
            raise NotImplementedError("dilated ConvBlock convolutions are not on the accelerated path")
        if norm is not None and (not isinstance(norm, LayerNorm) or not norm.elementwise_affine):
            raise NotImplementedError("ConvBlock norm: LayerNorm (elementwise_affine) or None")
        (kf, kt), (sf, st) = conv.kernel_size, conv.stride
        ln = norm.norm if norm is not None else None
        if x.dtype != dtype and cv.in_channels > 1:
            x = A.to_dtype(x, dtype)
        return A.ConvBlockFn.apply(x, cv.weight, cv.bias, None if ln is None else ln.weight,
                                   None if ln is None else ln.bias, 1e-5 if ln is None else ln.eps, slope, dtype,
                                   out_dtype, (kt, kf, st, sf))

    def general_run(self, x, dtype, out_dtype):
        """Any configuration, layer by layer (differentiable): convs → norm →
        LeakyReLU → dropout per layer, then (residual) + norm(conv1x1(x)) and
        the block dropout (convolution.py:170-175)."""
        if x.dim() == 3:
            x = x.unsqueeze(-1)
        x0 = x
        y = x
        last = self.num_layers - 1
        for i in range(self.num_layers):
            conv, norm, act, drop = self._layer(i)
            if not isinstance(act, nn.LeakyReLU):
                raise NotImplementedError(f"ConvBlock activation {type(act).__name__}: LeakyReLU only")
            od = out_dtype if (i == last and self.reduce_conv is None) else (_f32 if dtype == _f32 else dtype)
            y = self._conv_ln(y, conv, norm, act.negative_slope, dtype, od)
            y = A.dropout(y, drop.p, self.training)
        if self.reduce_conv is not None:
            r = self._conv_ln(x0, self.reduce_conv.conv, self.reduce_conv.norm, None, dtype, _f32)
            y = A.DropAddFn.apply(y, r, 1.0, None, 0.0, _f32)  # y + r in one launch
            y = A.dropout(y, self.drop.p, self.training, out_dtype=out_dtype)
        return y

    def train_run(self, x, dtype, out_dtype):
        """Differentiable block (training path)."""
        if not self._fusable():
            return self.general_run(x, dtype, out_dtype)
        c = self.convs
        if x.dim() == 3:
            x = x.unsqueeze(-1)
        y = self._conv_ln(x, c.conv_0, c.norm_0, c.act_0.negative_slope, dtype, out_dtype)
        return A.dropout(y, c.dropout_0.p, self.training)

    def wants_train_path(self, x):
        drops = [getattr(self.convs, f"dropout_{i}").p for i in range(self.num_layers)]
        if self.drop is not None:
            drops.append(self.drop.p)
        return A.needs_grad(self, x) or (self.training and any(p > 0 for p in drops))

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
        block_draws = []
        for i in range(num_blocks):
            # The reference's Sequential infers each block's input shape by a
            # dummy forward through the previous blocks in training mode
            # (nnet/containers.py get_output_shape), whose Dropout layers draw
            # from the CPU generator.  Consume the same draws so that a seeded
            # construction gives bit-identical initial weights.
            if i > 0:
                _dummy_dropouts(block_draws, dropout)
            blk = ConvBlock(num_layers=num_layers_per_block, out_channels=out_channels[i],
                            input_shape=shape, kernel_size=kernel_sizes[i], stride=strides[i],
                            dilation=dilations[i], residual=residuals[i], conv_module=conv_module,
                            activation=activation, norm=norm, dropout=dropout, conv_bias=conv_bias,
                            padding=padding, conv_init=conv_init)
            self.add_module(f"convblock_{i}", blk)
            self.block_names.append(f"convblock_{i}")
            shape = blk.out_shape
            block_draws += blk.dummy_draw_shapes()

    def _fusable2(self, x, dtype):
        if dtype != torch.bfloat16 or len(self.block_names) != 2 or x.dim() != 3:
            return False
        b1, b2 = (getattr(self, n) for n in self.block_names)
        if not (b1._fusable() and b2._fusable()):
            return False
        c1, c2 = b1.convs.conv_0.conv, b2.convs.conv_0.conv
        return (c1.in_channels == 1 and c1.out_channels == 64 and c2.in_channels == 64
                and c2.out_channels % 16 == 0 and c2.out_channels <= 32 and (x.shape[2] - 1) // 2 + 1 <= 40)

    def run(self, x, last_dtype, topdb=None):
        """Intermediate block outputs in the compute dtype, the last in
        `last_dtype`.  topdb = (slot maxima, top_db) from
        Fbank.forward_deferred: x has not had its top_db floor yet; the fused
        front-end applies it as it loads the rows, the other paths first."""
        dtype = _enc.compute_dtype()
        blocks = [getattr(self, n) for n in self.block_names]
        if topdb is not None and not (self._fusable2(x, dtype) and not any(b.wants_train_path(x) for b in blocks)):
            x = ops.topdb_clamp(x, topdb[0], topdb[1])
            topdb = None
        if any(b.wants_train_path(x) for b in blocks):
            n = len(blocks)
            for i, b in enumerate(blocks):
                x = b.train_run(x, dtype, last_dtype if i == n - 1 else dtype)
            return x
        if self._fusable2(x, dtype):
            # both blocks in one kernel: the block-1 activation stays in LDS
            b1, b2 = (getattr(self, n) for n in self.block_names)
            return _enc.conv_frontend2(x.float().contiguous(), b1.params(), b2.params(), b2.wperm(dtype),
                                       last_dtype, topdb=topdb)
        n = len(self.block_names)
        for i, name in enumerate(self.block_names):
            x = getattr(self, name).run(x, last_dtype if i == n - 1 else dtype)
        return x

    def forward(self, x):
        return self.run(x, _enc.compute_dtype())
