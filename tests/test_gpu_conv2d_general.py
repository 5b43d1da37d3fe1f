"""The standalone Conv2d drop-in beyond the ConvBlock geometry: dilation,
groups (incl. depthwise), every padding mode of "same" (reflect, constant,
replicate, circular), "valid", "causal", skip_transpose and 3-D inputs,
forward and gradients, against the reference's forward (CNN.py:616-691:
transpose, unsqueeze, get_padding_elem :1459-1481 + F.pad, nn.Conv2d)
restated on the CPU in fp32."""
import math

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _pad_elem(L_in, stride, k, d):  # CNN.py:1459-1481
    if stride > 1:
        return [math.floor(k / 2), math.floor(k / 2)]
    L_out = math.floor((L_in - d * (k - 1) - 1) / stride) + 1
    return [math.floor((L_in - L_out) / 2), math.floor((L_in - L_out) / 2)]


def _ref(x, w, b, kw):
    """CNN.py:616-657 with the module's geometry kw."""
    if not kw["skip_transpose"]:
        x = x.transpose(1, -1)
    unsq = x.dim() == 3
    if unsq:
        x = x.unsqueeze(1)
    k, s, d = kw["kernel_size"], kw["stride"], kw["dilation"]
    if kw["padding"] == "same":
        p = _pad_elem(kw["in_channels"], s[-1], k[-1], d[-1]) + _pad_elem(kw["in_channels"], s[-2], k[-2], d[-2])
        x = F.pad(x, p, mode=kw["padding_mode"])
    elif kw["padding"] == "causal":
        x = F.pad(x, (0, 0, (k[0] - 1) * d[1], 0))
    y = F.conv2d(x, w, b, stride=s, dilation=d, groups=kw["groups"])
    if unsq:
        y = y.squeeze(1)
    if not kw["skip_transpose"]:
        y = y.transpose(1, -1)
    return y


CASES = {
    # name: (input shape, Conv2d kwargs)
    "dil_groups": ((2, 23, 19, 4), dict(out_channels=6, kernel_size=(3, 5), dilation=(2, 1), groups=2)),
    "depthwise": ((2, 17, 12, 4), dict(out_channels=8, kernel_size=(3, 3), groups=4)),
    "constant": ((2, 15, 11, 3), dict(out_channels=5, kernel_size=(3, 3), dilation=(1, 2), padding_mode="constant")),
    "replicate": ((1, 14, 10, 2), dict(out_channels=3, kernel_size=(5, 3), padding_mode="replicate")),
    "circular": ((1, 13, 9, 2), dict(out_channels=3, kernel_size=(3, 5), padding_mode="circular")),
    "same_stride2_dil": ((2, 21, 16, 3), dict(out_channels=4, kernel_size=(3, 3), stride=(2, 2), dilation=(2, 2))),
    "valid_stride_dil": ((2, 30, 20, 3), dict(out_channels=4, kernel_size=(4, 2), stride=(2, 3), dilation=(2, 1),
                                              padding="valid")),
    "causal": ((2, 18, 12, 3), dict(out_channels=4, kernel_size=(3, 3), dilation=(1, 2), padding="causal")),
    "skip_transpose": ((2, 3, 12, 16), dict(out_channels=5, kernel_size=(3, 5), dilation=(1, 2), skip_transpose=True,
                                            in_channels=3)),
    "three_d": ((2, 20, 15), dict(out_channels=1, kernel_size=(3, 3), dilation=(2, 1))),
}


@pytest.mark.parametrize("name", list(CASES))
def test_conv2d_general_vs_reference(dev, name):
    from speechbrain_amd.nnet.CNN import Conv2d
    shape, kw = CASES[name]
    kw = dict(kw)
    if "in_channels" not in kw:
        kw["input_shape"] = shape
    torch.manual_seed(hash(name) % 1000)
    conv = Conv2d(**kw)
    full = dict(kernel_size=conv.kernel_size, stride=conv.stride, dilation=conv.dilation, padding=conv.padding,
                padding_mode=conv.padding_mode, groups=conv.groups, skip_transpose=conv.skip_transpose,
                in_channels=conv.in_channels)
    x = torch.randn(*shape)
    w = conv.conv.weight.detach().clone().requires_grad_(True)
    b = conv.conv.bias.detach().clone().requires_grad_(True)
    xr = x.clone().requires_grad_(True)
    ref = _ref(xr, w, b, full)
    conv = conv.to(dev)
    xd = x.to(dev).requires_grad_(True)
    y = conv(xd)
    assert y.shape == ref.shape, (y.shape, ref.shape)
    scale = float(ref.abs().max())
    assert float((y.detach().cpu() - ref.detach()).abs().max()) <= 1e-5 * max(1.0, scale), name
    gy = torch.randn_like(ref)
    ref.backward(gy)
    y.backward(gy.to(dev))
    for got, want, what in ((xd.grad, xr.grad, "dx"), (conv.conv.weight.grad, w.grad, "dw"),
                            (conv.conv.bias.grad, b.grad, "db")):
        sc = max(1.0, float(want.abs().max()))
        assert float((got.cpu() - want).abs().max()) <= 2e-5 * sc, (name, what)


def test_conv2d_reflect_pad_too_large_raises(dev):
    from speechbrain_amd.nnet.CNN import Conv2d
    conv = Conv2d(out_channels=2, kernel_size=(9, 3), input_shape=(1, 8, 3, 1)).to(dev)
    with pytest.raises(ValueError):
        conv(torch.randn(1, 8, 3, 1, device=dev))
