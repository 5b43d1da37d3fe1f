"""Host logic of the standalone Conv2d drop-in (no GPU): the pads, pad mode
and output size that `Conv2d._geometry` hands the HIP im2col kernels must be
those of the reference's forward (CNN.py:616-691: transpose, get_padding_elem
:1459-1481 with the channel count as L_in, F.pad in padding_mode, nn.Conv2d)
over a grid of kernels, strides, dilations and padding modes.  The reference
forward is restated here with torch's CPU conv2d as the checker."""
import itertools
import math

import pytest
import torch
import torch.nn.functional as F


def _pad_elem(L_in, stride, k, d):  # CNN.py:1459-1481
    if stride > 1:
        return [math.floor(k / 2), math.floor(k / 2)]
    L_out = math.floor((L_in - d * (k - 1) - 1) / stride) + 1
    return [math.floor((L_in - L_out) / 2), math.floor((L_in - L_out) / 2)]


def _ref_shape_and_pads(x, conv):
    """(B, C, F, T) after the reference's pads and conv; the pads it applied."""
    k, s, d = conv.kernel_size, conv.stride, conv.dilation
    h = x.transpose(1, -1)
    if conv.padding == "same":
        p = _pad_elem(conv.in_channels, s[-1], k[-1], d[-1]) + _pad_elem(conv.in_channels, s[-2], k[-2], d[-2])
        h = F.pad(h, p, mode=conv.padding_mode)
    elif conv.padding == "causal":
        p = [0, 0, (k[0] - 1) * d[1], 0]
        h = F.pad(h, p)
    else:
        p = [0, 0, 0, 0]
    w = torch.zeros(conv.conv.weight.shape)
    y = F.conv2d(h, w, None, stride=s, dilation=d, groups=conv.groups)
    return y.shape, p


KERNELS = [(3, 3), (5, 3), (3, 5), (1, 1), (4, 2)]
STRIDES = [(1, 1), (2, 2), (2, 1), (1, 3)]
DILATIONS = [(1, 1), (2, 1), (1, 2)]
PADDINGS = [("same", "reflect"), ("same", "constant"), ("same", "replicate"), ("same", "circular"),
            ("valid", "reflect"), ("causal", "reflect")]


@pytest.mark.parametrize("padding,mode", PADDINGS)
def test_conv2d_geometry_matches_reference(padding, mode):
    from speechbrain_amd.nnet.CNN import Conv2d
    n = 0
    for k, s, d in itertools.product(KERNELS, STRIDES, DILATIONS):
        if padding != "valid" and (k[0] % 2 == 0 or k[1] % 2 == 0):
            continue  # the reference rejects even kernels unless "valid" (CNN.py:_check_input)
        B, T, Fq, C = 2, 29, 17, 3
        conv = Conv2d(out_channels=4, kernel_size=k, stride=s, dilation=d, padding=padding, padding_mode=mode,
                      input_shape=(B, T, Fq, C))
        x = torch.zeros(B, T, Fq, C)
        try:
            ref_shape, p = _ref_shape_and_pads(x, conv)
        except RuntimeError:  # the reference itself rejects it (input smaller than the kernel / pad)
            with pytest.raises(ValueError):
                conv._geometry(T, Fq)
            continue
        kt, kf, st, sf, dt, df, pt, pf, To, Fo, m = conv._geometry(T, Fq)
        # reference spatial dims after transpose: (C, F, T) -> conv over (F, T)
        assert (Fo, To) == tuple(ref_shape[2:]), (k, s, d, padding)
        assert (pt, pf) == (p[0], p[2]), (k, s, d, padding)
        assert (kf, kt, sf, st, df, dt) == (k[0], k[1], s[0], s[1], d[0], d[1])
        if padding == "same":
            assert m == Conv2d._MODES[mode]
        n += 1
    assert n > 0
