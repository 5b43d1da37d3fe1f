"""CPU restatement of SpecAugment (test infrastructure).

Restates speechbrain/lobes/augment.py:32-201.  Random draws use the global
CPU generator in the reference's order (c, w for time warp; then mask_len,
mask_pos for the frequency masks; then mask_len, mask_pos for the time
masks), so the same torch.manual_seed reproduces the reference's mask
indices bit-exactly.
"""
import math

import torch

A_CUBIC = -0.75  # PyTorch's bicubic convolution constant


def _cubic1(x, A=A_CUBIC):
    return ((A + 2) * x - (A + 3)) * x * x + 1


def _cubic2(x, A=A_CUBIC):
    return ((A * x - 5 * A) * x + 8 * A) * x - 4 * A


def bicubic_resize_rows(x, out_rows):
    """1-D bicubic resize along dim -2 with align_corners=True (A=-0.75),
    border-clamped taps — the height pass of
    torch.nn.functional.interpolate(mode="bicubic", align_corners=True) when
    the width is unchanged (augment.py:134-145; the width pass is then the
    identity: weights (0,1,0,0) at t=0)."""
    in_rows = x.shape[-2]
    if in_rows == out_rows:
        return x.clone()
    f32 = torch.float32
    if out_rows > 1:
        scale = torch.tensor((in_rows - 1) / (out_rows - 1), dtype=f32)
    else:
        scale = torch.tensor(0.0, dtype=f32)
    dst = torch.arange(out_rows, dtype=f32)
    real = scale * dst
    idx = torch.floor(real)
    t = real - idx
    idx = idx.to(torch.int64)
    w = [_cubic2(t + 1.0), _cubic1(t), _cubic1(1.0 - t), _cubic2(2.0 - t)]
    out = torch.zeros(*x.shape[:-2], out_rows, x.shape[-1], dtype=x.dtype)
    for k in range(4):
        j = torch.clamp(idx - 1 + k, 0, in_rows - 1)
        out = out + w[k].view(-1, 1) * x[..., j, :]
    return out


def time_warp(x, window=5):
    """augment.py:116-150: one centre c and warped length w for the whole
    batch; [0,c) resized to w rows and [c,T) to T-w rows; in place."""
    original_size = x.shape
    if x.dim() == 3:
        x = x.unsqueeze(1)
    time = x.shape[2]
    if time - window <= window:
        return x.view(*original_size)
    c = torch.randint(window, time - window, (1,))[0]
    w = torch.randint(c - window, c + window, (1,))[0] + 1
    c, w = int(c), int(w)
    left = bicubic_resize_rows(x[:, :, :c], w)
    right = bicubic_resize_rows(x[:, :, c:], time - w)
    x[:, :, :w] = left
    x[:, :, w:] = right
    return x.view(*original_size)


def draw_masks(batch, D, n_mask, width_range):
    """augment.py:175-186: mask_len ~ U[lo,hi) (batch, n); mask_pos ~
    U[0, max(1, D - max(mask_len))) (batch, n)."""
    mask_len = torch.randint(width_range[0], width_range[1], (batch, n_mask))
    mask_pos = torch.randint(0, max(1, D - int(mask_len.max())), (batch, n_mask))
    return mask_len, mask_pos


def mask_along_axis(x, dim, n_mask, width_range, replace_with_zero):
    """augment.py:152-201: union of n masks [pos, pos+len) per sequence on
    axis `dim` (1=time, 2=freq), filled with 0 or the global mean; in place."""
    original_size = x.shape
    if x.dim() == 4:
        x = x.view(-1, x.shape[2], x.shape[3])
    batch, time, fea = x.shape
    D = time if dim == 1 else fea
    mask_len, mask_pos = draw_masks(batch, D, n_mask, width_range)
    ar = torch.arange(D).view(1, 1, -1)
    mask = ((mask_pos.unsqueeze(2) <= ar) & (ar < (mask_pos + mask_len).unsqueeze(2))).any(dim=1)
    mask = mask.unsqueeze(2) if dim == 1 else mask.unsqueeze(1)
    val = 0.0 if replace_with_zero else x.mean()
    x.masked_fill_(mask, val)
    return x.view(*original_size)


def spec_augment(x, time_warp_on=True, time_warp_window=5, freq_mask=True,
                 freq_mask_width=(0, 20), n_freq_mask=2, time_mask=True,
                 time_mask_width=(0, 100), n_time_mask=2, replace_with_zero=True):
    """augment.py:106-114 (SpecAugment.forward); mutates and returns x."""
    if isinstance(freq_mask_width, int):
        freq_mask_width = (0, freq_mask_width)
    if isinstance(time_mask_width, int):
        time_mask_width = (0, time_mask_width)
    if time_warp_on:
        x = time_warp(x, time_warp_window)
    if freq_mask:
        x = mask_along_axis(x, 2, n_freq_mask, freq_mask_width, replace_with_zero)
    if time_mask:
        x = mask_along_axis(x, 1, n_time_mask, time_mask_width, replace_with_zero)
    return x
