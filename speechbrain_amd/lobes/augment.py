"""Drop-in for speechbrain.lobes.augment.SpecAugment (augment.py:32-201).

Random draws (warp centre/width, mask lengths/positions) are made on the host
with the CPU generator in exactly the reference's order, so a given
torch.manual_seed reproduces the reference CPU path's mask indices bit for
bit — also for ROCm tensors, where the reference would draw masks on the
device generator.  The warp / mask / mean-fill arithmetic runs in
speechbrain_amd/csrc/augment.hip; the input is mutated in place and
returned, as in the reference.
"""
from typing import Optional

import torch

from .._lib import OPS, check, custom_op, lib, ptr, require_device, stream_of

__all__ = ["SpecAugment"]

_WARP_MODES = {"bicubic": 0, "bilinear": 1}


@custom_op("sbk::specaugment_", mutates_args=("x",))
def specaugment_(x: torch.Tensor, N: int, T: int, F: int, c: int, w: int, fm: Optional[torch.Tensor],
                 tm: Optional[torch.Tensor], use_mean: bool, n_fcells: int, warp_mode: int = 0) -> None:
    """Applies the drawn warp (c, w; -1 = none; warp_mode 0 bicubic, 1
    bilinear) and freq / time masks
    (fm, tm: (N, n, 2) int32 [len, pos]) to x (N, T, F) fp32 in place, with
    the batch-mean fill when use_mean (augment.py:116-201)."""
    n_f = fm.shape[1] if fm is not None else 0
    n_t = tm.shape[1] if tm is not None else 0
    # the in-place path (the float4 shapes of the recipe) needs no scratch copy
    tmp = (torch.empty_like(x) if lib().sbk_specaugment_needs_scratch(N, T, F, c, w, n_f, n_t,
                                                                       int(x.data_ptr() % 16 == 0)) else None)
    # partial sums: the copy path's 2 per 4 rows (+ its two fills), the
    # in-place path's 3 per column slab
    npart = max(2 * N * ((T + 3) // 4), 3 * N * (F // 4))
    partial = torch.empty(npart + 4, device=x.device, dtype=torch.float32) if use_mean else None
    rc = lib().sbk_specaugment(ptr(x), N, T, F, c, w, int(warp_mode), ptr(tmp), ptr(fm), n_f, ptr(tm), n_t,
                               int(use_mean),
                               ptr(partial), n_fcells, stream_of(x))
    check(rc, "sbk_specaugment")


@specaugment_.register_fake
def _(x, N, T, F, c, w, fm, tm, use_mean, n_fcells, warp_mode=0):
    return None


class SpecAugment(torch.nn.Module):
    def __init__(self, time_warp=True, time_warp_window=5, time_warp_mode="bicubic", freq_mask=True,
                 freq_mask_width=(0, 20), n_freq_mask=2, time_mask=True, time_mask_width=(0, 100), n_time_mask=2,
                 replace_with_zero=True):
        super().__init__()
        assert time_warp or freq_mask or time_mask, \
            "at least one of time_warp, time_mask, or freq_mask should be applied"
        if time_warp and time_warp_mode not in _WARP_MODES:
            # the reference interpolates with align_corners=True (augment.py:134-148), which torch
            # accepts for the (bi)linear / bicubic modes only; the other modes raise there too
            raise ValueError(f"time_warp_mode {time_warp_mode!r}: align_corners interpolation needs one of "
                             f"{sorted(_WARP_MODES)}")
        self.apply_time_warp = time_warp
        self.time_warp_window = time_warp_window
        self.time_warp_mode = time_warp_mode
        self.freq_mask = freq_mask
        if isinstance(freq_mask_width, int):
            freq_mask_width = (0, freq_mask_width)
        self.freq_mask_width = freq_mask_width
        self.n_freq_mask = n_freq_mask
        self.time_mask = time_mask
        if isinstance(time_mask_width, int):
            time_mask_width = (0, time_mask_width)
        self.time_mask_width = time_mask_width
        self.n_time_mask = n_time_mask
        self.replace_with_zero = replace_with_zero
        self.last_draws = None
        self._pin = None     # pinned staging of the mask draws (reused; see _upload)
        self._pin_ev = None  # completion of the last upload out of it

    def _upload(self, parts, device):
        """int32 host draws (concatenated) -> device, asynchronously from a
        reused pinned buffer (a pageable copy would block the host for the
        transfer)."""
        n = sum(p.numel() for p in parts)
        if self._pin is None or self._pin.numel() < n:
            self._pin = torch.empty(max(n, 1024), dtype=torch.int32).pin_memory()
            self._pin_ev = None
        if self._pin_ev is not None:
            self._pin_ev.synchronize()  # the previous copy out of the buffer is done
        o = 0
        for p in parts:
            self._pin[o:o + p.numel()].copy_(p)
            o += p.numel()
        dev = self._pin[:n].to(device, non_blocking=True)
        self._pin_ev = torch.cuda.Event()
        self._pin_ev.record(torch.cuda.current_stream(device))
        return dev

    def draws(self, N, T, F):
        """Host draws in the reference order (augment.py:131-133, :175-186)."""
        c = w = -1
        if self.apply_time_warp:
            win = self.time_warp_window
            if T - win > win:
                c = int(torch.randint(win, T - win, (1,))[0])
                w = int(torch.randint(c - win, c + win, (1,))[0]) + 1
        # (int32 draws: the same values as the reference's int64 ones — one
        # 32-bit generator draw per element either way, tests/test_augment_draws.py)
        i32 = torch.int32
        fm = tm = None
        if self.freq_mask:
            ln = torch.randint(self.freq_mask_width[0], self.freq_mask_width[1], (N, self.n_freq_mask), dtype=i32)
            ps = torch.randint(0, max(1, F - int(ln.max())), (N, self.n_freq_mask), dtype=i32)
            fm = torch.stack([ln, ps], -1)
        if self.time_mask:
            ln = torch.randint(self.time_mask_width[0], self.time_mask_width[1], (N, self.n_time_mask), dtype=i32)
            ps = torch.randint(0, max(1, T - int(ln.max())), (N, self.n_time_mask), dtype=i32)
            tm = torch.stack([ln, ps], -1)
        return c, w, fm, tm

    def forward(self, x):
        """Takes in input a tensor and returns an augmented one (in place)."""
        require_device(x)
        if x.dtype != torch.float32 or not x.is_contiguous():
            raise TypeError("SpecAugment kernel expects a contiguous fp32 tensor")
        if x.dim() == 3:
            N, T, F = x.shape
        elif x.dim() == 4:
            N, T, F = x.shape[0] * x.shape[1], x.shape[2], x.shape[3]
        else:
            raise ValueError("expected (batch, time, freq) or (batch, channel, time, freq)")
        c, w, fm, tm = self.draws(N, T, F)
        if c == w:
            c = w = -1  # identical segment sizes: the resize is the identity
        self.last_draws = (c, w, fm, tm)
        # both mask tables in one asynchronous pinned host -> device copy (the
        # per-step host work is this module's cost at config 2, not its
        # kernels); the second mean's masked-cell count is taken on the
        # device from the table (n_fcells = -1)
        parts = [m.reshape(-1) for m in (fm, tm) if m is not None]
        fm_d = tm_d = None
        if parts:
            buf = self._upload(parts, x.device)
            nf = fm.numel() if fm is not None else 0
            fm_d = buf[:nf].view(fm.shape) if fm is not None else None
            tm_d = buf[nf:].view(tm.shape) if tm is not None else None
        OPS.specaugment_(x, N, T, F, c, w, fm_d, tm_d, not self.replace_with_zero, -1,
                                   _WARP_MODES.get(self.time_warp_mode, 0))
        return x
