"""HIP SpecAugment vs the reference's golden outputs (same seeds → same
CPU-generator draws → bit-exact mask indices) and vs the oracle at the
BASELINE config-2 size."""
import numpy as np
import pytest
import torch

from conftest import assert_close
import oracle.augment as OA

pytestmark = pytest.mark.gpu

CFGS = {
    "recipe": dict(time_warp=True, time_warp_window=5, time_warp_mode="bicubic", freq_mask=True, n_freq_mask=2,
                   time_mask=True, n_time_mask=2, replace_with_zero=False, freq_mask_width=30, time_mask_width=40),
    "default": dict(),
    "nowarp": dict(time_warp=False, freq_mask_width=(5, 15), time_mask_width=(10, 20), n_freq_mask=3,
                   n_time_mask=1),
}


@pytest.mark.parametrize("cfg", list(CFGS))
def test_specaugment_vs_golden(golden, dev, cfg):
    from speechbrain_amd.lobes.augment import SpecAugment
    g = golden("specaug")
    feats = torch.from_numpy(g["feats"])
    for s in range(4):
        aug = SpecAugment(**CFGS[cfg])
        torch.manual_seed(s)
        x = feats.clone().to(dev)
        y = aug(x)
        assert y is x  # in place, like the reference
        ref = g[f"{cfg}_s{s}"]
        assert_close(y, ref, rtol=1e-5, name=f"{cfg}{s}")
        # bit-exact indices: the fill pattern matches cell for cell
        if cfg != "recipe":
            yn = y.cpu().numpy()
            assert np.array_equal(yn == 0, ref == 0)


def test_specaugment_draw_order_matches_reference(golden, dev):
    from speechbrain_amd.lobes.augment import SpecAugment
    g = golden("specaug")
    feats = torch.from_numpy(g["feats"])
    for s in range(4):
        aug = SpecAugment(**CFGS["recipe"])
        torch.manual_seed(s)
        aug(feats.clone().to(dev))
        c, w, fm, tm = aug.last_draws
        got = np.concatenate([[c], [w - 1], fm[..., 0].reshape(-1), fm[..., 1].reshape(-1),
                              tm[..., 0].reshape(-1), tm[..., 1].reshape(-1)]).astype(np.int64)
        assert np.array_equal(got, g[f"recipe_s{s}_draws"])


def test_time_warp_only_vs_golden(golden, dev):
    from speechbrain_amd.lobes.augment import SpecAugment
    g = golden("specaug")
    feats = torch.from_numpy(g["feats"])
    aug = SpecAugment(time_warp=True, freq_mask=False, time_mask=False)
    for s in range(4):
        torch.manual_seed(100 + s)
        assert_close(aug(feats.clone().to(dev)), g[f"warp_s{s}"], rtol=1e-5, name=f"warp{s}")


def test_specaugment_full_size_vs_oracle(dev):
    """B=32 x 1501 x 80 (BASELINE config 2), recipe parameters."""
    from speechbrain_amd.lobes.augment import SpecAugment
    x = torch.randn(32, 1501, 80, generator=torch.Generator().manual_seed(7)) * 10 - 40
    for seed in (1234, 1235):
        torch.manual_seed(seed)
        y = SpecAugment(**CFGS["recipe"])(x.clone().to(dev))
        torch.manual_seed(seed)
        ref = OA.spec_augment(x.clone(), time_warp_on=True, time_warp_window=5, freq_mask=True, n_freq_mask=2,
                              time_mask=True, n_time_mask=2, replace_with_zero=False, freq_mask_width=30,
                              time_mask_width=40)
        assert_close(y, ref, rtol=1e-5, name=f"full{seed}")


def test_specaugment_4d_and_short(dev):
    from speechbrain_amd.lobes.augment import SpecAugment
    x = torch.randn(2, 3, 40, 20)
    torch.manual_seed(5)
    y = SpecAugment(freq_mask_width=(0, 5), time_mask_width=(0, 8))(x.clone().to(dev))
    torch.manual_seed(5)
    ref = OA.spec_augment(x.clone(), freq_mask_width=(0, 5), time_mask_width=(0, 8))
    assert_close(y, ref, rtol=1e-5, name="4d")
    # T - window <= window: no warp, no draws for it (augment.py:128-129)
    x = torch.randn(2, 9, 20)
    torch.manual_seed(6)
    y = SpecAugment(freq_mask_width=(0, 5), time_mask_width=(0, 3))(x.clone().to(dev))
    torch.manual_seed(6)
    ref = OA.spec_augment(x.clone(), freq_mask_width=(0, 5), time_mask_width=(0, 3))
    assert_close(y, ref, rtol=1e-5, name="short")


@pytest.mark.parametrize("N,T,F,win,zero,warp", [
    (32, 1501, 240, 5, False, True),   # config 2 (Δ/ΔΔ features): in place, no scratch
    (3, 200, 240, 5, True, True),      # zero fill, in place
    (2, 300, 80, 40, False, True),     # a wide warp window (|c - w| <= 40: still in place)
    (2, 400, 80, 90, False, True),     # a wider window, still in place
    (2, 1200, 40, 450, False, True),   # |c - w| may pass the in-place halo (381): the copy path
    (2, 700, 240, 5, False, False),    # no warp: sums only, then the masked cells
    (1, 97, 40, 5, False, True),       # one utterance, narrow slabs
    (2, 120, 42, 5, False, True),      # F % 4 != 0: the scalar kernels
])
def test_specaugment_paths_vs_oracle(dev, N, T, F, win, zero, warp):
    """The in-place (x read once, masked cells written after the means), copy
    and scalar routes of sbk_specaugment, with the second mean's masked-cell
    count taken on the device, against the oracle."""
    from speechbrain_amd._lib import lib
    from speechbrain_amd.lobes.augment import SpecAugment
    x = torch.randn(N, T, F, generator=torch.Generator().manual_seed(T + F)) * 10 - 40
    kw = dict(time_warp=warp, time_warp_window=win, freq_mask=True, n_freq_mask=2, time_mask=True, n_time_mask=2,
              replace_with_zero=zero, freq_mask_width=min(30, F // 2), time_mask_width=40)
    for seed in (11, 12, 13):
        torch.manual_seed(seed)
        aug = SpecAugment(**kw)
        y = aug(x.clone().to(dev))
        c, w, _, _ = aug.last_draws
        in_place = F % 4 == 0 and (c < 0 or abs(c - w) + 3 <= 384)
        assert lib().sbk_specaugment_needs_scratch(N, T, F, c, w, 2, 2, 1) == int(c >= 0 and not in_place)
        torch.manual_seed(seed)
        ref = OA.spec_augment(x.clone(), time_warp_on=warp, time_warp_window=win, freq_mask=True, n_freq_mask=2,
                              time_mask=True, n_time_mask=2, replace_with_zero=zero,
                              freq_mask_width=kw["freq_mask_width"], time_mask_width=40)
        assert_close(y, ref, rtol=1e-5, name=f"N{N} T{T} F{F} win{win} seed{seed}")


@pytest.mark.parametrize("N,T,F,win,zero", [
    (2, 257, 240, 5, False),
    (2, 512, 80, 10, False),   # |c - w| + 3 up to 13
    (3, 769, 40, 10, True),    # zero fill
    (2, 1000, 24, 5, False),   # F / 4 = 6: two-column slabs
    (2, 600, 20, 5, False),    # F / 4 = 5: one-column slabs
])
def test_specaugment_long_and_narrow_vs_oracle(dev, N, T, F, win, zero):
    """The in-place route on longer utterances (T around multiples of 256,
    up to three windows of the roll kernel's ring) and on 1- / 2-column
    slabs (F / 4 odd or 6) against the oracle, masks and mean fills
    included."""
    from speechbrain_amd.lobes.augment import SpecAugment
    x = torch.randn(N, T, F, generator=torch.Generator().manual_seed(3 * T + F)) * 10 - 40
    kw = dict(time_warp=True, time_warp_window=win, freq_mask=True, n_freq_mask=2, time_mask=True, n_time_mask=2,
              replace_with_zero=zero, freq_mask_width=min(30, F // 2), time_mask_width=40)
    for seed in (21, 22, 23, 24):
        torch.manual_seed(seed)
        aug = SpecAugment(**kw)
        y = aug(x.clone().to(dev))
        torch.manual_seed(seed)
        ref = OA.spec_augment(x.clone(), time_warp_on=True, time_warp_window=win, freq_mask=True, n_freq_mask=2,
                              time_mask=True, n_time_mask=2, replace_with_zero=zero,
                              freq_mask_width=kw["freq_mask_width"], time_mask_width=40)
        assert_close(y, ref, rtol=1e-5, name=f"N{N} T{T} F{F} win{win} seed{seed}")


@pytest.mark.parametrize("T", [300, 1501])
def test_specaugment_bilinear_warp_in_place(dev, T):
    """The bilinear warp in place: torch's align_corners bilinear
    resize of the two segments (augment.py:134-148) at the drawn c, w."""
    import torch.nn.functional as Fn
    from speechbrain_amd.lobes.augment import SpecAugment
    x = torch.randn(3, T, 80, generator=torch.Generator().manual_seed(T)) * 10 - 40
    for seed in (31, 32, 33):
        torch.manual_seed(seed)
        aug = SpecAugment(time_warp=True, time_warp_window=8, time_warp_mode="bilinear", freq_mask=False,
                          time_mask=False)
        y = aug(x.clone().to(dev))
        c, w, _, _ = aug.last_draws
        if c < 0:
            assert_close(y, x, rtol=0, name="identity")
            continue
        x4 = x.unsqueeze(1)
        left = Fn.interpolate(x4[:, :, :c], size=(w, 80), mode="bilinear", align_corners=True)
        right = Fn.interpolate(x4[:, :, c:], size=(T - w, 80), mode="bilinear", align_corners=True)
        ref = torch.cat([left, right], dim=2).squeeze(1)
        assert_close(y, ref, rtol=1e-5, name=f"bilinear T{T} seed{seed}")
