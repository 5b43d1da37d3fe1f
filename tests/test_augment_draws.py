"""SpecAugment's host draws on the CPU (no GPU needed): SpecAugment.draws()
draws its mask lengths / positions as int32 (one 32-bit generator draw per
element, as the reference's int64 torch.randint over a < 2^32 range), so the
values must equal the reference order's int64 draws (augment.py:131-133,
175-186) and the reference's own recorded draws (tests/golden/specaug.npz)."""
import numpy as np
import torch


def _ref_draws(N, T, F, win, fw, nf, tw, nt):
    """The reference's draw order with its int64 tensors."""
    c = torch.randint(win, T - win, (1,))[0]
    w = torch.randint(c - win, c + win, (1,))[0] + 1
    ln = torch.randint(fw[0], fw[1], (N, nf))
    fm = torch.stack([ln, torch.randint(0, max(1, F - int(ln.max())), (N, nf))], -1)
    ln = torch.randint(tw[0], tw[1], (N, nt))
    tm = torch.stack([ln, torch.randint(0, max(1, T - int(ln.max())), (N, nt))], -1)
    return int(c), int(w), fm, tm


def test_int32_draws_equal_reference_int64_order():
    from speechbrain_amd.lobes.augment import SpecAugment
    sa = SpecAugment(time_warp=True, time_warp_window=5, freq_mask=True, freq_mask_width=(0, 30), n_freq_mask=2,
                     time_mask=True, time_mask_width=(0, 40), n_time_mask=2, replace_with_zero=False)
    for seed in range(64):
        for N, T, F in ((32, 1501, 240), (3, 97, 40)):
            torch.manual_seed(seed)
            c, w, fm, tm = sa.draws(N, T, F)
            torch.manual_seed(seed)
            rc, rw, rfm, rtm = _ref_draws(N, T, F, 5, (0, 30), 2, (0, 40), 2)
            assert (c, w) == (rc, rw)
            assert fm.dtype == tm.dtype == torch.int32
            assert torch.equal(fm.long(), rfm) and torch.equal(tm.long(), rtm)


def test_draws_match_reference_fixture(golden):
    from speechbrain_amd.lobes.augment import SpecAugment
    g = golden("specaug")
    N, T, F = g["feats"].shape
    for s in range(4):
        sa = SpecAugment(time_warp=True, time_warp_window=5, time_warp_mode="bicubic", freq_mask=True,
                         n_freq_mask=2, time_mask=True, n_time_mask=2, replace_with_zero=False, freq_mask_width=30,
                         time_mask_width=40)
        torch.manual_seed(s)
        c, w, fm, tm = sa.draws(N, T, F)
        got = np.concatenate([[c], [w - 1], fm[..., 0].reshape(-1), fm[..., 1].reshape(-1),
                              tm[..., 0].reshape(-1), tm[..., 1].reshape(-1)]).astype(np.int64)
        assert np.array_equal(got, g[f"recipe_s{s}_draws"])
