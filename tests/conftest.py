import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GOLDEN = os.path.join(ROOT, "tests", "golden")
if GOLDEN not in sys.path:
    sys.path.insert(0, GOLDEN)  # detinit / doctest_cases: shared with gen_golden.py


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a ROCm GPU (MI355X) and libsbk.so")


@pytest.fixture(scope="session")
def golden():
    cache = {}

    def load(name):
        if name not in cache:
            cache[name] = np.load(os.path.join(GOLDEN, name + ".npz"))
        return cache[name]
    return load


@pytest.fixture(scope="session")
def dev():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no ROCm device")
    from speechbrain_amd import _lib
    _lib.lib()  # fail loudly (not skip) if the HIP library is missing on a GPU box
    return torch.device("cuda:0")


def assert_close(a, b, rtol=1e-4, name=""):
    """|a-b| <= rtol * max(1, |b|) elementwise (dB values cross 0)."""
    import torch
    if isinstance(a, torch.Tensor):
        a = a.detach().float().cpu().numpy()
    if isinstance(b, torch.Tensor):
        b = b.detach().float().cpu().numpy()
    a = np.asarray(a)
    b = np.asarray(b)
    assert a.shape == b.shape, f"{name}: shape {a.shape} != {b.shape}"
    err = np.abs(a.astype(np.float64) - b.astype(np.float64))
    tol = rtol * np.maximum(1.0, np.abs(b.astype(np.float64)))
    bad = ~(err <= tol)
    assert not bad.any(), (f"{name}: {bad.sum()} / {bad.size} elements out of tolerance, "
                           f"max err {np.nanmax(err):.3e}, max rel {np.nanmax(err / np.maximum(1, np.abs(b))):.3e}")
