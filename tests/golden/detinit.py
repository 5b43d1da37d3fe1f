"""Deterministic parameter values for fixture models (test infrastructure).

The reference's seeded init (xavier_* under torch.manual_seed) depends on the
order in which every submodule draws from the global generator; for the
fixtures of the larger doctest models that would mean committing megabytes
of weights.  Instead both tests/golden/gen_golden.py (on the reference
modules) and the GPU tests (on the drop-ins) load the same state_dict made
here: each parameter, by its state_dict name, from numpy's PCG64 seeded with
(seed, crc32(name)) — independent of module construction order.

  >= 2-D weights  N(0, 1/fan_in)            (fan_in = numel / shape[0])
  1-D "...weight" 1 + 0.1·N(0, 1)           (LayerNorm gains)
  other 1-D       0.1·N(0, 1)               (biases, value_bias_weight)
Buffers (sine tables, inv_freq, Deltas kernels) keep their constructed values.
"""
import zlib

import numpy as np


def det_array(name, shape, seed):
    rng = np.random.default_rng([seed, zlib.crc32(name.encode())])
    n = rng.standard_normal(shape)
    if len(shape) >= 2:
        fan_in = int(np.prod(shape[1:]))
        return (n / np.sqrt(fan_in)).astype(np.float32)
    if name.endswith("weight"):
        return (1.0 + 0.1 * n).astype(np.float32)
    return (0.1 * n).astype(np.float32)


def det_state(module, seed=0):
    """A full state_dict for `module` (load with strict=True)."""
    import torch
    params = dict(module.named_parameters())
    out = {}
    for k, v in module.state_dict().items():
        if k in params:
            out[k] = torch.from_numpy(det_array(k, tuple(v.shape), seed))
        else:
            out[k] = v.clone()
    return out


def det_input(shape, seed, kind="randn"):
    """Seeded inputs (numpy PCG64, machine independent) as float32 arrays."""
    rng = np.random.default_rng(seed)
    if kind == "rand":
        return rng.random(shape).astype(np.float32)
    return rng.standard_normal(shape).astype(np.float32)
