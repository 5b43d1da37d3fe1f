"""The eager fast path of the sbk custom ops (speechbrain_amd._lib.custom_op):
outside tracing the op's body runs without the torch.library dispatcher, and
what the dispatcher would have done still happens — mutated inputs get their
version counter bumped, a differentiable call of an op with a registered
backward goes through autograd, a traced call is recorded as the op.  CPU
only: the ops here are defined by the test, no kernel runs."""
from typing import Optional

import torch

from speechbrain_amd._lib import custom_op


@custom_op("sbk::_test_scale_", mutates_args=("x",))
def _scale_(x: torch.Tensor, a: float, y: Optional[torch.Tensor] = None) -> None:
    x.numpy()[:] *= a  # mutated outside torch, as a kernel launch does: no version bump of its own


@custom_op("sbk::_test_double", mutates_args=())
def _double(x: torch.Tensor) -> torch.Tensor:
    return x * 2


_double.register_fake(lambda x: torch.empty_like(x))
_double.register_autograd(lambda ctx, g: g * 2)


def test_fast_path_bumps_mutated_versions():
    x = torch.ones(4)
    v = x._version
    _scale_(x, 3.0)
    assert torch.equal(x, torch.full((4,), 3.0))
    assert x._version == v + 1


def test_differentiable_call_goes_through_autograd():
    x = torch.ones(3, requires_grad=True)
    y = _double(x)
    assert y.grad_fn is not None
    y.sum().backward()
    assert torch.equal(x.grad, torch.full((3,), 2.0))
    with torch.no_grad():
        assert _double(x).grad_fn is None


def test_traced_call_is_recorded_as_the_op():
    tr = torch.jit.trace(lambda t: _double(t), torch.ones(2))
    assert "sbk::_test_double" in str(tr.graph)
    assert torch.equal(tr(torch.full((2,), 5.0)), torch.full((2,), 10.0))


@custom_op("sbk::_test_nograd", mutates_args=())
def _nograd(x: torch.Tensor) -> torch.Tensor:
    return x + 1


_nograd.register_fake(lambda x: torch.empty_like(x))


def test_op_without_backward_raises_at_the_call():
    import pytest
    x = torch.ones(3, requires_grad=True)
    with pytest.raises(RuntimeError, match="_test_nograd has no backward"):
        _nograd(x)
    with torch.no_grad():
        assert torch.equal(_nograd(x), torch.full((3,), 2.0))
    assert torch.equal(_nograd(x.detach()), torch.full((3,), 2.0))
