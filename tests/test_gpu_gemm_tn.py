"""Weight-gradient GEMM (csrc/gemm_tn.hip): C = A^T B for bf16 token-major
operands vs the same product in fp32 torch on the bf16 values (only the
fp32 summation order differs: |err| <= 1e-5 * sum|a||b|), and the Linear /
ConvBlock backward that uses it (dX on sbk_gemm) vs torch autograd."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("K,M,N,batch", [(12032, 256, 1024, 0), (1000, 136, 72, 0), (376, 64, 64, 4), (8, 256, 256, 0)])
def test_gemm_tn(dev, K, M, N, batch):
    from speechbrain_amd import _enc
    torch.manual_seed(K + M)
    shp = (batch,) if batch else ()
    a = torch.randn(*shp, K, M, device=dev).to(torch.bfloat16)
    b = torch.randn(*shp, K, N, device=dev).to(torch.bfloat16)
    c = _enc.gemm_tn(a, b)
    ref = a.float().transpose(-1, -2) @ b.float()
    bound = 1e-5 * (a.float().abs().transpose(-1, -2) @ b.float().abs()) + 1e-6
    assert c.shape == ref.shape and c.dtype == torch.float32
    assert ((c - ref).abs() <= bound).all(), ((c - ref).abs() / bound).max()


def test_linear_backward_on_sbk(dev):
    """LinearFn backward in bf16: dX = dY W (sbk_gemm), dW = dY^T X
    (sbk_gemm_tn), db = column sums, against torch autograd on the same bf16
    operands in fp32 (dY rounded to bf16 for the GEMMs; dX is returned in
    bf16: one more rounding)."""
    from speechbrain_amd import _autograd as A, _enc
    torch.manual_seed(0)
    M, K, N = 3000, 256, 1024
    x = torch.randn(M, K, device=dev).to(torch.bfloat16).requires_grad_()
    w = (torch.randn(N, K, device=dev) / 16).requires_grad_()
    b = torch.randn(N, device=dev).requires_grad_()
    y = A.linear(x, w, b, torch.bfloat16, _enc.WeightCache(), "w")
    g = torch.randn(M, N, device=dev)
    y.backward(g)
    xr = x.detach().float().requires_grad_()
    wr = w.detach().to(torch.bfloat16).float().requires_grad_()
    br = b.detach().clone().requires_grad_()
    yr = xr @ wr.t() + br
    yr.backward(g.to(torch.bfloat16).float())
    # db sums the fp32 dY (LinearFn keeps it unrounded for the bias)
    for name, got, want, tol in (("dX", x.grad, xr.grad, 1e-2), ("dW", w.grad, wr.grad, 1e-4), ("db", b.grad, g.sum(0), 1e-5)):
        e = ((got.float() - want).norm() / want.norm()).item()
        print(f"{name}: normwise rel err {e:.2e}")
        assert e <= tol, (name, e)
