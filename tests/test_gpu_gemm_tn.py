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


@pytest.mark.parametrize("tile", [64, 128])
@pytest.mark.parametrize("nsplit", [1, 3, 8])
def test_gemm_tn_cfg_tiles_and_splits(dev, tile, nsplit):
    """Every (tile, split) configuration of sbk_gemm_tn_cfg — plain stores at
    one split, fp32 atomics otherwise — on ragged M, N (multiples of 8) and a
    K that does not divide into the splits."""
    from speechbrain_amd._lib import lib, ptr, stream_of
    torch.manual_seed(tile + nsplit)
    K, M, N = 3001, 200, 136
    a = torch.randn(K, M, device=dev).to(torch.bfloat16)
    b = torch.randn(K, N, device=dev).to(torch.bfloat16)
    c = torch.zeros(M, N, device=dev)
    assert lib().sbk_gemm_tn_cfg(ptr(a), M, 0, ptr(b), N, 0, M, N, K, 1, ptr(c), N, 0, tile, nsplit,
                                 stream_of(a)) == 0
    ref = a.float().t() @ b.float()
    bound = 1e-5 * (a.float().abs().t() @ b.float().abs()) + 1e-6
    assert ((c - ref).abs() <= bound).all(), ((c - ref).abs() / bound).max()


def test_cast_bf16_paths_bit_exact(dev):
    """sbk_cast_bf16 (4-wide and per-element kernels) rounds exactly as torch's
    .to(bfloat16) (round to nearest even), incl. ties, infinities and NaN."""
    from speechbrain_amd import _enc
    torch.manual_seed(1)
    base = torch.randn(4097, device=dev) * 3
    base[:8] = torch.tensor([1.00390625, 1.01171875, -2.0078125, 65504.0, float("inf"), -float("inf"), 0.0, -0.0])
    for x in (base[:4096].contiguous(), base[1:].contiguous(), base[1:4096].clone()):  # n % 4 == 0 / odd sizes
        y = _enc.cast_bf16(x)
        assert torch.equal(y.view(torch.int16), x.to(torch.bfloat16).view(torch.int16))
    nan = _enc.cast_bf16(torch.full((8,), float("nan"), device=dev))
    assert torch.isnan(nan.float()).all()


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


@pytest.mark.parametrize("K,M,N,batch", [(12032, 256, 1024, 0), (1001, 37, 70, 0), (377, 40, 36, 4), (5, 3, 3, 0)])
def test_gemm_tn_f32(dev, K, M, N, batch):
    """Exact-f32 weight-gradient GEMM (sbk_gemm_tn_f32): aligned shapes on
    the 16-B loads, ragged M / N (37, 70, 3) on the element-wise loads, against
    float64 on the CPU: only the fp32 summation order differs."""
    from speechbrain_amd import _enc
    torch.manual_seed(K + M)
    shp = (batch,) if batch else ()
    a = torch.randn(*shp, K, M)
    b = torch.randn(*shp, K, N)
    c = _enc.gemm_tn(a.to(dev), b.to(dev)).cpu()
    ref = a.double().transpose(-1, -2) @ b.double()
    bound = 1e-5 * (a.double().abs().transpose(-1, -2) @ b.double().abs()) + 1e-6
    assert c.shape == ref.shape and c.dtype == torch.float32
    assert ((c.double() - ref).abs() <= bound).all(), ((c.double() - ref).abs() / bound).max()


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_gemm_batched_heads(dev, dt):
    """sbk_gemm_batched in both dtypes, over the first M rows of each batch
    entry, with batch z = b*H + h written straight into the (B*M, H*N)
    head-interleaved layout (the attention dropout product drop(P)·V)."""
    from speechbrain_amd import _enc
    torch.manual_seed(2)
    B, H, Mp, M, K, N = 3, 4, 48, 45, 48, 16
    a = torch.randn(B * H, Mp, K).to(dt)
    w = torch.randn(B * H, N + 8, K).to(dt)[:, :N]   # strided rows: batch stride (N+8)*K
    out = _enc.gemm_batched(a.to(dev), w.to(dev), out_dtype=torch.float32, M=M, heads=H).cpu()
    ref = (a[:, :M].double() @ w.double().transpose(-1, -2)).view(B, H, M, N).permute(0, 2, 1, 3).reshape(B * M, H * N)
    bound = 1e-5 * (a[:, :M].double().abs() @ w.double().abs().transpose(-1, -2)).view(B, H, M, N).permute(
        0, 2, 1, 3).reshape(B * M, H * N) + 1e-6
    assert out.shape == (B * M, H * N)
    assert ((out.double() - ref).abs() <= bound).all()
    plain = _enc.gemm_batched(a.to(dev), w.to(dev)).cpu()
    assert plain.shape == (B * H, Mp, N)
    assert torch.allclose(plain[:, :M].reshape(B, H, M, N).permute(0, 2, 1, 3).reshape(B * M, H * N), out, rtol=0,
                          atol=0)


def test_linear_backward_fp32_on_sbk(dev):
    """LinearFn backward in fp32 (the parity mode): dX on the exact-f32
    sbk_gemm, dW on sbk_gemm_tn_f32 — no library GEMM — against float64,
    including an odd width (N = 70, K = 37) on the element-wise loads."""
    from speechbrain_amd import _autograd as A, _enc
    for M, K, N in ((3000, 256, 1024), (777, 37, 70)):
        torch.manual_seed(M)
        x = torch.randn(M, K)
        w = torch.randn(N, K) / 16
        b = torch.randn(N)
        g = torch.randn(M, N)
        xd, wd, bd = (t.to(dev).requires_grad_() for t in (x, w, b))
        A.linear(xd, wd, bd, torch.float32, _enc.WeightCache(), "w").backward(g.to(dev))
        xr, wr, br = (t.double().requires_grad_() for t in (x, w, b))
        (xr @ wr.t() + br).backward(g.double())
        for name, got, want in (("dX", xd.grad, xr.grad), ("dW", wd.grad, wr.grad), ("db", bd.grad, br.grad)):
            e = ((got.cpu().double() - want).norm() / want.norm()).item()
            assert e <= 1e-5, (M, name, e)


def test_wgrad_bf16_strided_operands(dev):
    """_autograd.wgrad's bf16 fallback with operands that are not row-dense
    (a transposed g: stride(1) != 1) at N, K already multiples of 8 — the pad
    is zero there, and F.pad's clone keeps the strides, so the fallback must
    make them contiguous itself."""
    from speechbrain_amd import _autograd as A
    g0 = torch.Generator().manual_seed(5)
    M, N, K = 96, 64, 40
    gt = torch.randn(N, M, generator=g0).to(torch.bfloat16).to(dev)
    g = gt.t()  # (M, N), stride (1, M)
    a = torch.randn(M, K, generator=g0).to(torch.bfloat16).to(dev)
    assert g.stride(1) != 1
    dw = A.wgrad(g, a)
    ref = g.float().t() @ a.float()
    assert torch.allclose(dw.float(), ref, rtol=1e-3, atol=1e-3), float((dw.float() - ref).abs().max())
