"""fp32 projections (sae_gemm_f32, the exact-f32 MFMA) against float64 products of the same inputs.

The Dense / DenseGeneral dot_generals at compute dtype float32 (attention.py:29-37,60-63,
ff.py:8-34; the reference's fp32 CaiT trunk, cait.py:147-154) and their autodiff gradients
dX = dY W^T, dW = X^T dY, db = colsum(dY).  The kernel accumulates in fp32 (a k-ordered fmaf
chain per split), so the bar is the north_star fp32 tolerance, 1e-5 of the largest magnitude."""
import pytest
import torch

pytestmark = pytest.mark.gpu

TOL = 1e-5


def _rel(a, b):
    return float((a.double() - b.double()).abs().max() / b.double().abs().max().clamp_min(1e-30))


def _rand(dev, shape, seed, scale=1.0):
    g = torch.Generator(device=dev).manual_seed(seed)
    return torch.randn(*shape, device=dev, generator=g) * scale


FWD = [  # (M, K, N): x [M, K] @ W [K, N]
    (25216, 384, 1152),   # DeiT-S QKV projection at batch 128
    (18464, 768, 768),    # ViT-B@384 output projection at batch 32
    (197, 768, 1000),     # ragged tokens, head-like N (not a tile multiple)
    (5, 20, 12),          # below one tile everywhere
    (130, 132, 136),      # one past the tile on M / K / N
]


@pytest.mark.parametrize("M,K,N", FWD)
@pytest.mark.parametrize("bias", [False, True])
def test_forward(dev, M, K, N, bias):
    import sae_vision_amd.ops as ops
    x = _rand(dev, (M, K), M + K)
    w = _rand(dev, (K, N), N, K ** -0.5)
    b = _rand(dev, (N,), 1) if bias else None
    y = ops.gemm_f32(x, w, b)
    ref = x.double() @ w.double() + (b.double() if bias else 0)
    assert _rel(y, ref) <= TOL


@pytest.mark.parametrize("M,K,N", FWD[1:])
def test_input_gradient_layout(dev, M, K, N):
    """dX = dY W^T: B read k-contiguous straight from W (W.t() view, no copy)."""
    import sae_vision_amd.ops as ops
    dy = _rand(dev, (M, N), 3)
    w = _rand(dev, (K, N), 4)
    dx = ops.gemm_f32(dy, w.t())
    assert _rel(dx, dy.double() @ w.double().t()) <= TOL


@pytest.mark.parametrize("T,I,J", [(25216, 384, 1152), (18464, 3072, 768), (3000, 128, 40), (64, 8, 12)])
def test_weight_gradient_split_k(dev, T, I, J):
    """dW = X^T dY (A read m-contiguous from X: the X.t() view) with db from the ones row; the deep
    shapes split the token axis over the workspace (fixed-order reduction: bitwise repeatable)."""
    import sae_vision_amd.ops as ops
    x = _rand(dev, (T, I), T)
    dy = _rand(dev, (T, J), J)
    db = torch.empty(J, device=dev)
    dw = ops.gemm_f32(x.t(), dy, colsum=db)
    assert _rel(dw, x.double().t() @ dy.double()) <= TOL
    assert _rel(db, dy.double().sum(0)) <= TOL
    db2 = torch.empty(J, device=dev)
    dw2 = ops.gemm_f32(x.t(), dy, colsum=db2)
    assert torch.equal(dw, dw2) and torch.equal(db, db2)


@pytest.mark.parametrize("T", [500, 25216])   # unsplit / split
def test_accumulate_and_strided(dev, T):
    """accumulate=True adds into existing dW / db; operands may be column slices of wider rows."""
    import sae_vision_amd.ops as ops
    I, J = 128, 256
    xw = _rand(dev, (T, I + 64), 5)
    dyw = _rand(dev, (T, J + 8), 6)
    x, dy = xw[:, 64:], dyw[:, :J]
    dw0, db0 = _rand(dev, (I, J), 7), _rand(dev, (J,), 8)
    dw, db = dw0.clone(), db0.clone()
    ops.gemm_f32(x.t(), dy, out=dw, colsum=db, accumulate=True)
    assert _rel(dw, dw0.double() + x.double().t() @ dy.double()) <= TOL
    assert _rel(db, db0.double() + dy.double().sum(0)) <= TOL


def test_rejects_unsupported_strides(dev):
    import sae_vision_amd.ops as ops
    x = _rand(dev, (64, 30), 1)          # k extent 30: not a multiple of 4
    w = _rand(dev, (30, 16), 2)
    with pytest.raises(Exception, match="gemm_f32"):
        ops.gemm_f32(x, w)


@pytest.mark.parametrize("blocks", [[1152], [384, 384, 384]])
def test_dense_fp32_module(dev, blocks):
    """ops.dense at compute dtype float32 (the stacked queries / keys / values kernels as column
    blocks): forward and every gradient against float64 autograd, all on sae_gemm_f32."""
    import sae_vision_amd.ops as ops
    B, N, C = 4, 197, 384
    x = _rand(dev, (B, N, C), 11).requires_grad_(True)
    ws = [_rand(dev, (C, n), 12 + i, C ** -0.5).requires_grad_(True) for i, n in enumerate(blocks)]
    b = _rand(dev, (sum(blocks),), 20).requires_grad_(True)
    y = ops.dense(x, ws if len(ws) > 1 else ws[0], b, torch.float32)
    dy = _rand(dev, y.shape, 21)
    y.backward(dy)
    xd = x.detach().double().requires_grad_(True)
    wds = [w.detach().double().requires_grad_(True) for w in ws]
    bd = b.detach().double().requires_grad_(True)
    yd = xd @ torch.cat(wds, 1) + bd
    yd.backward(dy.double())
    assert _rel(y, yd) <= TOL
    assert _rel(x.grad, xd.grad) <= TOL
    assert _rel(b.grad, bd.grad) <= TOL
    for w, wd in zip(ws, wds):
        assert _rel(w.grad, wd.grad) <= TOL
