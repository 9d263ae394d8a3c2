"""Host logic of ``ops.dense`` with column-block kernels (the queries / keys / values kernels of
one stacked projection, attention.py:29-37) on CPU tensors: forward equals x @ concat(W_j) and
each block's gradient is the matching column slice of the stacked gradient.  (The CPU branch is
the library path; the GPU branch is checked against the same math in test_gpu_gemm*.py.)"""
import torch


def test_dense_column_blocks_match_concat():
    import sae_vision_amd.ops as ops
    torch.manual_seed(0)
    x = torch.randn(5, 7, 16, dtype=torch.float64)
    ws = [torch.randn(16, n, dtype=torch.float64, requires_grad=True) for n in (8, 8, 8)]
    b = torch.randn(24, dtype=torch.float64, requires_grad=True)
    y = ops.dense(x, ws, b, torch.float64)
    ref_w = [w.detach().clone().requires_grad_(True) for w in ws]
    ref_b = b.detach().clone().requires_grad_(True)
    yr = x @ torch.cat(ref_w, dim=1) + ref_b
    assert torch.allclose(y, yr)
    g = torch.randn_like(yr)
    y.backward(g)
    yr.backward(g)
    for a, r in zip(ws, ref_w):
        assert torch.allclose(a.grad, r.grad)
    assert torch.allclose(b.grad, ref_b.grad)


def test_dense_single_kernel_unchanged():
    import sae_vision_amd.ops as ops
    torch.manual_seed(1)
    x = torch.randn(3, 4, 12, dtype=torch.float64, requires_grad=True)
    w = torch.randn(12, 6, dtype=torch.float64, requires_grad=True)
    y = ops.dense(x, w, None, torch.float64)
    assert torch.allclose(y, x @ w)
    y.sum().backward()
    assert torch.allclose(w.grad, x.detach().reshape(-1, 12).t() @ torch.ones(12, 6, dtype=torch.float64))
