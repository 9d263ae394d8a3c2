"""GPU parity of the fused attention core (sae_attn_fwd / sae_attn_bwd through the C ABI)
against the CPU oracle (oracle/attention_ref.py restating attention.py:39-58).

Tolerances (north_star): fp32 max|a-b|/max|ref| <= 1e-5, bf16 <= 2e-2.
"""
import math

import numpy as np
import pytest

import attention_ref as R
from _util import TOL, randn, rel_err

pytestmark = pytest.mark.gpu

CASES = [
    # B, Nq, Nk, H, D, mode                       what it covers
    (2, 17, 17, 3, 64, "f32"),                   # tiny, ragged tiles
    (2, 197, 197, 6, 64, "bf16"),                # DeiT-S layer
    (2, 197, 197, 6, 64, "f32"),
    (1, 577, 577, 2, 64, "bf16"),                # ViT-B/16@384 (N >= 577)
    (2, 196, 196, 8, 48, "bf16"),                # CaiT-S24 head dim 48
    (2, 196, 196, 8, 48, "f32"),                 # CaiT trunk runs fp32 (survey D7)
    (1, 49, 49, 4, 128, "bf16"),                 # BoTNet 7x7, D = 128
    (1, 49, 49, 4, 128, "f32"),
    (2, 196, 196, 4, 128, "bf16"),               # BoTNet 14x14, D = 128 (two-pass lean backward)
    (1, 130, 70, 2, 96, "bf16"),                 # head dim 96 in 128-wide tiles, Nq != Nk
    (3, 16, 16, 4, 10, "f32"),                   # TNT inner attention, D = 10 (scalar path)
    (3, 16, 16, 4, 6, "bf16"),                   # TNT-B inner, D = 6
    (2, 1, 197, 8, 48, "bf16"),                  # CaiT class attention (Nq = 1: K/V stream kernels)
    (2, 1, 197, 4, 128, "bf16"),                 # Nq = 1 at head dim 128 (two chunks per lane)
    (1, 1, 1000, 2, 40, "bf16"),                 # Nq = 1, many key passes, head dim not a chunk multiple of 64
    (3, 1, 12, 3, 64, "bf16"),                   # CeiT LCA in bf16
    (2, 1, 12, 3, 64, "f32"),                    # CeiT LCA (Nq = 1, Nk = 12)
    (2, 100, 37, 3, 32, "bf16"),                 # CvT-style Nq != Nk
    (1, 1, 1, 1, 64, "f32"),                     # single key
    (1, 129, 65, 1, 64, "f32"),                  # tile boundaries + 1
    (1, 300, 600, 2, 64, "bf16"),                # single-pass backward: 3 key blocks, fp32 dQ partials
    (2, 64, 257, 1, 32, "bf16"),                 # key block of one key, head dim 32
    (1, 33, 513, 3, 48, "bf16"),                 # 3 key blocks, last holds one key
    (2, 3136, 784, 1, 64, "bf16"),               # CvT-13 stage 1 (Nq 56x56, Nk 28x28 after stride 2)
]


def _torch_dtype(mode):
    import torch
    return torch.bfloat16 if mode == "bf16" else torch.float32


@pytest.mark.parametrize("B,Nq,Nk,H,D,mode", CASES)
def test_attention_fwd_bwd(dev, B, Nq, Nk, H, D, mode):
    import torch
    import sae_vision_amd.ops as ops

    rng = np.random.default_rng(0)
    q, k, v = (randn(rng, (B, n, H, D), mode) for n in (Nq, Nk, Nk))
    do = randn(np.random.default_rng(2), (B, Nq, H, D), mode)
    td = _torch_dtype(mode)
    tq, tk, tv = (torch.tensor(x, device=dev, dtype=td, requires_grad=True) for x in (q, k, v))
    o = ops.attention(tq, tk, tv)
    o.backward(torch.tensor(do, device=dev, dtype=td))
    torch.cuda.synchronize()

    o_ref = R.attention_core_fwd(q, k, v, mode)
    assert rel_err(o, o_ref) <= TOL[mode]
    g = R.attention_core_bwd(q, k, v, do)
    for name, t in (("dq", tq), ("dk", tk), ("dv", tv)):
        err = rel_err(t.grad, g[name])
        assert err <= TOL[mode], f"{name}: rel err {err:.3e}"


@pytest.mark.parametrize("mode", ["f32", "bf16"])
def test_lse_matches_oracle(dev, mode):
    import torch
    import sae_vision_amd.ops as ops

    rng = np.random.default_rng(0)
    B, N, H, D = 2, 197, 3, 64
    q, k, v = (randn(rng, (B, N, H, D), mode) for _ in range(3))
    td = _torch_dtype(mode)
    o, lse = ops._fwd(*(torch.tensor(x, device=dev, dtype=td) for x in (q, k, v)), 1.0 / math.sqrt(D))
    _, aux = R.attention_core_fwd(q, k, v, "f64", return_aux=True)
    np.testing.assert_allclose(lse.cpu().numpy(), aux["lse"], rtol=0, atol=1e-4 if mode == "f32" else 2e-2)


@pytest.mark.parametrize("mode", ["f32", "bf16"])
def test_packed_qkv_strided(dev, mode):
    """q/k/v read in place from a packed [B, N, 3, H, D] projection (strided descriptor)."""
    import torch
    import sae_vision_amd.ops as ops

    rng = np.random.default_rng(1)
    B, N, H, D = 2, 197, 6, 64
    qkv = randn(rng, (B, N, 3, H, D), mode)
    do = randn(np.random.default_rng(2), (B, N, H, D), mode)
    td = _torch_dtype(mode)
    t = torch.tensor(qkv, device=dev, dtype=td, requires_grad=True)
    o = ops.attention_packed(t)
    o.backward(torch.tensor(do, device=dev, dtype=td))
    q, k, v = qkv[:, :, 0], qkv[:, :, 1], qkv[:, :, 2]
    assert rel_err(o, R.attention_core_fwd(q, k, v, mode)) <= TOL[mode]
    g = R.attention_core_bwd(q, k, v, do)
    gg = t.grad
    for i, name in enumerate(("dq", "dk", "dv")):
        assert rel_err(gg[:, :, i], g[name]) <= TOL[mode], name


@pytest.mark.parametrize("N", [197, 577])
def test_deterministic(dev, N):
    """Backward has no HBM atomics (dQ partials of several key blocks are summed in block
    order): two runs are bitwise identical."""
    import torch
    import sae_vision_amd.ops as ops

    g = torch.Generator(device="cpu").manual_seed(0)
    q, k, v = (torch.randn(2, N, 6, 64, generator=g).to(dev, torch.bfloat16).requires_grad_() for _ in range(3))
    do = torch.randn(2, N, 6, 64, generator=g).to(dev, torch.bfloat16)
    outs = []
    for _ in range(2):
        for t in (q, k, v):
            t.grad = None
        o = ops.attention(q, k, v)
        o.backward(do)
        outs.append([o.detach().clone()] + [t.grad.clone() for t in (q, k, v)])
    for a, b in zip(*outs):
        assert torch.equal(a, b)


@pytest.mark.parametrize("mode", ["f32", "bf16"])
@pytest.mark.parametrize("gain", [0.05, 0.6, 4.0, 6.0, 8.0])
def test_softmax_spike(dev, mode, gain):
    """Forces the online-softmax max to jump at a late key tile (rule 26): gain 4 jumps far past
    the lazy-rescale threshold (rescale branch; ~46 log2 units, inside the bf16 forward's
    fixed-max range), gains 6 / 8 up to ~70 / ~92 log2 units (past it: the fixed-max fallback
    sweep), gain 0.6 jumps by a few log2 units (P > 1 path), gain 0.05 barely moves it.

    bf16 rounding of the scores: the reference's bf16 einsum rounds S to
    bf16 before the softmax (attention.py:41-42); the kernels exponentiate the fp32 MFMA
    accumulator.  At large logits that rounding alone moves the reference's output by more than
    the 2e-2 bar (gain 8: the bf16-emulated oracle is 0.024 from float64, 0.025 from the same
    program with fp32 scores), so the bf16 forward is pinned to the oracle with unrounded scores
    at 2e-2 AND must be at least as close to float64 as the reference's own bf16 program."""
    import torch
    import sae_vision_amd.ops as ops

    rng = np.random.default_rng(5)
    B, N, H, D = 1, 300, 2, 64
    q = randn(rng, (B, N, H, D), mode)
    k = randn(rng, (B, N, H, D), mode) * 0.3
    v = randn(rng, (B, N, H, D), mode)
    for qi in (7, 40, 127, 200):
        k[0, 250 - qi // 2] = q[0, qi] * gain          # spike in a late tile
        k[0, qi % 64] = -q[0, qi] * gain                 # anti-spike in the first tile
    if mode == "bf16":
        k = R.round_bf16(k)
    td = torch.bfloat16 if mode == "bf16" else torch.float32
    tq, tk, tv = (torch.tensor(x, device=dev, dtype=td, requires_grad=True) for x in (q, k, v))
    o = ops.attention(tq, tk, tv)
    do = randn(np.random.default_rng(2), (B, N, H, D), mode)
    o.backward(torch.tensor(do, device=dev, dtype=td))
    o64 = R.attention_core_fwd(q, k, v, "f64")
    if mode == "f32":
        assert rel_err(o, o64) <= TOL[mode]
    else:
        assert rel_err(o, R.attention_core_fwd(q, k, v, "bf16", round_scores=False)) <= TOL[mode]
        assert rel_err(o, o64) <= max(TOL[mode], rel_err(R.attention_core_fwd(q, k, v, "bf16"), o64))
    g = R.attention_core_bwd(q, k, v, do)
    for n, t in (("dq", tq), ("dk", tk), ("dv", tv)):
        assert rel_err(t.grad, g[n]) <= TOL[mode], n


@pytest.mark.parametrize("gain", [0.05, 0.6, 4.0, 8.0])
def test_lone_key_spike(dev, gain):
    """Nk = 64 n + 1 (ViT at 384 px: 576 patches + the class token): the last key tile holds one key
    (half a tile of MFMA work, the rest masked).  A spike AT that key raises the row max in the last
    tile (rescale / fixed-max fallback); an anti-spike keeps it far below."""
    import torch
    import sae_vision_amd.ops as ops

    rng = np.random.default_rng(9)
    B, N, H, D = 1, 321, 2, 64
    q = randn(rng, (B, N, H, D), "bf16")
    k = randn(rng, (B, N, H, D), "bf16") * 0.3
    v = randn(rng, (B, N, H, D), "bf16")
    k[0, N - 1, 0] = q[0, 5, 0] * gain                # the lone key: spike for query 5 of head 0
    k[0, N - 1, 1] = -q[0, 200, 1] * gain             # and an anti-spike for query 200 of head 1
    k = R.round_bf16(k)
    tq, tk, tv = (torch.tensor(x, device=dev, dtype=torch.bfloat16, requires_grad=True) for x in (q, k, v))
    o = ops.attention(tq, tk, tv)
    do = randn(np.random.default_rng(2), (B, N, H, D), "bf16")
    o.backward(torch.tensor(do, device=dev, dtype=torch.bfloat16))
    o64 = R.attention_core_fwd(q, k, v, "f64")
    assert rel_err(o, R.attention_core_fwd(q, k, v, "bf16", round_scores=False)) <= TOL["bf16"]
    assert rel_err(o, o64) <= max(TOL["bf16"], rel_err(R.attention_core_fwd(q, k, v, "bf16"), o64))
    g = R.attention_core_bwd(q, k, v, do)
    for n, t in (("dq", tq), ("dk", tk), ("dv", tv)):
        assert rel_err(t.grad, g[n]) <= TOL["bf16"], n


@pytest.mark.parametrize("spike", [6, 12])
def test_fixed_max_fallback(dev, spike):
    """The bf16 forward keeps the running max where the first key tile put it and redoes a block
    with the tracking sweep when a row sum leaves [1, 2^64) (fwd2.h FIX).  Integer-valued q / k
    make every score exact in bf16 and fp32 (multiples of 1/8 below 128), so the oracle's
    bf16-rounded scores equal the kernel's: spike 12 puts late scores ~93 log2 units above the
    first tile's max (fallback taken), spike 6 up to ~55 units (fixed-max sweep kept)."""
    import torch
    import sae_vision_amd.ops as ops

    rng = np.random.default_rng(11)
    B, N, H, D = 2, 300, 2, 64
    q = rng.integers(-1, 2, (B, N, H, D)).astype(np.float32)
    k = rng.integers(-1, 2, (B, N, H, D)).astype(np.float32)
    v = R.round_bf16(rng.standard_normal((B, N, H, D)).astype(np.float32))
    for qi in (3, 40, 127, 200, 299):
        k[:, 250 - qi // 3] = q[:, qi] * spike    # spike in a late tile
    tq, tk, tv = (torch.tensor(x, device=dev, dtype=torch.bfloat16, requires_grad=True) for x in (q, k, v))
    o = ops.attention(tq, tk, tv)
    assert rel_err(o, R.attention_core_fwd(q, k, v, "bf16")) <= TOL["bf16"]
    do = randn(np.random.default_rng(2), (B, N, H, D), "bf16")
    o.backward(torch.tensor(do, device=dev, dtype=torch.bfloat16))
    g = R.attention_core_bwd(q, k, v, do)
    for n, t in (("dq", tq), ("dk", tk), ("dv", tv)):
        assert rel_err(t.grad, g[n]) <= TOL["bf16"], n


def test_error_reporting(dev):
    """Invalid descriptors fail loudly with the C ABI's message."""
    import torch
    import sae_vision_amd.ops as ops
    from sae_vision_amd import SaeError

    q = torch.zeros(1, 4, 1, 256, device=dev)
    with pytest.raises(SaeError, match="head_dim 256"):
        ops.attention(q, q, q)
