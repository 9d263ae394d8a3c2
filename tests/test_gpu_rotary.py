"""Rotary embedding fused into the attention kernels (position_embed.py:8-20 on q and k before the
scores; README to-do, survey D6): q / k are handed over un-rotated and the kernels rotate them as
they stage them (sae_attn_fwd_rotary / sae_attn_bwd_rotary / sae_th_attn_*_rotary), and rotate
dq / dk back as they store them.

Two checks per shape:
  * against the oracle (oracle/attention_ref.py: apply_rotary + attention_core_fwd / _bwd, float64)
    at the bf16 bar 2e-2;
  * bit for bit against the unfused composition (standalone sae_rotary pass, plain attention, the
    inverse rotary pass on the gradients): the fused kernels round exactly where that chain does.
The standalone pass is patched to raise inside the fused calls, so they cannot fall back to it."""
import numpy as np
import pytest

import attention_ref as R
from _util import TOL, randn, rel_err

pytestmark = pytest.mark.gpu

CORE = [  # (B, Nq, Nk, H, D)
    (2, 197, 197, 6, 64),    # DeiT-S heads (single-pass backward, Nk <= 256)
    (1, 577, 577, 2, 64),    # ViT-B@384 length (two-pass backward)
    (2, 100, 37, 3, 32),     # Nq != Nk (CvT-like), head_dim 32
    (2, 196, 196, 8, 48),    # CaiT head_dim 48 (padded 64-wide tiles)
]


def _tensors(dev, B, Nq, Nk, H, D, seed=0):
    import torch
    rng = np.random.default_rng(seed)
    q, k, v = (randn(rng, (B, n, H, D), "bf16") for n in (Nq, Nk, Nk))
    do = randn(np.random.default_rng(seed + 1), (B, Nq, H, D), "bf16")
    t = [torch.tensor(x, device=dev, dtype=torch.bfloat16, requires_grad=True) for x in (q, k, v)]
    return (q, k, v, do), t, torch.tensor(do, device=dev, dtype=torch.bfloat16)


def _no_standalone(monkeypatch):
    import sae_vision_amd.ops as ops

    def boom(*a, **k):
        raise AssertionError("standalone rotary pass called on the fused path")
    monkeypatch.setattr(ops._Rotary, "apply", boom)


@pytest.mark.parametrize("shape", CORE)
def test_rotary_fused_core(dev, monkeypatch, shape):
    import torch
    import sae_vision_amd.ops as ops
    B, Nq, Nk, H, D = shape
    (q, k, v, do), (tq, tk, tv), tdo = _tensors(dev, *shape)
    assert ops.rope_fused_ok(tq, tk, tv)
    with monkeypatch.context() as m:
        _no_standalone(m)
        o = ops.attention(tq, tk, tv, rotary=10000.0)
        o.backward(tdo)
    # oracle: rotate (float64 tables), then the float64 core
    n = max(Nq, Nk)
    s, c = R.rotary_sincos(n, D)
    qr = R.apply_rotary(q.astype(np.float64), s[:Nq], c[:Nq])
    kr = R.apply_rotary(k.astype(np.float64), s[:Nk], c[:Nk])
    assert rel_err(o, R.attention_core_fwd(qr, kr, v, "f64")) <= TOL["bf16"]
    g = R.attention_core_bwd(qr, kr, v, do)
    assert rel_err(tq.grad, R.apply_rotary(g["dq"], -s[:Nq], c[:Nq])) <= TOL["bf16"]
    assert rel_err(tk.grad, R.apply_rotary(g["dk"], -s[:Nk], c[:Nk])) <= TOL["bf16"]
    assert rel_err(tv.grad, g["dv"]) <= TOL["bf16"]
    # unfused composition, bit for bit
    uq, uk, uv = (t.detach().clone().requires_grad_(True) for t in (tq, tk, tv))
    # (the standalone pass takes its own length's table: the same rows as the fused max(Nq, Nk) one)
    ou = ops.attention(ops.rotary(uq), ops.rotary(uk), uv)
    ou.backward(tdo)
    assert torch.equal(o, ou)
    for a, b in ((tq, uq), (tk, uk), (tv, uv)):
        assert torch.equal(a.grad, b.grad)


@pytest.mark.parametrize("shape", [(2, 196, 196, 8, 48), (1, 70, 45, 12, 48), (2, 50, 50, 4, 48)])
def test_rotary_fused_talking_heads(dev, monkeypatch, shape):
    import torch
    import sae_vision_amd.ops as ops
    B, Nq, Nk, H, D = shape
    (q, k, v, do), (tq, tk, tv), tdo = _tensors(dev, *shape, seed=3)
    rng = np.random.default_rng(7)
    th1, th2 = (np.linalg.qr(rng.standard_normal((H, H)))[0].astype(np.float32) for _ in range(2))
    t1, t2 = (torch.tensor(x, device=dev, requires_grad=True) for x in (th1, th2))
    with monkeypatch.context() as m:
        _no_standalone(m)
        o = ops.talking_heads_attention(tq, tk, tv, t1, t2, rotary=10000.0)
        o.backward(tdo)
    s, c = R.rotary_sincos(max(Nq, Nk), D)
    qr = R.apply_rotary(q.astype(np.float64), s[:Nq], c[:Nq])
    kr = R.apply_rotary(k.astype(np.float64), s[:Nk], c[:Nk])
    assert rel_err(o, R.attention_core_fwd(qr, kr, v, "f64", th1=th1, th2=th2)) <= TOL["bf16"]
    g = R.attention_core_bwd(qr, kr, v, do, th1=th1, th2=th2)
    assert rel_err(tq.grad, R.apply_rotary(g["dq"], -s[:Nq], c[:Nq])) <= TOL["bf16"]
    assert rel_err(tk.grad, R.apply_rotary(g["dk"], -s[:Nk], c[:Nk])) <= TOL["bf16"]
    assert rel_err(tv.grad, g["dv"]) <= TOL["bf16"]
    assert rel_err(t1.grad, g["dth1"]) <= TOL["bf16"] and rel_err(t2.grad, g["dth2"]) <= TOL["bf16"]
    uq, uk, uv = (t.detach().clone().requires_grad_(True) for t in (tq, tk, tv))
    u1, u2 = (t.detach().clone().requires_grad_(True) for t in (t1, t2))
    ou = ops.talking_heads_attention(ops.rotary(uq), ops.rotary(uk), uv, u1, u2)
    ou.backward(tdo)
    assert torch.equal(o, ou)
    for a, b in ((tq, uq), (tk, uk), (tv, uv), (t1, u1), (t2, u2)):
        assert torch.equal(a.grad, b.grad)


@pytest.mark.parametrize("talking", [False, True])
def test_rotary_block_packed_bf16(dev, monkeypatch, talking):
    """SelfAttentionBlock(rotary=True) in bf16 stays on the packed [B, N, 3, H, D] path (one QKV GEMM,
    fused rotary inside the kernels) and matches the oracle block."""
    import torch
    import sae_vision_amd.layers as layers
    B, N, C, H = 2, 65, 128, 4
    x = np.random.default_rng(0).standard_normal((B, N, C)).astype(np.float32)
    mod = layers.SelfAttentionBlock(num_heads=H, in_ch=C, rotary=True, talking_heads=talking,
                                    dtype=torch.bfloat16, device=dev)
    tree = layers.flax_params(mod)
    p = R.AttnParams(queries=tree["queries"]["kernel"].cpu().numpy(), keys=tree["keys"]["kernel"].cpu().numpy(),
                     values=tree["values"]["kernel"].cpu().numpy(),
                     out=tree["DenseGeneral_0"]["kernel"].cpu().numpy(),
                     th1=tree["TalkingHeadsBlock_0"]["talking_heads_transform"].cpu().numpy() if talking else None,
                     th2=tree["TalkingHeadsBlock_1"]["talking_heads_transform"].cpu().numpy() if talking else None)
    tx = torch.tensor(x, device=dev, requires_grad=True)
    with monkeypatch.context() as m:
        _no_standalone(m)
        y = mod(tx, is_training=True)
        dy = np.random.default_rng(1).standard_normal(y.shape).astype(np.float32)
        y.float().backward(torch.tensor(dy, device=dev))
    assert rel_err(y.float(), R.attention_block_fwd(x, x, p, "f64", rotary=True)) <= TOL["bf16"]
    g = R.attention_block_bwd(x, x, p, dy, rotary=True)
    assert rel_err(tx.grad, g["x_q"] + g["x_kv"]) <= TOL["bf16"]
    for name in ("queries", "keys", "values", "DenseGeneral_0"):
        assert rel_err(getattr(mod, name).kernel.grad, g[name]) <= TOL["bf16"], name


def test_rotary_fused_rejects(dev):
    """The C ABI refuses what the fused kernels do not take (the ops then use the standalone pass)."""
    import ctypes
    import torch
    import sae_vision_amd.ops as ops
    from sae_vision_amd import _lib as L
    lib = L.load()
    q = torch.zeros(1, 8, 1, 64, device=dev)   # fp32
    d = ops._make_desc(q, q, q, q, 0.125)
    s = torch.zeros(8, 32, device=dev)
    rc = lib.sae_attn_fwd_rotary(None, ctypes.byref(d), q.data_ptr(), q.data_ptr(), q.data_ptr(), s.data_ptr(),
                                 s.data_ptr(), q.data_ptr(), s.data_ptr())
    assert rc == L.SAE_EUNSUPPORTED and "bf16" in lib.sae_last_error().decode()
    assert not ops.rope_fused_ok(q)
    # fp32 still works end to end (standalone pass + fp32 kernels)
    tq = torch.randn(1, 8, 1, 64, device=dev)
    o = ops.attention(tq, tq, tq, rotary=10000.0)
    assert torch.isfinite(o).all()
