"""GPU parity of the variant epilogues and the drop-in modules against the CPU oracle:
talking heads (attention.py:44-52), BoTNet relative logits (botnet.py:70-141), rotary
(position_embed.py:8-20), CLS / last-token queries (cait.py:14, ceit.py:15)."""
import numpy as np
import pytest

import attention_ref as R
from _util import TOL, randn, rel_err, to_np

pytestmark = pytest.mark.gpu


def _td(mode):
    import torch
    return torch.bfloat16 if mode == "bf16" else torch.float32


def _orth(rng, h):
    a = rng.standard_normal((h, h))
    qm, r = np.linalg.qr(a)
    return (qm * np.sign(np.diag(r))).astype(np.float32)


@pytest.mark.parametrize("B,N,H,D,mode", [
    (2, 196, 8, 48, "f32"),     # CaiT-S24 trunk (fp32 per survey D7)
    (2, 196, 8, 48, "bf16"),
    (2, 50, 4, 48, "f32"),      # CaiT-XXS heads
    (1, 37, 6, 64, "bf16"),     # CaiT-XS heads, ragged N
    (1, 33, 3, 10, "f32"),      # scalar path
])
def test_talking_heads(dev, B, N, H, D, mode):
    import torch
    import sae_vision_amd.ops as ops

    rng = np.random.default_rng(0)
    q, k, v = (randn(rng, (B, N, H, D), mode) for _ in range(3))
    th1, th2 = _orth(np.random.default_rng(3), H), _orth(np.random.default_rng(4), H)
    do = randn(np.random.default_rng(2), (B, N, H, D), mode)
    td = _td(mode)
    tq, tk, tv = (torch.tensor(x, device=dev, dtype=td, requires_grad=True) for x in (q, k, v))
    t1, t2 = (torch.tensor(x, device=dev, requires_grad=True) for x in (th1, th2))
    o = ops.talking_heads_attention(tq, tk, tv, t1, t2)
    o.backward(torch.tensor(do, device=dev, dtype=td))
    o_ref = R.attention_core_fwd(q, k, v, "f64", th1=th1, th2=th2)
    assert rel_err(o, o_ref) <= TOL[mode]
    g = R.attention_core_bwd(q, k, v, do, th1=th1, th2=th2)
    for name, t in (("dq", tq), ("dk", tk), ("dv", tv), ("dth1", t1), ("dth2", t2)):
        err = rel_err(t.grad, g[name])
        assert err <= TOL[mode], f"{name}: {err:.3e}"


@pytest.mark.parametrize("Hs,Ws,H,D,mode", [
    (7, 7, 4, 128, "f32"),      # BoTNet 7x7
    (7, 7, 4, 128, "bf16"),
    (14, 14, 4, 16, "f32"),     # 14x14 grid, small D
    (5, 7, 2, 32, "f32"),       # non-square grid
])
def test_botnet_relpos(dev, Hs, Ws, H, D, mode):
    import torch
    import sae_vision_amd.ops as ops

    rng = np.random.default_rng(0)
    B, N = 2, Hs * Ws
    q, k, v = (randn(rng, (B, N, H, D), mode) for _ in range(3))
    eh = (rng.standard_normal((2 * Hs - 1, D)) * D ** -0.5).astype(np.float32)
    ew = (rng.standard_normal((2 * Ws - 1, D)) * D ** -0.5).astype(np.float32)
    do = randn(np.random.default_rng(2), (B, N, H, D), mode)
    td = _td(mode)
    tq, tk, tv = (torch.tensor(x, device=dev, dtype=td, requires_grad=True) for x in (q, k, v))
    teh, tew = (torch.tensor(x, device=dev, requires_grad=True) for x in (eh, ew))
    qhat = tq / float(np.sqrt(D))
    bh, bw = ops.relpos_bias(qhat, teh, tew, (Hs, Ws))
    o = ops.attention(qhat, tk, tv, scale=1.0, bias=(bh, bw, (Hs, Ws)))
    o.backward(torch.tensor(do, device=dev, dtype=td))

    # oracle: literal reference relative logits (pad/reshape/tile form) on the scaled query
    qh64 = q.astype(np.float64) / np.sqrt(D)
    rel = R.relative_logits(qh64.reshape(B, Hs, Ws, H, D).transpose(0, 3, 1, 2, 4), eh.astype(np.float64),
                            ew.astype(np.float64)).reshape(B, H, N, N)
    o_ref = R.attention_core_fwd(qh64, k, v, "f64", scale=1.0, bias=rel)
    assert rel_err(o, o_ref) <= TOL[mode]

    # gradients: autograd-free f64 chain rule through the index map
    g = R.attention_core_bwd(qh64, k, v, do, scale=1.0, bias=rel)
    dbias = g["dbias"]                                     # [B, H, N, N]
    xs, ys = np.arange(N) // Ws, np.arange(N) % Ws
    deh = np.zeros_like(eh, dtype=np.float64)
    dew = np.zeros_like(ew, dtype=np.float64)
    dqh = g["dq"].copy()
    dbh = np.zeros((B, H, N, Hs))
    dbw = np.zeros((B, H, N, Ws))
    for kk in range(N):
        dbh[..., xs[kk]] += dbias[..., kk]
        dbw[..., ys[kk]] += dbias[..., kk]
    for n in range(N):
        for p in range(Hs):
            m = p - xs[n] + Hs - 1
            deh[m] += np.einsum("bh,bhd->d", dbh[:, :, n, p], qh64[:, n])
            dqh[:, n] += dbh[:, :, n, p][..., None] * eh[m]
        for c in range(Ws):
            m = c - ys[n] + Ws - 1
            dew[m] += np.einsum("bh,bhd->d", dbw[:, :, n, c], qh64[:, n])
            dqh[:, n] += dbw[:, :, n, c][..., None] * ew[m]
    dq_ref = dqh / np.sqrt(D)
    for name, t, ref in (("dq", tq, dq_ref), ("dk", tk, g["dk"]), ("dv", tv, g["dv"]), ("demb_h", teh, deh),
                         ("demb_w", tew, dew)):
        err = rel_err(t.grad, ref)
        assert err <= TOL[mode], f"{name}: {err:.3e}"


def test_relpos_index_map_exact(dev):
    """One-hot embeddings make every relative-logit entry an exact small integer: the fused
    bias tables must reproduce the reference's pad/reshape index map bit-exactly."""
    import torch
    import sae_vision_amd.ops as ops

    Hs, Ws, H, D, B = 5, 7, 2, 32, 1
    N = Hs * Ws
    rng = np.random.default_rng(0)
    qh = rng.integers(-3, 4, size=(B, N, H, D)).astype(np.float32)
    eh = np.zeros((2 * Hs - 1, D), np.float32)
    ew = np.zeros((2 * Ws - 1, D), np.float32)
    for m in range(2 * Hs - 1):
        eh[m, m % D] = m + 1
    for m in range(2 * Ws - 1):
        ew[m, (m + 11) % D] = 100 * (m + 1)
    bh, bw = ops.relpos_bias(torch.tensor(qh, device=dev), torch.tensor(eh, device=dev),
                             torch.tensor(ew, device=dev), (Hs, Ws))
    kx, ky = np.arange(N) // Ws, np.arange(N) % Ws
    full = bh.cpu().numpy()[..., kx] + bw.cpu().numpy()[..., ky]
    ref = R.relative_logits(qh.reshape(B, Hs, Ws, H, D).transpose(0, 3, 1, 2, 4), eh, ew).reshape(B, H, N, N)
    assert np.array_equal(full, ref.astype(np.float32))


@pytest.mark.parametrize("mode", ["f32", "bf16"])
def test_rotary(dev, mode):
    import torch
    import sae_vision_amd.ops as ops

    rng = np.random.default_rng(0)
    B, N, H, D = 2, 197, 3, 64
    x = randn(rng, (B, N, H, D), mode)
    dy = randn(np.random.default_rng(1), (B, N, H, D), mode)
    tx = torch.tensor(x, device=dev, dtype=_td(mode), requires_grad=True)
    y = ops.rotary(tx)
    y.backward(torch.tensor(dy, device=dev, dtype=_td(mode)))
    s, c = R.rotary_sincos(N, D)
    assert rel_err(y, R.apply_rotary(x.astype(np.float64), s, c)) <= TOL[mode]
    assert rel_err(tx.grad, R.apply_rotary(dy.astype(np.float64), -s, c)) <= TOL[mode]


@pytest.mark.parametrize("cls,picker", [("ClassSelfAttentionBlock", R.class_query),
                                         ("LCSelfAttentionBlock", R.lc_query),
                                         ("SelfAttentionBlock", None)])
@pytest.mark.parametrize("mode", ["f32", "bf16"])
def test_modules_against_oracle(dev, cls, picker, mode):
    """Whole AttentionBlock (projections + fused core) vs attention_block_fwd/bwd with the
    same params, exported/imported through the Flax-layout param tree."""
    import torch
    import sae_vision_amd.layers as layers

    B, N, C, H = 2, 197, 96, 3
    rng = np.random.default_rng(0)
    x = randn(rng, (B, N, C), mode)
    mod = getattr(layers, cls)(num_heads=H, dtype=_td(mode), in_ch=C, device=dev)
    tree = layers.flax_params(mod)
    p = R.AttnParams(queries=tree["queries"]["kernel"].cpu().numpy(), keys=tree["keys"]["kernel"].cpu().numpy(),
                     values=tree["values"]["kernel"].cpu().numpy(),
                     out=tree["DenseGeneral_0"]["kernel"].cpu().numpy())
    tx = torch.tensor(x, device=dev, requires_grad=True)
    y = mod(tx, is_training=True)
    xq = picker(x) if picker else x
    y_ref = R.attention_block_fwd(xq, x, p, mode)
    assert y.shape == y_ref.shape
    assert rel_err(y.float(), y_ref) <= TOL[mode] * (2 if mode == "bf16" else 1)
    dy = randn(np.random.default_rng(2), y_ref.shape, "f32")
    y.float().backward(torch.tensor(dy, device=dev))
    g = R.attention_block_bwd(xq, x, p, dy)
    gx = g["x_kv"].copy()
    if picker is R.class_query:
        gx[:, 0:1] += g["x_q"]
    elif picker is R.lc_query:
        gx[:, -1:] += g["x_q"]
    else:
        gx += g["x_q"]
    tol = TOL[mode] * (2 if mode == "bf16" else 1)
    assert rel_err(tx.grad.cpu().numpy(), gx) <= tol
    for name in ("queries", "keys", "values", "DenseGeneral_0"):
        got = getattr(mod, name).kernel.grad.cpu().numpy()
        assert rel_err(got, g[name]) <= tol, name


def test_talking_heads_module(dev):
    import torch
    import sae_vision_amd.layers as layers

    B, N, C, H = 2, 50, 96, 4
    rng = np.random.default_rng(0)
    x = rng.standard_normal((B, N, C)).astype(np.float32)
    mod = layers.SelfAttentionBlock(num_heads=H, talking_heads=True, in_ch=C, device=dev)
    tree = layers.flax_params(mod)
    assert set(tree) == {"queries", "keys", "values", "TalkingHeadsBlock_0", "TalkingHeadsBlock_1",
                         "DenseGeneral_0"}
    p = R.AttnParams(queries=tree["queries"]["kernel"].cpu().numpy(), keys=tree["keys"]["kernel"].cpu().numpy(),
                     values=tree["values"]["kernel"].cpu().numpy(),
                     out=tree["DenseGeneral_0"]["kernel"].cpu().numpy(),
                     th1=tree["TalkingHeadsBlock_0"]["talking_heads_transform"].cpu().numpy(),
                     th2=tree["TalkingHeadsBlock_1"]["talking_heads_transform"].cpu().numpy())
    y = mod(torch.tensor(x, device=dev), is_training=False)
    assert rel_err(y, R.attention_block_fwd(x, x, p, "f64")) <= TOL["f32"]


def test_rotary_attention_block(dev):
    import torch
    import sae_vision_amd.layers as layers

    B, N, C, H = 2, 65, 64, 2
    x = np.random.default_rng(0).standard_normal((B, N, C)).astype(np.float32)
    mod = layers.SelfAttentionBlock(num_heads=H, in_ch=C, rotary=True, device=dev)
    tree = layers.flax_params(mod)
    p = R.AttnParams(queries=tree["queries"]["kernel"].cpu().numpy(), keys=tree["keys"]["kernel"].cpu().numpy(),
                     values=tree["values"]["kernel"].cpu().numpy(),
                     out=tree["DenseGeneral_0"]["kernel"].cpu().numpy())
    tx = torch.tensor(x, device=dev, requires_grad=True)
    y = mod(tx, is_training=False)
    assert rel_err(y, R.attention_block_fwd(x, x, p, "f64", rotary=True)) <= TOL["f32"]
    dy = np.random.default_rng(1).standard_normal(y.shape).astype(np.float32)
    y.backward(torch.tensor(dy, device=dev))
    g = R.attention_block_bwd(x, x, p, dy, rotary=True)
    assert rel_err(tx.grad.cpu().numpy(), g["x_q"] + g["x_kv"]) <= TOL["f32"]


def test_botmhsa_module(dev):
    import torch
    import sae_vision_amd.layers as layers

    B, Hs, Ws, Cin, h, d = 2, 7, 7, 64, 4, 16
    x = np.random.default_rng(0).standard_normal((B, Hs, Ws, Cin)).astype(np.float32)
    mod = layers.BoTMHSA(num_heads=h, head_ch=d, in_ch=Cin, device=dev)
    y = mod(torch.tensor(x, device=dev))
    assert y.shape == (B, Hs, Ws, h * d)
    Wq, Wk, Wv = (to_np(getattr(mod, n)).reshape(Cin, h, d) for n in ("query", "key", "value"))
    xt = x.reshape(B, Hs * Ws, Cin).astype(np.float64)
    q, k, v = (np.einsum("bnc,chd->bnhd", xt, W) for W in (Wq, Wk, Wv))
    eh = to_np(mod.RelativeLogits_0.rel_pos_emb_h)
    ew = to_np(mod.RelativeLogits_0.rel_pos_emb_w)
    o = R.botnet_mhsa_core_fwd(q, k, v, eh, ew, Hs, Ws, "f64")
    assert rel_err(y, o.reshape(B, Hs, Ws, h * d)) <= TOL["f32"]
