"""GPU parity of the variant epilogues and the drop-in modules against the CPU oracle:
talking heads (attention.py:44-52), BoTNet relative logits (botnet.py:70-141), rotary
(position_embed.py:8-20), CLS / last-token queries (cait.py:14, ceit.py:15)."""
import math

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


@pytest.mark.parametrize("B,N,Nk,H,D,mode", [
    (2, 196, 196, 8, 48, "f32"),     # CaiT-S24 trunk (fp32 per survey D7)
    (2, 196, 196, 8, 48, "bf16"),
    (2, 50, 50, 4, 48, "f32"),       # CaiT-XXS heads
    (1, 37, 37, 6, 64, "bf16"),      # CaiT-XS heads, ragged N
    (1, 33, 33, 3, 10, "f32"),       # scalar path
    (2, 100, 37, 3, 32, "bf16"),     # CvT talking heads (cvt_attention.py:90-98): Nq != Nk
    (1, 64, 100, 4, 48, "f32"),
    (2, 196, 196, 16, 48, "bf16"),   # cait_m_24 / _36 / _48: 16 heads (create_model.py:142-168)
    (1, 70, 45, 12, 48, "bf16"),     # 12 heads, ragged, Nq != Nk
    (2, 50, 50, 4, 48, "bf16"),      # cait_xxs heads
    (1, 45, 45, 9, 48, "bf16"),      # odd head count > 8: the last wave's second head is empty
    (1, 40, 33, 11, 32, "bf16"),     # 11 heads at head_dim 32, Nq != Nk
    (1, 45, 37, 5, 40, "bf16"),      # D 40: the 16 x 16 head-dim tail (d 32..47) half past D, ragged blocks
])
def test_talking_heads(dev, B, N, Nk, H, D, mode):
    import torch
    import sae_vision_amd.ops as ops

    rng = np.random.default_rng(0)
    q, k, v = (randn(rng, (B, n, H, D), mode) for n in (N, Nk, Nk))
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
    (14, 14, 4, 128, "f32"),    # BoTNet 14x14 at its real head dim (BASELINE configs[3])
    (14, 14, 4, 128, "bf16"),
    (14, 14, 4, 16, "f32"),     # 14x14 grid, small D
    (14, 14, 4, 16, "bf16"),    # lean kernels at 32-wide tiles
    (5, 7, 2, 32, "f32"),       # non-square grid
    (5, 7, 2, 32, "bf16"),
    (7, 7, 4, 64, "bf16"),      # lean kernels at 64-wide tiles
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
    # bf16: the oracle rounds at the reference's bf16 op boundaries (forward) and takes the bf16
    # cotangents of JAX autodiff (backward); the bar is the stated 2e-2 either way
    y_ref = R.attention_block_fwd(xq, x, p, mode)
    assert y.shape == y_ref.shape
    assert rel_err(y.float(), y_ref) <= TOL[mode]
    dy = randn(np.random.default_rng(2), y_ref.shape, mode)
    y.float().backward(torch.tensor(dy, device=dev))
    g = R.attention_block_bwd_bf16(xq, x, p, dy) if mode == "bf16" else R.attention_block_bwd(xq, x, p, dy)
    gx = g["x_kv"].copy()
    if picker is R.class_query:
        gx[:, 0:1] += g["x_q"]
    elif picker is R.lc_query:
        gx[:, -1:] += g["x_q"]
    else:
        gx += g["x_q"]
    assert rel_err(tx.grad.cpu().numpy(), gx) <= TOL[mode]
    for name in ("queries", "keys", "values", "DenseGeneral_0"):
        got = getattr(mod, name).kernel.grad.cpu().numpy()
        assert rel_err(got, g[name]) <= TOL[mode], name


@pytest.mark.parametrize("N,H,mode", [(50, 4, "f32"), (50, 4, "bf16"), (196, 8, "bf16")])
def test_talking_heads_module(dev, N, H, mode):
    """SelfAttentionBlock(talking_heads=True) -- projections, fused talking-heads core, output
    projection -- forward and EVERY gradient (x, queries / keys / values / DenseGeneral_0 kernels,
    both talking-heads transforms) against the oracle: fp32 vs the float64 chain at 1e-5, bf16 vs
    the bf16-emulated JAX-autodiff chain (fp32 mixes, survey D8) at 2e-2.  (196, 8): CaiT-S24."""
    import torch
    import sae_vision_amd.layers as layers

    B, C = 2, 96 if H == 4 else 384
    rng = np.random.default_rng(0)
    x = randn(rng, (B, N, C), mode)
    mod = layers.SelfAttentionBlock(num_heads=H, talking_heads=True, dtype=_td(mode), in_ch=C, device=dev)
    tree = layers.flax_params(mod)
    assert set(tree) == {"queries", "keys", "values", "TalkingHeadsBlock_0", "TalkingHeadsBlock_1",
                         "DenseGeneral_0"}
    p = R.AttnParams(queries=tree["queries"]["kernel"].cpu().numpy(), keys=tree["keys"]["kernel"].cpu().numpy(),
                     values=tree["values"]["kernel"].cpu().numpy(),
                     out=tree["DenseGeneral_0"]["kernel"].cpu().numpy(),
                     th1=tree["TalkingHeadsBlock_0"]["talking_heads_transform"].cpu().numpy(),
                     th2=tree["TalkingHeadsBlock_1"]["talking_heads_transform"].cpu().numpy())
    tx = torch.tensor(x, device=dev, requires_grad=True)
    y = mod(tx, is_training=True)
    assert rel_err(y.float(), R.attention_block_fwd(x, x, p, "f64" if mode == "f32" else "bf16")) <= TOL[mode]
    dy = randn(np.random.default_rng(2), (B, N, C), mode)
    y.float().backward(torch.tensor(dy, device=dev))
    g = R.attention_block_bwd(x, x, p, dy) if mode == "f32" else R.attention_block_bwd_bf16(x, x, p, dy)
    assert rel_err(tx.grad, g["x_q"] + g["x_kv"]) <= TOL[mode]
    for name in ("queries", "keys", "values", "DenseGeneral_0"):
        assert rel_err(getattr(mod, name).kernel.grad, g[name]) <= TOL[mode], name
    for name in ("TalkingHeadsBlock_0", "TalkingHeadsBlock_1"):
        got = getattr(mod, name).talking_heads_transform.grad
        assert rel_err(got, g[name]) <= TOL[mode], name


def test_vitb384_block_against_oracle(dev):
    """BASELINE configs[2] at full width: the ViT-B/16@384 SelfAttentionBlock (C 768, H 12, D 64,
    N 577 = 24 x 24 patches + CLS) in bf16 -- the packed QKV GEMM, the fused core on its N > 256
    kernels, the output projection -- forward and every gradient against the bf16-emulated oracle
    chain at 2e-2."""
    import torch
    import sae_vision_amd.layers as layers

    B, N, C, H = 2, 577, 768, 12
    rng = np.random.default_rng(0)
    x = randn(rng, (B, N, C), "bf16")
    mod = layers.SelfAttentionBlock(num_heads=H, dtype=torch.bfloat16, in_ch=C, device=dev)
    tree = layers.flax_params(mod)
    p = R.AttnParams(*(tree[n]["kernel"].cpu().numpy() for n in ("queries", "keys", "values", "DenseGeneral_0")))
    tx = torch.tensor(x, device=dev, requires_grad=True)
    y = mod(tx, is_training=True)
    assert rel_err(y.float(), R.attention_block_fwd(x, x, p, "bf16")) <= TOL["bf16"]
    dy = randn(np.random.default_rng(2), (B, N, C), "bf16")
    y.float().backward(torch.tensor(dy, device=dev))
    g = R.attention_block_bwd_bf16(x, x, p, dy)
    assert rel_err(tx.grad, g["x_q"] + g["x_kv"]) <= TOL["bf16"]
    for name in ("queries", "keys", "values", "DenseGeneral_0"):
        assert rel_err(getattr(mod, name).kernel.grad, g[name]) <= TOL["bf16"], name


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


def _botmhsa_ref(x, Wq, Wk, Wv, eh, ew, h, d):
    """Intended BoTMHSA (botnet.py:158-199 with survey decisions D1, D3, D4) in float64 torch on
    the CPU: 1x1-conv projections, qhat = q / sqrt(d), logits = qhat k^T + relative logits of
    qhat (index map p - x + H - 1, pinned bit-exactly against the reference's pad/reshape form
    by test_relpos_index_map_exact), softmax over all H*W keys, out = P V (no output projection)."""
    import torch
    b, Hs, Ws, cin = x.shape
    N = Hs * Ws
    xt = x.reshape(b, N, cin)
    q, k, v = ((xt @ W.reshape(cin, h * d)).reshape(b, N, h, d) for W in (Wq, Wk, Wv))
    qh = q / math.sqrt(d)
    xs, ys = torch.arange(N) // Ws, torch.arange(N) % Ws
    ih = xs[None, :] - xs[:, None] + Hs - 1
    iw = ys[None, :] - ys[:, None] + Ws - 1
    logits = torch.einsum("bnhd,bkhd->bhnk", qh, k)
    logits = logits + torch.einsum("bnhd,nkd->bhnk", qh, eh[ih]) + torch.einsum("bnhd,nkd->bhnk", qh, ew[iw])
    p = torch.softmax(logits, -1)
    return torch.einsum("bhnk,bkhd->bnhd", p, v).reshape(b, Hs, Ws, h * d)


@pytest.mark.parametrize("Hs,Ws,Cin,h,d,mode", [
    (7, 7, 64, 4, 16, "f32"),
    (14, 14, 256, 4, 128, "f32"),     # BoTNet-50 MHSA at 14x14, head dim 128 (configs[3])
    (14, 14, 256, 4, 128, "bf16"),
    (7, 7, 256, 4, 128, "bf16"),
])
def test_botmhsa_module(dev, Hs, Ws, Cin, h, d, mode):
    """BoTMHSA forward and backward (x, the query / key / value kernels, rel_pos_emb_h / _w)
    against float64 autograd of the intended module."""
    import torch
    import sae_vision_amd.layers as layers

    B = 2
    x = np.random.default_rng(0).standard_normal((B, Hs, Ws, Cin)).astype(np.float32)
    td = _td(mode)
    mod = layers.BoTMHSA(num_heads=h, head_ch=d, dtype=td, in_ch=Cin, device=dev)
    tree = layers.flax_params(mod)
    assert set(tree) == {"query", "key", "value", "RelativeLogits_0"} or set(tree) == {"query", "key", "value"}
    assert tuple(tree["query"]["kernel"].shape) == (1, 1, Cin, h * d)
    tx = torch.tensor(x, device=dev, requires_grad=True)
    y = mod(tx)
    assert y.shape == (B, Hs, Ws, h * d)
    dy = np.random.default_rng(1).standard_normal(y.shape).astype(np.float32)
    y.float().backward(torch.tensor(dy, device=dev))

    leaves = [torch.tensor(x, dtype=torch.float64)] + [
        torch.tensor(to_np(t), dtype=torch.float64) for t in (mod.query.kernel, mod.key.kernel, mod.value.kernel,
                                                            mod.RelativeLogits_0.rel_pos_emb_h,
                                                            mod.RelativeLogits_0.rel_pos_emb_w)]
    if mode == "bf16":   # the module computes on bf16 casts of its input and 1x1-conv kernels
        leaves = [t.float().to(torch.bfloat16).double() if i < 4 else t for i, t in enumerate(leaves)]
    for t in leaves:
        t.requires_grad_(True)
    y_ref = _botmhsa_ref(*leaves, h, d)
    y_ref.backward(torch.tensor(dy, dtype=torch.float64))
    assert rel_err(y, y_ref.detach().numpy()) <= TOL[mode]
    got = [tx.grad, mod.query.kernel.grad, mod.key.kernel.grad, mod.value.kernel.grad,
           mod.RelativeLogits_0.rel_pos_emb_h.grad, mod.RelativeLogits_0.rel_pos_emb_w.grad]
    for name, gt, lf in zip(("x", "query", "key", "value", "rel_pos_emb_h", "rel_pos_emb_w"), got, leaves):
        err = rel_err(gt, lf.grad.numpy())
        assert err <= TOL[mode], f"{name}: {err:.3e}"


@pytest.mark.parametrize("talking_heads", [False, True])
@pytest.mark.parametrize("mode", ["f32", "bf16"])
def test_cvt_attention_block(dev, talking_heads, mode):
    """CvTSelfAttentionBlock (cvt_attention.py:43-120): conv projections (query stride 1, key /
    value stride 2) into the fused core with Nq != Nk (and talking heads), output projection;
    checked against the oracle core fed with float64 torch-CPU projections of the same params."""
    import torch
    import torch.nn.functional as F
    import sae_vision_amd.layers as layers

    B, S, C, H = 2, 14, 96, 3
    D = C // H
    x = np.random.default_rng(0).standard_normal((B, S, S, C)).astype(np.float32)
    mod = layers.CvTSelfAttentionBlock(num_heads=H, talking_heads=talking_heads, dtype=_td(mode), in_ch=C,
                                       device=dev)
    tree = layers.flax_params(mod)
    assert {"ConvProjectionBlock_0", "ConvProjectionBlock_1", "ConvProjectionBlock_2", "DenseGeneral_0"} <= set(tree)
    y = mod(torch.tensor(x, device=dev), is_training=True)
    assert y.shape == (B, S * S, C)

    def proj(blk, xx, s):
        k0 = torch.tensor(to_np(blk.Conv_0.kernel)).permute(3, 2, 0, 1)
        xc = xx.permute(0, 3, 1, 2)
        H_ = xc.shape[-1]
        pad = max((math.ceil(H_ / s) - 1) * s + 3 - H_, 0)
        xc = F.pad(xc, (pad // 2, pad - pad // 2, pad // 2, pad - pad // 2))
        t = F.conv2d(xc, k0, stride=s, groups=C).permute(0, 2, 3, 1)
        mu, var = t.mean((0, 1, 2)), t.var((0, 1, 2), unbiased=False)
        t = (t - mu) / torch.sqrt(var + 1e-5)
        return t @ torch.tensor(to_np(blk.Conv_1.kernel)).reshape(C, H * D)

    xt = torch.tensor(x, dtype=torch.float64)
    q, k, v = (proj(getattr(mod, f"ConvProjectionBlock_{i}"), xt, s) for i, s in enumerate((1, 2, 2)))
    q, k, v = (t.reshape(B, -1, H, D).numpy() for t in (q, k, v))
    assert k.shape[1] == 49 and q.shape[1] == 196
    th = {}
    if talking_heads:
        th = dict(th1=to_np(mod.TalkingHeadsBlock_0.talking_heads_transform),
                  th2=to_np(mod.TalkingHeadsBlock_1.talking_heads_transform))
    o = R.attention_core_fwd(q, k, v, "f64", **th)
    y_ref = np.einsum("bnhd,hdc->bnc", o, to_np(mod.DenseGeneral_0.kernel))
    # bf16: projections, scores and output are bf16 values in the module (3 roundings on the path)
    assert rel_err(y, y_ref) <= TOL[mode]
