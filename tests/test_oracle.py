"""CPU tests of the oracle itself (no GPU): the numpy restatement against an independent
torch-CPU autograd derivation, the BoTNet relative-logit index map against the literal
pad/reshape algorithm of botnet.py:77-111, bf16 rounding, and the committed golden fixtures."""
import glob
import os

import numpy as np
import pytest
import torch

import attention_ref as R
import vit_ref

HERE = os.path.dirname(os.path.abspath(__file__))


def _t(x):
    return torch.tensor(np.asarray(x), dtype=torch.float64, requires_grad=True)


def torch_attention_block(xq, xkv, Wq, Wk, Wv, Wo, th1=None, th2=None, rotary=False):
    """Independent torch restatement of attention.py:20-67 (float64, autograd)."""
    q = torch.einsum("bnc,chd->bnhd", xq, Wq)
    k = torch.einsum("bnc,chd->bnhd", xkv, Wk)
    v = torch.einsum("bnc,chd->bnhd", xkv, Wv)
    if rotary:
        def rot(x):
            n, d = x.shape[1], x.shape[3]
            s, c = R.rotary_sincos(n, d)
            s = torch.tensor(np.repeat(s, 2, -1))[None, :, None, :]
            c = torch.tensor(np.repeat(c, 2, -1))[None, :, None, :]
            x1, x2 = x[..., ::2], x[..., 1::2]
            r = torch.stack((-x2, x1), -1).reshape(x.shape)
            return x * c + r * s
        q, k = rot(q), rot(k)
    q = q / np.sqrt(q.shape[-1])
    s = torch.einsum("bqhd,bkhd->bhqk", q, k)
    if th1 is not None:
        s = torch.einsum("hi,bh...->bi...", th1, s)
    p = torch.softmax(s, -1)
    if th2 is not None:
        p = torch.einsum("hi,bh...->bi...", th2, p)
    o = torch.einsum("bhqk,bkhd->bqhd", p, v)
    return torch.einsum("bnhd,hdc->bnc", o, Wo)


@pytest.mark.parametrize("talking,rotary,nq", [(False, False, 13), (True, False, 13), (False, True, 13),
                                               (False, False, 1)])
def test_block_fwd_bwd_vs_torch_autograd(talking, rotary, nq):
    rng = np.random.default_rng(0)
    B, Nk, C, H, D = 2, 13, 12, 3, 4
    xkv = rng.standard_normal((B, Nk, C))
    xq = xkv[:, :nq] if nq != Nk else xkv
    Wq, Wk, Wv = (rng.standard_normal((C, H, D)) * 0.3 for _ in range(3))
    Wo = rng.standard_normal((H, D, C)) * 0.3
    th1 = np.linalg.qr(rng.standard_normal((H, H)))[0] if talking else None
    th2 = np.linalg.qr(rng.standard_normal((H, H)))[0] if talking else None
    p = R.AttnParams(Wq, Wk, Wv, Wo, th1, th2)
    y = R.attention_block_fwd(xq, xkv, p, "f64", rotary=rotary)
    dy = rng.standard_normal(y.shape)
    g = R.attention_block_bwd(xq, xkv, p, dy, rotary=rotary)

    txq, txkv = _t(xq), _t(xkv)
    tW = [_t(w) for w in (Wq, Wk, Wv, Wo)]
    tth = [_t(th1), _t(th2)] if talking else [None, None]
    ty = torch_attention_block(txq, txkv, *tW, *tth, rotary=rotary)
    np.testing.assert_allclose(ty.detach().numpy(), y, rtol=1e-10, atol=1e-12)
    ty.backward(torch.tensor(dy))
    np.testing.assert_allclose(txq.grad.numpy(), g["x_q"], rtol=1e-9, atol=1e-11)
    np.testing.assert_allclose(txkv.grad.numpy(), g["x_kv"], rtol=1e-9, atol=1e-11)
    for name, t in zip(("queries", "keys", "values", "DenseGeneral_0"), tW):
        np.testing.assert_allclose(t.grad.numpy(), g[name], rtol=1e-9, atol=1e-11)
    if talking:
        np.testing.assert_allclose(tth[0].grad.numpy(), g["TalkingHeadsBlock_0"], rtol=1e-9, atol=1e-11)
        np.testing.assert_allclose(tth[1].grad.numpy(), g["TalkingHeadsBlock_1"], rtol=1e-9, atol=1e-11)


@pytest.mark.parametrize("L", [1, 2, 5, 7, 14])
def test_to_absolute_logits_index_map(L):
    """botnet.py:77-93 pad/reshape == gather rel[i, j - i + L - 1] (exact integers)."""
    rel = np.arange(2 * 3 * L * (2 * L - 1), dtype=np.float64).reshape(2, 3, L, 2 * L - 1)
    out = R.to_absolute_logits(rel)
    i, j = np.meshgrid(np.arange(L), np.arange(L), indexing="ij")
    np.testing.assert_array_equal(out, rel[:, :, i, j - i + L - 1])


@pytest.mark.parametrize("Hs,Ws", [(7, 7), (14, 14), (5, 7), (3, 1)])
def test_relative_logits_indexed_equals_literal(Hs, Ws):
    rng = np.random.default_rng(1)
    B, H, D = 2, 2, 8
    qh = rng.integers(-4, 5, size=(B, Hs * Ws, H, D)).astype(np.float64)
    eh = rng.integers(-4, 5, size=(2 * Hs - 1, D)).astype(np.float64)
    ew = rng.integers(-4, 5, size=(2 * Ws - 1, D)).astype(np.float64)
    lit = R.relative_logits(qh.reshape(B, Hs, Ws, H, D).transpose(0, 3, 1, 2, 4), eh, ew)
    idx = R.relative_logits_indexed(qh, eh, ew, Hs, Ws)
    np.testing.assert_array_equal(lit.reshape(B, H, Hs * Ws, Hs * Ws), idx)


def test_round_bf16():
    x = np.array([1.0, 1.00390625, 1.005859375, -3.14159, 65504.0, 1e-40, np.inf, np.nan], np.float32)
    r = R.round_bf16(x)
    assert r[0] == 1.0 and r[1] == 1.0            # tie to even
    assert r[2] == np.float32(1.0078125)
    assert np.isinf(r[6]) and np.isnan(r[7])
    assert np.all((r.view(np.uint32) & 0xFFFF) == 0)
    t = torch.tensor(x).to(torch.bfloat16).float().numpy()
    np.testing.assert_array_equal(r[:6], t[:6])


def test_bf16_mode_close_to_f64():
    rng = np.random.default_rng(0)
    q, k, v = (rng.standard_normal((2, 33, 3, 64)) for _ in range(3))
    ref = R.attention_core_fwd(q, k, v, "f64")
    b = R.attention_core_fwd(q, k, v, "bf16")
    assert np.abs(b - ref).max() / np.abs(ref).max() < 2e-2


def test_vit_ref_grads_vs_torch_autograd():
    """numpy ViT training-step oracle (bench cpu_baseline) vs torch CPU autograd, tiny ViT."""
    import sae_vision_amd.vit as vit
    torch.manual_seed(0)
    m = vit.ViT(num_classes=10, num_layers=2, num_heads=2, embed_dim=16, patch_shape=(8, 8), img_size=16,
                dtype=torch.float64)
    m = m.double()
    with torch.no_grad():
        m.Dense_0.kernel.normal_(0, 0.1)
    params = {k: v.detach().numpy().copy() for k, v in m.named_parameters()}
    rng = np.random.default_rng(0)
    images = rng.standard_normal((3, 16, 16, 3))
    labels = rng.integers(0, 10, size=3)
    loss, logits, grads = vit_ref.vit_loss_and_grads(params, images, labels, 2, 2, 8)

    # torch autograd on the same math (torch reference attention instead of the HIP op)
    def fwd(P, x):
        pe = torch.tensor(vit_ref.patchify(x, 8)) @ P["PatchEmbedBlock_0.Dense_0.kernel"]
        h = torch.cat([P["cls"].expand(3, 1, 16), pe], 1) + P["Encoder_0.AddAbsPosEmbed_0.pos_embed"]
        ln = lambda t, pre: torch.nn.functional.layer_norm(t, (16,), P[pre + ".scale"], P[pre + ".bias"], 1e-6)
        for i in range(2):
            pre = f"Encoder_0.EncoderBlock_{i}."
            a = torch_attention_block(ln(h, pre + "LayerNorm_0"), ln(h, pre + "LayerNorm_0"),
                                      *(P[pre + f"SelfAttentionBlock_0.{n}.kernel"]
                                        for n in ("queries", "keys", "values", "DenseGeneral_0")))
            h = h + a
            u = ln(h, pre + "LayerNorm_1") @ P[pre + "FFBlock_0.Dense_0.kernel"] + P[pre + "FFBlock_0.Dense_0.bias"]
            f = (torch.nn.functional.gelu(u, approximate="tanh") @ P[pre + "FFBlock_0.Dense_1.kernel"]
                 + P[pre + "FFBlock_0.Dense_1.bias"])
            h = h + f
        z = ln(h, "Encoder_0.LayerNorm_0")
        return z[:, 0] @ P["Dense_0.kernel"] + P["Dense_0.bias"]

    P = {k: torch.tensor(v, requires_grad=True) for k, v in params.items()}
    lt = fwd(P, images)
    np.testing.assert_allclose(lt.detach().numpy(), logits, rtol=1e-9, atol=1e-10)
    tl = torch.nn.functional.cross_entropy(lt, torch.tensor(labels), label_smoothing=0.1)
    np.testing.assert_allclose(float(tl), loss, rtol=1e-10)
    tl.backward()
    for k, t in P.items():
        np.testing.assert_allclose(t.grad.numpy(), grads[k], rtol=1e-7, atol=1e-10, err_msg=k)


GOLDEN = sorted(glob.glob(os.path.join(HERE, "golden", "*.npz")))


@pytest.mark.parametrize("path", GOLDEN, ids=[os.path.basename(p) for p in GOLDEN])
def test_golden_fixtures_reproduce(path):
    """The committed fixtures (tests/golden/make_golden.py) are reproduced by the oracle."""
    import importlib.util
    spec = importlib.util.spec_from_file_location("make_golden", os.path.join(HERE, "golden", "make_golden.py"))
    mg = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mg)
    with np.load(path, allow_pickle=False) as f:
        data = dict(f)
    fresh = mg.compute(os.path.basename(path)[:-4], {k: v for k, v in data.items() if k.startswith("in_")})
    for k, v in fresh.items():
        np.testing.assert_allclose(v, data[k], rtol=1e-6, atol=1e-7, err_msg=k)
