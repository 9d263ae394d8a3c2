"""The C / OpenMP restatement of the unfused attention core (oracle/attn_cpu.c, the CPU baseline
of SURVEY §8d) against the float64 restatement (oracle/attention_ref.py) at the fp32 bar 1e-5:
forward (o, lse), backward (dq, dk, dv) and the BoTNet relative-logit gradients (dbias tables),
on DeiT-like, Nq != Nk (CvT), CLS-query (CaiT) and 7x7 relpos (BoTNet) shapes."""
import numpy as np
import pytest

import attention_ref as R
from _util import TOL, rel_err

C = pytest.importorskip("attn_cpu")


@pytest.fixture(scope="module", autouse=True)
def _lib():
    try:
        C.load()
    except Exception as e:   # no compiler / OpenMP runtime in this environment
        pytest.skip(f"libattn_cpu.so unavailable: {e}")


@pytest.mark.parametrize("B,Nq,Nk,H,D", [(2, 17, 17, 3, 64), (1, 100, 37, 2, 32), (2, 1, 50, 4, 48),
                                         (1, 197, 197, 2, 64)])
def test_cpu_core_matches_oracle(B, Nq, Nk, H, D):
    rng = np.random.default_rng(0)
    q = rng.standard_normal((B, Nq, H, D)).astype(np.float32)
    k, v = (rng.standard_normal((B, Nk, H, D)).astype(np.float32) for _ in range(2))
    do = rng.standard_normal((B, Nq, H, D)).astype(np.float32)
    o, lse = C.attn_fwd(q, k, v)
    ref, aux = R.attention_core_fwd(q, k, v, "f64", return_aux=True)
    assert rel_err(o, ref) <= TOL["f32"]
    assert np.abs(lse - aux["lse"]).max() <= 1e-5 * np.abs(aux["lse"]).max()
    g = C.attn_bwd(q, k, v, o, lse, do)
    gr = R.attention_core_bwd(q, k, v, do)
    for n in ("dq", "dk", "dv"):
        assert rel_err(g[n], gr[n]) <= TOL["f32"], n


def test_cpu_relpos_matches_oracle():
    B, H, Hs, Ws, D = 1, 2, 7, 7, 32
    N = Hs * Ws
    rng = np.random.default_rng(1)
    q, k, v, do = (rng.standard_normal((B, N, H, D)).astype(np.float32) for _ in range(4))
    eh = (rng.standard_normal((2 * Hs - 1, D)) / np.sqrt(D)).astype(np.float32)
    ew = (rng.standard_normal((2 * Ws - 1, D)) / np.sqrt(D)).astype(np.float32)
    sc = 1.0 / np.sqrt(D)
    bh, bw = R.relpos_bias_tables(q.astype(np.float64) * sc, eh, ew, Hs, Ws)
    bias = R.relative_logits_indexed(q.astype(np.float64) * sc, eh, ew, Hs, Ws)
    o, lse = C.attn_fwd(q, k, v, bias_h=bh, bias_w=bw, rel=(Hs, Ws))
    assert rel_err(o, R.attention_core_fwd(q, k, v, "f64", bias=bias)) <= TOL["f32"]
    g = C.attn_bwd(q, k, v, o, lse, do, bias_h=bh, bias_w=bw, rel=(Hs, Ws))
    gr = R.attention_core_bwd(q, k, v, do, bias=bias)
    for n in ("dq", "dk", "dv"):   # dq here excludes the bias path (the tables are inputs)
        assert rel_err(g[n], gr[n]) <= TOL["f32"], n
    ds = gr["dbias"].reshape(B, H, N, Hs, Ws)
    assert rel_err(g["dbias_h"], ds.sum(-1)) <= TOL["f32"]
    assert rel_err(g["dbias_w"], ds.sum(-2)) <= TOL["f32"]
