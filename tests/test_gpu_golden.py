"""GPU parity against the committed golden fixtures (tests/golden/*.npz, made by
tests/golden/make_golden.py from the oracle): the HIP path through the C ABI must reproduce
every stored output within the north_star tolerance (fp32 1e-5, bf16 2e-2) and the
relative-logit index map bit-exactly for integer inputs (test_gpu_variants)."""
import glob
import os

import numpy as np
import pytest

from _util import TOL, rel_err

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
FIXTURES = sorted(glob.glob(os.path.join(HERE, "golden", "*.npz")))


@pytest.mark.parametrize("path", FIXTURES, ids=[os.path.basename(p)[:-4] for p in FIXTURES])
def test_golden(dev, path):
    import torch
    import sae_vision_amd.layers as layers
    import sae_vision_amd.ops as ops

    name = os.path.basename(path)[:-4]
    kind = name.split("_")[0]
    with np.load(path, allow_pickle=False) as f:
        z = dict(f)
    mode = "bf16" if "_bf16_" in name else "f32"
    td = torch.bfloat16 if mode == "bf16" else torch.float32
    tol = TOL[mode]
    T = lambda x, dt=td, g=False: torch.tensor(x, device=dev, dtype=dt, requires_grad=g)

    if kind in ("core", "cls", "cvt", "th"):
        q, k, v = T(z["in_q"], g=True), T(z["in_k"], g=True), T(z["in_v"], g=True)
        if kind == "th":
            t1, t2 = T(z["in_th1"], torch.float32, True), T(z["in_th2"], torch.float32, True)
            o = ops.talking_heads_attention(q, k, v, t1, t2)
        else:
            o = ops.attention(q, k, v)
        o.backward(T(z["in_do"]))
        assert rel_err(o, z["out_o_bf16emu"] if mode == "bf16" else z["out_o"]) <= tol
        for n, t in (("dq", q), ("dk", k), ("dv", v)):
            assert rel_err(t.grad, z["out_" + n]) <= tol, n
        if kind == "th":
            assert rel_err(t1.grad, z["out_dth1"]) <= tol
            assert rel_err(t2.grad, z["out_dth2"]) <= tol
    elif kind == "relpos":
        Hs, Ws = (int(x) for x in z["in_grid"])
        D = z["in_q"].shape[-1]
        qhat = T(z["in_q"]) / float(np.sqrt(D))
        bh, bw = ops.relpos_bias(qhat, T(z["in_emb_h"], torch.float32), T(z["in_emb_w"], torch.float32), (Hs, Ws))
        assert rel_err(bh, z["out_bias_h"]) <= tol and rel_err(bw, z["out_bias_w"]) <= tol
        o = ops.attention(qhat, T(z["in_k"]), T(z["in_v"]), scale=1.0, bias=(bh, bw, (Hs, Ws)))
        assert rel_err(o, z["out_o"]) <= tol
    elif kind == "rotary":
        assert rel_err(ops.rotary(T(z["in_x"])), z["out_y"]) <= tol
    elif kind == "block":
        C = z["in_x"].shape[-1]
        H = z["in_queries"].shape[1]
        mod = layers.SelfAttentionBlock(num_heads=H, dtype=td, in_ch=C, device=dev)
        layers.load_flax_params(mod, {"queries": {"kernel": z["in_queries"]}, "keys": {"kernel": z["in_keys"]},
                                      "values": {"kernel": z["in_values"]},
                                      "DenseGeneral_0": {"kernel": z["in_out"]}})
        x = T(z["in_x"], torch.float32, True)
        y = mod(x, is_training=False)
        y.backward(T(z["in_dy"], torch.float32))
        assert rel_err(y, z["out_y"]) <= tol
        assert rel_err(x.grad, z["out_dx"]) <= tol
        for n, key in (("queries", "out_dqueries"), ("keys", "out_dkeys"), ("values", "out_dvalues"),
                       ("DenseGeneral_0", "out_dout")):
            assert rel_err(getattr(mod, n).kernel.grad, z[key]) <= tol, n
    else:
        pytest.fail(f"unknown fixture kind {kind}")
