#!/usr/bin/env python3
"""Generate the golden fixtures in tests/golden/*.npz from the CPU oracle.

The reference holds no numeric vectors (shape-only tests) and cannot run here (no JAX), so
the fixtures are oracle outputs ("parity unpinned" by the reference).  Inputs
are numpy-seeded (default_rng(0) inputs, (1) params, (2) output gradients); bf16 cases use
bf16-representable inputs.  Outputs are float64 oracle results stored as float32.

    python tests/golden/make_golden.py          # (re)writes the .npz files
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "oracle"))
import attention_ref as R  # noqa: E402

# name -> (kind, dims, mode)
CASES = {
    "core_f32_b2_n17_h3_d64": ("core", dict(B=2, Nq=17, Nk=17, H=3, D=64), "f32"),
    "core_bf16_b1_n197_h2_d64": ("core", dict(B=1, Nq=197, Nk=197, H=2, D=64), "bf16"),
    "core_f32_b1_n196_h2_d48": ("core", dict(B=1, Nq=196, Nk=196, H=2, D=48), "f32"),
    "cls_bf16_b1_nq1_nk197_h4_d48": ("core", dict(B=1, Nq=1, Nk=197, H=4, D=48), "bf16"),
    "cvt_f32_b1_nq100_nk25_h1_d64": ("core", dict(B=1, Nq=100, Nk=25, H=1, D=64), "f32"),
    "th_f32_b1_n50_h4_d48": ("th", dict(B=1, Nq=50, Nk=50, H=4, D=48), "f32"),
    "relpos_f32_b1_7x7_h2_d32": ("relpos", dict(B=1, Hs=7, Ws=7, H=2, D=32), "f32"),
    "rotary_f32_b1_n17_h2_d16": ("rotary", dict(B=1, N=17, H=2, D=16), "f32"),
    "block_f32_b2_n17_c24_h3": ("block", dict(B=2, N=17, C=24, H=3), "f32"),
}


def _rn(rng, shape, mode):
    x = rng.standard_normal(shape).astype(np.float32)
    return R.round_bf16(x) if mode == "bf16" else x


def make_inputs(name):
    kind, d, mode = CASES[name]
    r0, r1, r2 = (np.random.default_rng(s) for s in (0, 1, 2))
    if kind in ("core", "th"):
        inp = {"in_q": _rn(r0, (d["B"], d["Nq"], d["H"], d["D"]), mode),
               "in_k": _rn(r0, (d["B"], d["Nk"], d["H"], d["D"]), mode),
               "in_v": _rn(r0, (d["B"], d["Nk"], d["H"], d["D"]), mode),
               "in_do": _rn(r2, (d["B"], d["Nq"], d["H"], d["D"]), mode)}
        if kind == "th":
            for i, nm in enumerate(("in_th1", "in_th2")):
                a = r1.standard_normal((d["H"], d["H"]))
                qm, rr = np.linalg.qr(a)
                inp[nm] = (qm * np.sign(np.diag(rr))).astype(np.float32)
        return inp
    if kind == "relpos":
        N = d["Hs"] * d["Ws"]
        return {"in_q": _rn(r0, (d["B"], N, d["H"], d["D"]), mode),
                "in_k": _rn(r0, (d["B"], N, d["H"], d["D"]), mode),
                "in_v": _rn(r0, (d["B"], N, d["H"], d["D"]), mode),
                "in_emb_h": (r1.standard_normal((2 * d["Hs"] - 1, d["D"])) * d["D"] ** -0.5).astype(np.float32),
                "in_emb_w": (r1.standard_normal((2 * d["Ws"] - 1, d["D"])) * d["D"] ** -0.5).astype(np.float32),
                "in_grid": np.array([d["Hs"], d["Ws"]], np.int32)}
    if kind == "rotary":
        return {"in_x": _rn(r0, (d["B"], d["N"], d["H"], d["D"]), mode)}
    if kind == "block":
        C, H = d["C"], d["H"]
        D = C // H
        return {"in_x": _rn(r0, (d["B"], d["N"], C), mode),
                "in_queries": (r1.standard_normal((C, H, D)) / np.sqrt(C)).astype(np.float32),
                "in_keys": (r1.standard_normal((C, H, D)) / np.sqrt(C)).astype(np.float32),
                "in_values": (r1.standard_normal((C, H, D)) / np.sqrt(C)).astype(np.float32),
                "in_out": (r1.standard_normal((H, D, C)) / np.sqrt(C)).astype(np.float32),
                "in_dy": _rn(r2, (d["B"], d["N"], C), mode)}
    raise KeyError(name)


def compute(name, inp):
    """Oracle outputs (float32) for fixture ``name`` from its inputs."""
    kind, d, mode = CASES[name]
    f = lambda x: np.asarray(x, np.float32)
    if kind in ("core", "th"):
        th1, th2 = inp.get("in_th1"), inp.get("in_th2")
        o, aux = R.attention_core_fwd(inp["in_q"], inp["in_k"], inp["in_v"], "f64", th1=th1, th2=th2,
                                      return_aux=True)
        g = R.attention_core_bwd(inp["in_q"], inp["in_k"], inp["in_v"], inp["in_do"], th1=th1, th2=th2)
        out = {"out_o": f(o), "out_lse": f(aux["lse"]), "out_dq": f(g["dq"]), "out_dk": f(g["dk"]),
               "out_dv": f(g["dv"])}
        if mode == "bf16":
            out["out_o_bf16emu"] = f(R.attention_core_fwd(inp["in_q"], inp["in_k"], inp["in_v"], "bf16"))
        if kind == "th":
            out["out_dth1"], out["out_dth2"] = f(g["dth1"]), f(g["dth2"])
        return out
    if kind == "relpos":
        Hs, Ws = (int(x) for x in inp["in_grid"])
        D = inp["in_q"].shape[-1]
        B, N, H, _ = inp["in_q"].shape
        qh = inp["in_q"].astype(np.float64) / np.sqrt(D)
        eh, ew = inp["in_emb_h"].astype(np.float64), inp["in_emb_w"].astype(np.float64)
        bh, bw = R.relpos_bias_tables(qh, eh, ew, Hs, Ws)
        rel = R.relative_logits(qh.reshape(B, Hs, Ws, H, D).transpose(0, 3, 1, 2, 4), eh, ew).reshape(B, H, N, N)
        o = R.attention_core_fwd(qh, inp["in_k"], inp["in_v"], "f64", scale=1.0, bias=rel)
        return {"out_bias_h": f(bh), "out_bias_w": f(bw), "out_rel_logits": f(rel), "out_o": f(o)}
    if kind == "rotary":
        x = inp["in_x"].astype(np.float64)
        s, c = R.rotary_sincos(x.shape[1], x.shape[3])
        return {"out_y": f(R.apply_rotary(x, s, c))}
    if kind == "block":
        p = R.AttnParams(inp["in_queries"], inp["in_keys"], inp["in_values"], inp["in_out"])
        y = R.attention_block_fwd(inp["in_x"], inp["in_x"], p, "f64")
        g = R.attention_block_bwd(inp["in_x"], inp["in_x"], p, inp["in_dy"])
        return {"out_y": f(y), "out_dx": f(g["x_q"] + g["x_kv"]), "out_dqueries": f(g["queries"]),
                "out_dkeys": f(g["keys"]), "out_dvalues": f(g["values"]), "out_dout": f(g["DenseGeneral_0"])}
    raise KeyError(name)


def main():
    total = 0
    for name in CASES:
        inp = make_inputs(name)
        out = compute(name, inp)
        path = os.path.join(HERE, name + ".npz")
        np.savez_compressed(path, **inp, **out)
        total += os.path.getsize(path)
        print(f"wrote {path} ({os.path.getsize(path) / 1024:.0f} KiB)")
    print(f"total {total / 1024:.0f} KiB")


if __name__ == "__main__":
    main()
