"""Shared helpers for the parity tests (oracle = oracle/attention_ref.py, CPU)."""
import numpy as np

TOL = {"f32": 1e-5, "bf16": 2e-2}   # north_star: max|a-b| / max|ref|


def to_np(x):
    if hasattr(x, "detach"):
        x = x.detach().float().cpu().numpy()
    return np.asarray(x, np.float64)


def rel_err(a, ref):
    a = to_np(a)
    ref = np.asarray(ref, np.float64)
    den = np.abs(ref).max()
    return float(np.abs(a - ref).max() / (den if den > 0 else 1.0))


def bf16_round(x):
    import attention_ref as R
    return R.round_bf16(np.asarray(x, np.float32))


def randn(rng, shape, mode):
    x = rng.standard_normal(shape).astype(np.float32)
    return bf16_round(x) if mode == "bf16" else x
