"""ctypes wrapper of oracle/libattn_cpu.so (attn_cpu.c): the unfused fp32 attention core on the
host cores, OpenMP over (batch, head).

TEST INFRASTRUCTURE / CPU BASELINE ONLY (see attention_ref.py's header): loaded by
tests/test_cpu_attn.py (pinned there to the float64 restatement) and by bench.py's cpu_baseline
leg.  The product path never imports it.  Built by ``make -C oracle`` (``__graft_entry__.build()``).
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "libattn_cpu.so")
SAE_FLAG_RELPOS = 1


class Desc(ctypes.Structure):
    """Mirror of sae_attn_desc (include/sae_attn.h)."""
    _fields_ = [("batch", ctypes.c_int32), ("heads", ctypes.c_int32), ("seq_q", ctypes.c_int32),
                ("seq_k", ctypes.c_int32), ("head_dim", ctypes.c_int32), ("dtype", ctypes.c_int32),
                ("flags", ctypes.c_int32), ("scale", ctypes.c_float)] + \
               [(n, ctypes.c_int64 * 3) for n in ("q_stride", "k_stride", "v_stride", "o_stride", "do_stride",
                                                  "dq_stride", "dk_stride", "dv_stride")] + \
               [("rel_h", ctypes.c_int32), ("rel_w", ctypes.c_int32)]


_lib = None


def load(build: bool = True):
    global _lib
    if _lib is None:
        if build and not os.path.exists(LIB):
            subprocess.run(["make", "-C", HERE], check=True, capture_output=True)
        lib = ctypes.CDLL(LIB)
        P = ctypes.c_void_p
        lib.sae_cpu_attn_fwd.argtypes = [P, ctypes.POINTER(Desc)] + [P] * 7
        lib.sae_cpu_attn_bwd.argtypes = [P, ctypes.POINTER(Desc)] + [P] * 13
        lib.sae_cpu_attn_fwd.restype = lib.sae_cpu_attn_bwd.restype = ctypes.c_int
        lib.sae_cpu_threads.restype = ctypes.c_int
        _lib = lib
    return _lib


def _strides(x):
    return (ctypes.c_int64 * 3)(*(s // 4 for s in x.strides[:3]))


def _ptr(x):
    return None if x is None else x.ctypes.data_as(ctypes.c_void_p)


def _desc(q, k, scale, rel=None):
    B, Nq, H, D = q.shape
    d = Desc(batch=B, heads=H, seq_q=Nq, seq_k=k.shape[1], head_dim=D, dtype=0, flags=0, scale=scale)
    if rel is not None:
        d.flags, d.rel_h, d.rel_w = SAE_FLAG_RELPOS, rel[0], rel[1]
    return d


def attn_fwd(q, k, v, scale=None, bias_h=None, bias_w=None, rel=None):
    """q [B,Nq,H,D], k/v [B,Nk,H,D] fp32 -> (o, lse)."""
    q, k, v = (np.ascontiguousarray(t, np.float32) for t in (q, k, v))
    scale = 1.0 / np.sqrt(q.shape[-1]) if scale is None else scale
    d = _desc(q, k, scale, rel)
    o = np.empty_like(q)
    lse = np.empty((q.shape[0], q.shape[2], q.shape[1]), np.float32)
    for n, t in (("q", q), ("k", k), ("v", v), ("o", o)):
        setattr(d, n + "_stride", _strides(t))
    bh, bw = (None if t is None else np.ascontiguousarray(t, np.float32) for t in (bias_h, bias_w))
    rc = load().sae_cpu_attn_fwd(None, ctypes.byref(d), _ptr(q), _ptr(k), _ptr(v), _ptr(bh), _ptr(bw), _ptr(o),
                                 _ptr(lse))
    if rc:
        raise RuntimeError(f"sae_cpu_attn_fwd: {rc}")
    return o, lse


def attn_bwd(q, k, v, o, lse, do, scale=None, bias_h=None, bias_w=None, rel=None):
    """-> dict(dq, dk, dv[, dbias_h, dbias_w])."""
    q, k, v, o, do = (np.ascontiguousarray(t, np.float32) for t in (q, k, v, o, do))
    lse = np.ascontiguousarray(lse, np.float32)
    scale = 1.0 / np.sqrt(q.shape[-1]) if scale is None else scale
    d = _desc(q, k, scale, rel)
    dq, dk, dv = np.empty_like(q), np.empty_like(k), np.empty_like(v)
    for n, t in (("q", q), ("k", k), ("v", v), ("o", o), ("do", do), ("dq", dq), ("dk", dk), ("dv", dv)):
        setattr(d, n + "_stride", _strides(t))
    bh, bw = (None if t is None else np.ascontiguousarray(t, np.float32) for t in (bias_h, bias_w))
    dbh = np.empty_like(bh) if rel is not None else None
    dbw = np.empty_like(bw) if rel is not None else None
    rc = load().sae_cpu_attn_bwd(None, ctypes.byref(d), _ptr(q), _ptr(k), _ptr(v), _ptr(o), _ptr(lse), _ptr(do),
                                 _ptr(bh), _ptr(bw), _ptr(dq), _ptr(dk), _ptr(dv), _ptr(dbh), _ptr(dbw))
    if rc:
        raise RuntimeError(f"sae_cpu_attn_bwd: {rc}")
    out = dict(dq=dq, dk=dk, dv=dv)
    if rel is not None:
        out.update(dbias_h=dbh, dbias_w=dbw)
    return out


def threads() -> int:
    return int(load().sae_cpu_threads())
