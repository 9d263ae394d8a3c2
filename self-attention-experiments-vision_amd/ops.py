"""Autograd operators over the C ABI (include/sae_attn.h).

Each ``torch.autograd.Function`` below is a thin host-side shim: it allocates outputs with
the framework's caching allocator, fills an ``sae_attn_desc`` with the tensors' element
strides, and calls the HIP library on the current stream.  Forward saves the log-sum-exp
rows, never the [B, H, Nq, Nk] probabilities (the reference materialises them:
models/layers/attentions/attention.py:41-58).

Public functions
  attention(q, k, v, scale, bias=None)         core of AttentionBlock (attention.py:39-58)
  attention_packed(qkv, scale)                  same, q/k/v packed [B, N, 3, H, D] (one buffer,
                                                one gradient buffer, no copies)
  talking_heads_attention(q, k, v, th1, th2, scale)   attention.py:41-52 with talking_heads
  relpos_bias(qhat, emb_h, emb_w, grid)         BoTNet RelativeLogits tables (botnet.py:70-141)
  rotary(x, base=10000.)                        rotary embedding (position_embed.py:8-20)
"""
from __future__ import annotations

import contextlib
import ctypes
import math
import os
from typing import Optional, Tuple

import torch

from . import _lib as L

__all__ = ["attention", "attention_packed", "dense", "ff_block", "gemm_nt", "weight_cast", "cast_weights", "clear_weight_cache", "gemm_dw", "set_weight_grad_stream", "join_weight_grad_stream", "layer_norm", "add_layer_norm", "add_layer_norm_scaled", "layer_norm_ok", "talking_heads_attention", "talking_heads_attention_packed", "relpos_bias", "rotary",
           "rotary_tables", "dtype_code", "KernelTimer", "set_kernel_timer"]


class KernelTimer:
    """Brackets every C-ABI launch group with HIP events on the launch stream (used by
    bench.py to time the fused kernels inside the timed region of a training step)."""

    def __init__(self):
        self.events = {}

    def begin(self, name):
        e0 = torch.cuda.Event(enable_timing=True)
        e0.record(torch.cuda.current_stream())
        return name, e0

    def end(self, token, work=None):
        name, e0 = token
        e1 = torch.cuda.Event(enable_timing=True)
        e1.record(torch.cuda.current_stream())
        self.events.setdefault(name, []).append((e0, e1, work))

    def summary(self):
        torch.cuda.synchronize()
        out = {}
        for name, lst in self.events.items():
            ms = [a.elapsed_time(b) for a, b, _ in lst]
            out[name] = {"launches": len(ms), "total_ms": sum(ms), "mean_ms": sum(ms) / max(1, len(ms)),
                         "work": [w for _, _, w in lst]}
        return out


_TIMER = None


def _sinking(bwd):
    """Backward of an op that may write gradient sinks (the flat DP buffer, see set_grad_sinks):
    once its kernels are enqueued, report every sink it claimed to the sink listener (the training
    step launches a gradient bucket's all-reduce as soon as all of the bucket's gradients are
    written, overlapping it with the rest of the backward)."""
    import functools

    @functools.wraps(bwd)
    def wrapped(ctx, *grads):
        n0 = len(_CLAIM_LOG)
        out = bwd(ctx, *grads)
        if len(_CLAIM_LOG) > n0:
            done = _CLAIM_LOG[n0:]
            del _CLAIM_LOG[n0:]
            if _SINK_LISTENER is not None:
                if _WG_STREAM is not None:
                    # a sink may have been written on the weight-gradient stream: the listener's
                    # collective waits on that stream, which first picks up the main stream's work
                    _WG_STREAM.wait_stream(torch.cuda.current_stream(_WG_STREAM.device))
                with torch.cuda.stream(_WG_STREAM) if _WG_STREAM is not None else contextlib.nullcontext():
                    for ptr in done:
                        _SINK_LISTENER(ptr)
        return out
    return wrapped


def occupy_cus(stream, workgroups: int, usec: float, threads: int = 256, lds_bytes: int = 64 * 1024) -> None:
    """Diagnostic (``sae_occupy_cus``): ``workgroups`` workgroups that hold their CUs for ``usec``
    microseconds on ``stream`` -- the CU footprint of an RCCL all-reduce's ring channels, for the
    one-GPU contention emulation of the data-parallel step (bench.py --emulate-rccl)."""
    lib = L.load()
    L.check(lib.sae_occupy_cus(ctypes.c_void_p(stream.cuda_stream), int(workgroups), int(threads), int(lds_bytes),
                               float(usec)))


def flag_bump(flags: torch.Tensor, index: int) -> None:
    """flags[index] += 1 on the current stream (``sae_flag_bump``; flags int32 on the GPU): a mark in
    a captured kernel chain that another stream can wait for (``stream_wait_flag``)."""
    lib = L.load()
    _require_gpu(flags)
    L.check(lib.sae_flag_bump(_stream(flags), ctypes.c_void_p(flags.data_ptr()), int(index)))


def stream_wait_flag(stream, flags: torch.Tensor, index: int, value: int) -> None:
    """Make ``stream`` wait until flags[index] >= value (``sae_stream_wait_flag``)."""
    lib = L.load()
    _require_gpu(flags)
    L.check(lib.sae_stream_wait_flag(ctypes.c_void_p(stream.cuda_stream),
                                     ctypes.c_void_p(flags.data_ptr() + 4 * int(index)), int(value) & 0xffffffff))


def set_kernel_timer(t):
    global _TIMER
    _TIMER = t


def dtype_code(dt: torch.dtype) -> int:
    if dt == torch.bfloat16:
        return L.SAE_DTYPE_BF16
    if dt == torch.float32:
        return L.SAE_DTYPE_F32
    raise TypeError(f"sae_vision_amd kernels take bfloat16 or float32, got {dt}")


def _require_gpu(*ts: torch.Tensor):
    for t in ts:
        if t is not None and not t.is_cuda:
            raise RuntimeError("sae_vision_amd attention runs on the GPU only (HIP kernels); "
                               f"got a tensor on {t.device}")


def _bnh(t: torch.Tensor):
    if t.dim() != 4:
        raise ValueError(f"expected a [B, N, H, D] tensor, got shape {tuple(t.shape)}")
    if t.stride(3) != 1:
        raise ValueError("head_dim must be the innermost (stride-1) dimension")
    return (t.stride(0), t.stride(1), t.stride(2))


def _stream(t: torch.Tensor) -> int:
    return torch.cuda.current_stream(t.device).cuda_stream


def _ptr(t: Optional[torch.Tensor]):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def _make_desc(q, k, v, o, scale, dout=None, dq=None, dk=None, dv=None, grid=None) -> L.SaeAttnDesc:
    lib = L.load()
    B, Nq, H, D = q.shape
    Nk = k.shape[1]
    if k.shape != (B, Nk, H, D) or v.shape != (B, Nk, H, D):
        raise ValueError(f"q {tuple(q.shape)} / k {tuple(k.shape)} / v {tuple(v.shape)} mismatch")
    if not (q.dtype == k.dtype == v.dtype):
        raise TypeError("q, k and v must share a dtype")
    d = L.SaeAttnDesc()
    lib.sae_attn_desc_init(ctypes.byref(d), B, H, Nq, Nk, D, dtype_code(q.dtype), float(scale))
    d.q_stride, d.k_stride, d.v_stride = L.s3(_bnh(q)), L.s3(_bnh(k)), L.s3(_bnh(v))
    if o is not None:
        d.o_stride = L.s3(_bnh(o))
    if dout is not None:
        d.do_stride, d.dq_stride = L.s3(_bnh(dout)), L.s3(_bnh(dq))
        d.dk_stride, d.dv_stride = L.s3(_bnh(dk)), L.s3(_bnh(dv))
    if grid is not None:
        d.flags = L.SAE_FLAG_RELPOS
        d.rel_h, d.rel_w = int(grid[0]), int(grid[1])
    return d


def _rope_tabs(q, k, rope):
    """(sin, cos) fp32 [max(Nq, Nk), D / 2] for the fused-rotary entry points (``rope`` = base)."""
    return rotary_tables(max(q.shape[1], k.shape[1]), q.shape[-1], q.device, rope)


def rope_fused_ok(*ts: torch.Tensor) -> bool:
    """Whether the fused-rotary kernels take these [B, N, H, D] tensors (sae_attn_*_rotary:
    bf16, head_dim % 8 == 0 and <= 64, 16-byte aligned token / head strides)."""
    t0 = ts[0]
    D = t0.shape[-1]
    return (t0.dtype == torch.bfloat16 and D % 8 == 0 and D <= 64 and
            all(t.stride(-1) == 1 and t.stride(0) % 8 == 0 and t.stride(1) % 8 == 0 and t.stride(2) % 8 == 0
                and t.data_ptr() % 16 == 0 for t in ts))


def _fwd(q, k, v, scale, bias_h=None, bias_w=None, grid=None, rope=None):
    lib = L.load()
    B, Nq, H, D = q.shape
    o = torch.empty((B, Nq, H, D), dtype=q.dtype, device=q.device)
    lse = torch.empty((B, H, Nq), dtype=torch.float32, device=q.device)
    d = _make_desc(q, k, v, o, scale, grid=grid)
    tok = _TIMER.begin("attn_fwd") if _TIMER is not None else None
    if rope is not None:   # q / k un-rotated: the kernels rotate them while staging
        sin, cos = _rope_tabs(q, k, rope)
        L.check(lib.sae_attn_fwd_rotary(_stream(q), ctypes.byref(d), _ptr(q), _ptr(k), _ptr(v), _ptr(sin),
                                        _ptr(cos), _ptr(o), _ptr(lse)))
    else:
        L.check(lib.sae_attn_fwd(_stream(q), ctypes.byref(d), _ptr(q), _ptr(k), _ptr(v), _ptr(bias_h),
                                 _ptr(bias_w), _ptr(o), _ptr(lse)))
    if tok is not None:
        _TIMER.end(tok, (B, Nq, k.shape[1], H, D))
    return o, lse


def _bwd(q, k, v, o, lse, do, dq, dk, dv, scale, bias_h=None, bias_w=None, grid=None, rope=None):
    lib = L.load()
    d = _make_desc(q, k, v, o, scale, do, dq, dk, dv, grid=grid)
    ws = torch.empty(lib.sae_attn_bwd_workspace_bytes(ctypes.byref(d)), dtype=torch.uint8, device=q.device)
    dbh = dbw = None
    if grid is not None:
        dbh, dbw = torch.empty_like(bias_h), torch.empty_like(bias_w)
    tok = _TIMER.begin("attn_bwd") if _TIMER is not None else None
    if rope is not None:   # dq / dk for the un-rotated q / k
        sin, cos = _rope_tabs(q, k, rope)
        L.check(lib.sae_attn_bwd_rotary(_stream(q), ctypes.byref(d), _ptr(q), _ptr(k), _ptr(v), _ptr(o), _ptr(lse),
                                        _ptr(do), _ptr(sin), _ptr(cos), _ptr(dq), _ptr(dk), _ptr(dv), _ptr(ws)))
    else:
        L.check(lib.sae_attn_bwd(_stream(q), ctypes.byref(d), _ptr(q), _ptr(k), _ptr(v), _ptr(o), _ptr(lse),
                                 _ptr(do), _ptr(bias_h), _ptr(bias_w), _ptr(dq), _ptr(dk), _ptr(dv), _ptr(dbh),
                                 _ptr(dbw), _ptr(ws)))
    if tok is not None:
        _TIMER.end(tok, tuple(q.shape[:2]) + (k.shape[1],) + tuple(q.shape[2:]))
    return dbh, dbw


def _grad_in(g: torch.Tensor) -> torch.Tensor:
    return g if g.stride(-1) == 1 else g.contiguous()


class _Attention(torch.autograd.Function):
    @staticmethod
    def forward(ctx, q, k, v, scale, bias_h, bias_w, grid, rope):
        _require_gpu(q, k, v)
        o, lse = _fwd(q, k, v, scale, bias_h, bias_w, grid, rope)
        ctx.save_for_backward(q, k, v, o, lse, bias_h, bias_w)
        ctx.scale, ctx.grid, ctx.rope = scale, grid, rope
        return o

    @staticmethod
    @_sinking
    def backward(ctx, do):
        q, k, v, o, lse, bias_h, bias_w = ctx.saved_tensors
        do = _grad_in(do)
        dq = torch.empty(q.shape, dtype=q.dtype, device=q.device)
        dk = torch.empty(k.shape, dtype=k.dtype, device=k.device)
        dv = torch.empty(v.shape, dtype=v.dtype, device=v.device)
        dbh, dbw = _bwd(q, k, v, o, lse, do, dq, dk, dv, ctx.scale, bias_h, bias_w, ctx.grid, ctx.rope)
        return dq, dk, dv, None, dbh, dbw, None, None


class _AttentionPacked(torch.autograd.Function):
    @staticmethod
    def forward(ctx, qkv, scale, rope):
        _require_gpu(qkv)
        q, k, v = qkv[:, :, 0], qkv[:, :, 1], qkv[:, :, 2]
        o, lse = _fwd(q, k, v, scale, rope=rope)
        ctx.save_for_backward(qkv, o, lse)
        ctx.scale, ctx.rope = scale, rope
        return o

    @staticmethod
    @_sinking
    def backward(ctx, do):
        qkv, o, lse = ctx.saved_tensors
        do = _grad_in(do)
        dqkv = torch.empty(qkv.shape, dtype=qkv.dtype, device=qkv.device)
        _bwd(qkv[:, :, 0], qkv[:, :, 1], qkv[:, :, 2], o, lse, do, dqkv[:, :, 0], dqkv[:, :, 1], dqkv[:, :, 2],
             ctx.scale, rope=ctx.rope)
        return dqkv, None, None


def attention(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor, scale: Optional[float] = None,
              bias: Optional[Tuple[torch.Tensor, torch.Tensor, Tuple[int, int]]] = None,
              rotary: Optional[float] = None) -> torch.Tensor:
    """softmax(scale * q k^T [+ relpos bias]) v on token-major [B, N, H, D] tensors.

    ``scale`` defaults to the reference's 1/sqrt(head_ch) (attention.py:39).  ``bias`` is
    ``(bias_h, bias_w, (Hs, Ws))`` from :func:`relpos_bias` (BoTNet).  ``rotary`` (a base, e.g.
    10000.0): q and k are rotated first (position_embed.py:8-20) -- inside the kernels' staging
    where they take it (:func:`rope_fused_ok`), else by the standalone rotary pass."""
    if scale is None:
        scale = 1.0 / math.sqrt(q.shape[-1])
    if rotary is not None and bias is None:
        if rope_fused_ok(q, k, v):
            return _Attention.apply(q, k, v, float(scale), None, None, None, float(rotary))
        q, k = _Rotary.apply(q, float(rotary)), _Rotary.apply(k, float(rotary))
    elif rotary is not None:
        q, k = _Rotary.apply(q, float(rotary)), _Rotary.apply(k, float(rotary))
    if bias is None:
        return _Attention.apply(q, k, v, float(scale), None, None, None, None)
    bh, bw, grid = bias
    return _Attention.apply(q, k, v, float(scale), bh, bw, tuple(grid), None)


def attention_packed(qkv: torch.Tensor, scale: Optional[float] = None, rotary: Optional[float] = None) -> torch.Tensor:
    """Self-attention on a packed projection ``qkv`` [B, N, 3, H, D] (one fused QKV GEMM output);
    ``rotary`` as in :func:`attention`."""
    if qkv.dim() != 5 or qkv.shape[2] != 3:
        raise ValueError(f"expected qkv [B, N, 3, H, D], got {tuple(qkv.shape)}")
    if scale is None:
        scale = 1.0 / math.sqrt(qkv.shape[-1])
    if rotary is not None and not rope_fused_ok(qkv[:, :, 0]):
        return attention(qkv[:, :, 0], qkv[:, :, 1], qkv[:, :, 2], scale, rotary=rotary)
    return _AttentionPacked.apply(qkv, float(scale), None if rotary is None else float(rotary))


# ----------------------------------------------------------------------------- talking heads
def _th_fwd(q, k, v, th1, th2, scale, rope=None):
    lib = L.load()
    B, Nq, H, D = q.shape
    th1c = th1.detach().to(torch.float32).contiguous()
    th2c = th2.detach().to(torch.float32).contiguous()
    o = torch.empty((B, Nq, H, D), dtype=q.dtype, device=q.device)
    lse = torch.empty((B, H, Nq), dtype=torch.float32, device=q.device)
    d = _make_desc(q, k, v, o, scale)
    tok = _TIMER.begin("th_attn_fwd") if _TIMER is not None else None
    if rope is not None:
        sin, cos = _rope_tabs(q, k, rope)
        L.check(lib.sae_th_attn_fwd_rotary(_stream(q), ctypes.byref(d), _ptr(q), _ptr(k), _ptr(v), _ptr(th1c),
                                           _ptr(th2c), _ptr(sin), _ptr(cos), _ptr(o), _ptr(lse)))
    else:
        L.check(lib.sae_th_attn_fwd(_stream(q), ctypes.byref(d), _ptr(q), _ptr(k), _ptr(v), _ptr(th1c),
                                    _ptr(th2c), _ptr(o), _ptr(lse)))
    if tok is not None:
        _TIMER.end(tok, (B, Nq, k.shape[1], H, D))
    return o, lse, th1c, th2c


def _th_bwd(q, k, v, th1, th2, lse, do, dq, dk, dv, scale, rope=None, dth1=None, dth2=None):
    """dT1 / dT2 go into ``dth1`` / ``dth2`` when given (fp32 [H, H]: the transforms' gradient
    sinks -- the reduce kernel writes them whole), else into fresh tensors."""
    lib = L.load()
    dth1 = torch.empty_like(th1) if dth1 is None else dth1
    dth2 = torch.empty_like(th2) if dth2 is None else dth2
    d = _make_desc(q, k, v, None, scale, do, dq, dk, dv)
    ws = torch.empty(lib.sae_th_attn_bwd_workspace_bytes(ctypes.byref(d)), dtype=torch.uint8, device=q.device)
    tok = _TIMER.begin("th_attn_bwd") if _TIMER is not None else None
    if rope is not None:
        sin, cos = _rope_tabs(q, k, rope)
        L.check(lib.sae_th_attn_bwd_rotary(_stream(q), ctypes.byref(d), _ptr(q), _ptr(k), _ptr(v), _ptr(th1),
                                           _ptr(th2), _ptr(lse), _ptr(do), _ptr(sin), _ptr(cos), _ptr(dq), _ptr(dk),
                                           _ptr(dv), _ptr(dth1), _ptr(dth2), _ptr(ws)))
    else:
        L.check(lib.sae_th_attn_bwd(_stream(q), ctypes.byref(d), _ptr(q), _ptr(k), _ptr(v), _ptr(th1), _ptr(th2),
                                    _ptr(lse), _ptr(do), _ptr(dq), _ptr(dk), _ptr(dv), _ptr(dth1), _ptr(dth2),
                                    _ptr(ws)))
    if tok is not None:
        _TIMER.end(tok, tuple(q.shape))
    return dth1, dth2


def _th_sinks(th1, th2):
    """Gradient sinks of the two transforms (fp32 contiguous parameters only: the reduce kernel
    writes fp32 [H, H] in place), or None each."""
    ok = lambda t: t.dtype == torch.float32 and t.is_contiguous() and t.data_ptr() % 16 == 0
    s1 = _sink(th1) if ok(th1) else None
    s2 = _sink(th2) if ok(th2) else None
    if s1 is not None and s2 is not None and s1.data_ptr() == s2.data_ptr():
        # one parameter used as both transforms: autograd adds the two gradients.  Sink neither:
        # a sink counts as final the moment its kernel is enqueued (the overlapped all-reduce
        # launches its bucket then), so sinking dT1 while autograd still adds dT2 into the same
        # view would race the bucket's all-reduce; the post-accumulate hook marks it ready instead
        s1 = s2 = None
    return s1, s2


class _TalkingHeads(torch.autograd.Function):
    @staticmethod
    def forward(ctx, q, k, v, th1, th2, scale, rope):
        _require_gpu(q, k, v, th1, th2)
        o, lse, th1c, th2c = _th_fwd(q, k, v, th1, th2, scale, rope)
        ctx.save_for_backward(q, k, v, th1c, th2c, lse)
        ctx.scale, ctx.rope = scale, rope
        ctx.th_dtypes = (th1.dtype, th2.dtype)
        ctx.sinks = _th_sinks(th1, th2)
        return o

    @staticmethod
    @_sinking
    def backward(ctx, do):
        q, k, v, th1, th2, lse = ctx.saved_tensors
        do = _grad_in(do)
        dq, dk, dv = (torch.empty(t.shape, dtype=t.dtype, device=t.device) for t in (q, k, v))
        s1, s2 = ctx.sinks
        dth1, dth2 = _th_bwd(q, k, v, th1, th2, lse, do, dq, dk, dv, ctx.scale, ctx.rope, _claim(s1), _claim(s2))
        return (dq, dk, dv, _unsunk(dth1.to(ctx.th_dtypes[0]), s1), _unsunk(dth2.to(ctx.th_dtypes[1]), s2), None,
                None)


class _TalkingHeadsPacked(torch.autograd.Function):
    """Talking heads on the packed projection [B, N, 3, H, D]: dq / dk / dv land in ONE gradient
    buffer through strides (no per-view gradient accumulation passes)."""

    @staticmethod
    def forward(ctx, qkv, th1, th2, scale, rope):
        _require_gpu(qkv, th1, th2)
        o, lse, th1c, th2c = _th_fwd(qkv[:, :, 0], qkv[:, :, 1], qkv[:, :, 2], th1, th2, scale, rope)
        ctx.save_for_backward(qkv, th1c, th2c, lse)
        ctx.scale, ctx.rope = scale, rope
        ctx.th_dtypes = (th1.dtype, th2.dtype)
        ctx.sinks = _th_sinks(th1, th2)
        return o

    @staticmethod
    @_sinking
    def backward(ctx, do):
        qkv, th1, th2, lse = ctx.saved_tensors
        do = _grad_in(do)
        dqkv = torch.empty(qkv.shape, dtype=qkv.dtype, device=qkv.device)
        s1, s2 = ctx.sinks
        dth1, dth2 = _th_bwd(qkv[:, :, 0], qkv[:, :, 1], qkv[:, :, 2], th1, th2, lse, do, dqkv[:, :, 0],
                             dqkv[:, :, 1], dqkv[:, :, 2], ctx.scale, ctx.rope, _claim(s1), _claim(s2))
        return dqkv, _unsunk(dth1.to(ctx.th_dtypes[0]), s1), _unsunk(dth2.to(ctx.th_dtypes[1]), s2), None, None


def _th_rope_ok(q, k, v) -> bool:
    return rope_fused_ok(q, k, v) and q.shape[2] <= L.SAE_TH_MAX_HEADS


def talking_heads_attention_packed(qkv, th1, th2, scale: Optional[float] = None, rotary: Optional[float] = None):
    """Talking-heads self-attention on a packed projection ``qkv`` [B, N, 3, H, D]; ``rotary`` as
    in :func:`attention`."""
    if qkv.dim() != 5 or qkv.shape[2] != 3:
        raise ValueError(f"expected qkv [B, N, 3, H, D], got {tuple(qkv.shape)}")
    if scale is None:
        scale = 1.0 / math.sqrt(qkv.shape[-1])
    q, k, v = qkv[:, :, 0], qkv[:, :, 1], qkv[:, :, 2]
    if rotary is not None and not _th_rope_ok(q, k, v):
        return talking_heads_attention(q, k, v, th1, th2, scale, rotary)
    return _TalkingHeadsPacked.apply(qkv, th1, th2, float(scale), None if rotary is None else float(rotary))


def talking_heads_attention(q, k, v, th1, th2, scale: Optional[float] = None, rotary: Optional[float] = None):
    """Talking-heads attention (attention.py:41-58, talking_heads.py:9-14); th1/th2 are the
    fp32 [H, H] ``talking_heads_transform`` params of TalkingHeadsBlock_0 / _1; ``rotary`` as in
    :func:`attention`."""
    if scale is None:
        scale = 1.0 / math.sqrt(q.shape[-1])
    if rotary is not None and not _th_rope_ok(q, k, v):
        q, k = _Rotary.apply(q, float(rotary)), _Rotary.apply(k, float(rotary))
        rotary = None
    return _TalkingHeads.apply(q, k, v, th1, th2, float(scale), None if rotary is None else float(rotary))


# ------------------------------------------------------------------------ relative logits
class _RelposBias(torch.autograd.Function):
    @staticmethod
    def forward(ctx, qhat, emb_h, emb_w, Hs, Ws):
        _require_gpu(qhat, emb_h, emb_w)
        lib = L.load()
        B, N, H, D = qhat.shape
        if N != Hs * Ws:
            raise ValueError(f"relpos grid {Hs}x{Ws} does not match {N} tokens")
        eh = emb_h.detach().to(torch.float32).contiguous()
        ew = emb_w.detach().to(torch.float32).contiguous()
        bh = torch.empty((B, H, N, Hs), dtype=torch.float32, device=qhat.device)
        bw = torch.empty((B, H, N, Ws), dtype=torch.float32, device=qhat.device)
        L.check(lib.sae_relpos_bias_fwd(_stream(qhat), B, H, Hs, Ws, D, dtype_code(qhat.dtype), _ptr(qhat),
                                        L.s3(_bnh(qhat)), _ptr(eh), _ptr(ew), _ptr(bh), _ptr(bw)))
        ctx.save_for_backward(qhat, eh, ew)
        ctx.grid = (Hs, Ws)
        ctx.emb_dtypes = (emb_h.dtype, emb_w.dtype)
        return bh, bw

    @staticmethod
    @_sinking
    def backward(ctx, dbh, dbw):
        qhat, eh, ew = ctx.saved_tensors
        lib = L.load()
        Hs, Ws = ctx.grid
        B, N, H, D = qhat.shape
        dbh = dbh.contiguous() if dbh is not None else torch.zeros((B, H, N, Hs), device=qhat.device)
        dbw = dbw.contiguous() if dbw is not None else torch.zeros((B, H, N, Ws), device=qhat.device)
        dq = torch.empty((B, N, H, D), dtype=qhat.dtype, device=qhat.device)
        deh, dew = torch.empty_like(eh), torch.empty_like(ew)
        ws = torch.empty(lib.sae_relpos_bias_bwd_workspace_bytes(B, Hs, Ws, D), dtype=torch.uint8,
                         device=qhat.device)
        L.check(lib.sae_relpos_bias_bwd(_stream(qhat), B, H, Hs, Ws, D, dtype_code(qhat.dtype), _ptr(qhat),
                                        L.s3(_bnh(qhat)), _ptr(eh), _ptr(ew), _ptr(dbh), _ptr(dbw), None, _ptr(dq),
                                        L.s3(_bnh(dq)), _ptr(deh), _ptr(dew), _ptr(ws)))
        return dq, deh.to(ctx.emb_dtypes[0]), dew.to(ctx.emb_dtypes[1]), None, None


def relpos_bias(qhat, emb_h, emb_w, grid: Tuple[int, int]):
    """BoTNet RelativeLogits (botnet.py:113-141) as two fp32 tables per query row:
    bias_h [B,H,N,Hs], bias_w [B,H,N,Ws]; the attention kernel adds
    ``bias_h[q, k // Ws] + bias_w[q, k % Ws]`` to the score tile."""
    return _RelposBias.apply(qhat, emb_h, emb_w, int(grid[0]), int(grid[1]))


# ---------------------------------------------------------------------------------- rotary
_TABLES = {}


def rotary_tables(n: int, dim: int, device, base: float = 10000.0):
    """fp32 sin/cos tables [n, dim/2] computed in float64 on the host (exact angles for the
    long CvT sequences; device sinf at |theta| ~ 3e3 would lose ~1e-4)."""
    key = (n, dim, float(base), str(device))
    t = _TABLES.get(key)
    if t is None:
        i = torch.arange(dim // 2, dtype=torch.float64)
        inv_freq = base ** (-2.0 * i / dim)
        ang = torch.arange(n, dtype=torch.float64)[:, None] * inv_freq[None, :]
        t = (torch.sin(ang).float().to(device), torch.cos(ang).float().to(device))
        _TABLES[key] = t
    return t


def _rotary_call(x, y, sin, cos, inverse):
    lib = L.load()
    B, N, H, D = x.shape
    L.check(lib.sae_rotary(_stream(x), B, N, H, D, dtype_code(x.dtype), _ptr(x), L.s3(_bnh(x)), _ptr(y),
                           L.s3(_bnh(y)), _ptr(sin), _ptr(cos), 1 if inverse else 0))


class _Rotary(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, base):
        _require_gpu(x)
        B, N, H, D = x.shape
        if D % 2:
            raise ValueError("rotary needs an even head_dim")
        sin, cos = rotary_tables(N, D, x.device, base)
        y = torch.empty((B, N, H, D), dtype=x.dtype, device=x.device)
        _rotary_call(x, y, sin, cos, False)
        ctx.base = base
        return y

    @staticmethod
    @_sinking
    def backward(ctx, dy):
        dy = _grad_in(dy)
        B, N, H, D = dy.shape
        sin, cos = rotary_tables(N, D, dy.device, ctx.base)
        dx = torch.empty((B, N, H, D), dtype=dy.dtype, device=dy.device)
        _rotary_call(dy, dx, sin, cos, True)
        return dx, None


def rotary(x: torch.Tensor, base: float = 10000.0) -> torch.Tensor:
    """GPT-J interleaved rotary on [B, N, H, D] (position_embed.py:8-20; build-defined base
    10000, survey D6)."""
    return _Rotary.apply(x, float(base))


# ------------------------------------------------------------------ gradient sinks (flat DP buffer)
# The multi-rank step keeps every parameter gradient in one flat fp32 buffer (train.py).  Left to
# autograd, each parameter gradient would be computed into a fresh tensor and then ADDED into its
# zeroed flat view (one extra elementwise kernel per parameter, ~150 per DeiT-S step).  A sink is
# that flat view: the backward kernels of this module (weight / bias GEMMs, LayerNorm dgamma /
# dbeta, patch embedding) write the gradient straight into it and hand autograd None for that
# parameter.  A parameter may feed at most one such op per backward (each Dense / LayerNorm of the
# models is applied once per step); a second write raises instead of silently overwriting.
_GRAD_SINKS = {}      # id(param) -> (weakref(param), fp32 view shaped like the param)
_SINK_WRITTEN = set()
_SINK_WINDOW = False  # sinks are used only between begin_backward_sinks() and end_backward_sinks()
_CLAIM_LOG = []       # data pointers of the sinks claimed by the backward function now running
_SINK_LISTENER = None  # called with a sink's data pointer once the kernel writing it is enqueued


def set_grad_sinks(params, views=None) -> None:
    """Register ``views[i]`` (fp32, contiguous, shaped like ``params[i]``) as the gradient sink of
    ``params[i]``; ``params=None`` clears every sink."""
    import weakref
    if params is None:
        _GRAD_SINKS.clear()
        return
    for p, v in zip(params, views):
        if v.dtype != torch.float32 or not v.is_contiguous() or v.shape != p.shape:
            raise ValueError("set_grad_sinks: a sink must be an fp32 contiguous view shaped like its parameter")
        _GRAD_SINKS[id(p)] = (weakref.ref(p), v)


def begin_backward_sinks() -> None:
    """Open the sink window for one backward (the training step's): every sink may be written once
    again.  Outside the window the ops ignore the sinks and hand autograd ordinary gradients, so a
    backward outside a training step (gradient accumulation, a manual check) keeps autograd's
    accumulate semantics."""
    global _SINK_WINDOW
    _SINK_WRITTEN.clear()
    del _CLAIM_LOG[:]
    _SINK_WINDOW = True


def end_backward_sinks() -> None:
    """Close the sink window (the written set stays readable until the next begin)."""
    global _SINK_WINDOW
    _SINK_WINDOW = False


def set_sink_listener(fn) -> None:
    """``fn(data_ptr)`` is called for every sink once the kernel that writes it has been enqueued on
    the current stream (None: no listener)."""
    global _SINK_LISTENER
    _SINK_LISTENER = fn


def _sink(t: Optional[torch.Tensor]) -> Optional[torch.Tensor]:
    """The sink of parameter ``t`` (or of the parameter ``t`` is a full reshape view of), viewed as
    ``t``'s shape; None when it has none."""
    if t is None or not t.requires_grad or not _GRAD_SINKS or not _SINK_WINDOW:
        return None
    base = t if t._base is None else t._base
    e = _GRAD_SINKS.get(id(base))
    if e is None or e[0]() is not base or t.numel() != base.numel():
        return None
    g = base.grad   # a sink is live only while it is still the parameter's .grad (not replaced / reset)
    if g is None or g.data_ptr() != e[1].data_ptr():
        return None
    return e[1].view(t.shape)


def _claim(sink: Optional[torch.Tensor]) -> Optional[torch.Tensor]:
    """Mark a sink as written by this backward (at most once per step)."""
    if sink is not None:
        key = sink.data_ptr()
        if key in _SINK_WRITTEN:
            raise RuntimeError("gradient sink written twice in one backward: a parameter feeds two ops")
        _SINK_WRITTEN.add(key)
        _CLAIM_LOG.append(key)
    return sink


# ------------------------------------------------------------------------------ projections
# Side stream of the weight-gradient GEMMs (set_weight_grad_stream): inside the training step's
# sink window, a weight gradient that goes into a sink is off the backward's critical path, so its
# GEMM runs on this stream beside the input-gradient chain (LayerNorm / attention backward and the
# next dX GEMM) instead of between them; the step joins it before the optimizer.
_WG_STREAM = None


def set_weight_grad_stream(stream) -> None:
    """Run the sink-bound weight-gradient GEMMs of the following backwards on ``stream`` (None:
    on the current stream).  The caller joins it with :func:`join_weight_grad_stream`."""
    global _WG_STREAM
    _WG_STREAM = stream


def join_weight_grad_stream() -> None:
    """Make the current stream wait for every weight-gradient GEMM enqueued on the side stream."""
    if _WG_STREAM is not None:
        torch.cuda.current_stream(_WG_STREAM.device).wait_stream(_WG_STREAM)


def gemm_dw(x2: torch.Tensor, dy2: torch.Tensor, dw: torch.Tensor, db: Optional[torch.Tensor] = None,
            accumulate: bool = False, jblock: int = 0, offload: bool = False) -> None:
    """dw (+)= x2^T dy2 and db (+)= colsum(dy2) in fp32 through ``sae_gemm_dw`` (split over the
    token axis, fixed-order reduction).  x2 [M, I], dy2 [M, J] bf16 with unit column stride.
    ``jblock`` > 0: dw is [J / jblock, I, jblock] (contiguous column blocks).  ``offload``: dw / db
    are gradient sinks nobody reads before the step's join, so the GEMM may run on the
    weight-gradient side stream (when one is set and the sink window is open)."""
    lib = L.load()
    _require_gpu(x2, dy2, dw)
    M, I = x2.shape
    J = dy2.shape[1]
    side = _WG_STREAM if (offload and _SINK_WINDOW and _WG_STREAM is not None) else None
    if side is not None:
        side.wait_stream(torch.cuda.current_stream(x2.device))   # x2 / dy2 are written on the main stream
        x2.record_stream(side)    # ... and stay allocated until the side stream has read them
        dy2.record_stream(side)
    with torch.cuda.stream(side) if side is not None else contextlib.nullcontext():
        ws = torch.empty(lib.sae_gemm_dw_workspace_bytes(M, I, J), dtype=torch.uint8, device=x2.device)
        tok = _TIMER.begin("gemm_dw") if _TIMER is not None else None
        if jblock:
            L.check(lib.sae_gemm_dw_blocked(_stream(x2), M, I, J, int(jblock), _ptr(x2), x2.stride(0), _ptr(dy2),
                                            dy2.stride(0), _ptr(dw), _ptr(db), int(accumulate), _ptr(ws)))
        else:
            L.check(lib.sae_gemm_dw(_stream(x2), M, I, J, _ptr(x2), x2.stride(0), _ptr(dy2), dy2.stride(0),
                                    _ptr(dw), dw.stride(0), _ptr(db), int(accumulate), _ptr(ws)))
        if tok is not None:
            _TIMER.end(tok, (M, I, J))


def gemm_f32(a: torch.Tensor, b: torch.Tensor, bias: Optional[torch.Tensor] = None,
             out: Optional[torch.Tensor] = None, colsum: Optional[torch.Tensor] = None,
             accumulate: bool = False) -> torch.Tensor:
    """``a @ b (+ bias)`` in exact fp32 through ``sae_gemm_f32`` (f32-input MFMA).  ``a`` [M, K] and
    ``b`` [K, N] are fp32 views with a unit stride along one dimension each (a transposed view is
    read in place: ``x.t()`` for a weight gradient, ``w.t()`` for an input gradient).  ``colsum``
    (fp32 [N]) also receives the column sums of ``b`` (a bias gradient); ``accumulate`` adds into
    ``out`` / ``colsum``."""
    lib = L.load()
    _require_gpu(a, b)
    M, K = a.shape
    N = b.shape[1]
    if b.shape[0] != K:
        raise ValueError(f"gemm_f32: a {tuple(a.shape)} and b {tuple(b.shape)} disagree on K")
    if out is None:
        out = torch.empty((M, N), dtype=torch.float32, device=a.device)
    elif (out.dtype != torch.float32 or tuple(out.shape) != (M, N) or out.stride(1) != 1
          or out.device != a.device):
        raise ValueError(f"gemm_f32: out must be fp32 [{M}, {N}] with unit column stride on {a.device}")
    if colsum is not None and (colsum.dtype != torch.float32 or colsum.dim() != 1 or colsum.numel() < N
                               or colsum.stride(0) != 1 or colsum.device != a.device):
        # the kernel writes colsum[0 .. N) as fp32: anything else would be corrupted silently
        raise ValueError(f"gemm_f32: colsum must be a unit-stride fp32 vector of >= {N} elements on {a.device}")
    if bias is not None:
        bias = bias.float().contiguous()
    nbytes = lib.sae_gemm_f32_workspace_bytes(M, N, K)
    ws = torch.empty(nbytes, dtype=torch.uint8, device=a.device) if nbytes else None
    tok = _TIMER.begin("gemm_f32") if _TIMER is not None else None
    L.check(lib.sae_gemm_f32(_stream(a), M, N, K, _ptr(a), a.stride(0), a.stride(1), _ptr(b), b.stride(0),
                             b.stride(1), _ptr(bias), _ptr(out), out.stride(0), _ptr(colsum), int(accumulate),
                             _ptr(ws)))
    if tok is not None:
        _TIMER.end(tok, (M, K, N))
    return out


def _f32_operand_ok(t: torch.Tensor) -> bool:
    """A view sae_gemm_f32 reads in place: fp32, unit stride along one dim, 16-byte aligned, the
    other stride and the contiguous extent multiples of 4."""
    if not t.is_cuda or t.dtype != torch.float32 or t.dim() != 2 or t.data_ptr() % 16:
        return False
    r, c = t.shape
    if t.stride(1) == 1:
        return t.stride(0) % 4 == 0 and c % 4 == 0 and t.stride(0) >= c
    if t.stride(0) == 1:
        return t.stride(1) % 4 == 0 and r % 4 == 0 and t.stride(1) >= r
    return False


def _dw_ok(x2: torch.Tensor, dy2: torch.Tensor) -> bool:
    return (x2.is_cuda and x2.dtype == dy2.dtype == torch.bfloat16 and x2.shape[1] % 8 == 0 and dy2.shape[1] % 8 == 0
            and x2.stride(1) == 1 and dy2.stride(1) == 1 and x2.stride(0) % 8 == 0 and dy2.stride(0) % 8 == 0
            and x2.data_ptr() % 16 == 0 and dy2.data_ptr() % 16 == 0)


# ----------------------------------------------------- per-forward cache of the bf16 weight casts
# ``cast_weights`` casts every Dense kernel of an encoder in ONE launch (sae_weight_cast_multi) at
# the start of its forward; the projections look their casts up while that forward runs and the
# encoder clears the cache when it returns (nothing outlives the forward: the next optimizer step
# changes the fp32 weights).  Keys are the fp32 weights' data pointers, checked with versions.
_WCACHE = {}


def _wkey(ws):
    return tuple(w.data_ptr() for w in ws)


def cast_weights(groups) -> None:
    """``groups``: lists of fp32 2-D weights [K, n_j] (same K) stacked along columns; each group
    gets a bf16 [K, sum n_j] and its transpose, cached under the group's key."""
    lib = L.load()
    items = []
    dev = None
    for ws in groups:
        K = ws[0].shape[0]
        if any(w.dim() != 2 or w.shape[0] != K or w.dtype != torch.float32 or not w.is_contiguous() for w in ws):
            continue
        if _wkey(ws) in _PERSIST:   # the optimizer keeps this group's copies
            continue
        dev = ws[0].device
        N = sum(w.shape[1] for w in ws)
        w16 = torch.empty((K, N), dtype=torch.bfloat16, device=dev)
        wt16 = torch.empty((N, K), dtype=torch.bfloat16, device=dev)
        items += _cast_items(ws, w16, wt16)
        _WCACHE[_wkey(ws)] = (tuple(w._version for w in ws), w16, wt16)
    if items:
        arr = (L.WeightCastItem * len(items))(*items)
        L.check(lib.sae_weight_cast_multi(_stream(groups[0][0]), len(items), arr))


def clear_weight_cache() -> None:
    _WCACHE.clear()


# ---------------------------------------------------------- persistent bf16 weight copies
# Groups whose bf16 copies the optimizer writes (FusedAdamW with cast_groups: the update and the
# cast in one pass, sae_adamw_step_cast) stay registered across steps: the forward neither casts
# nor allocates for them.  An in-place change of a weight OUTSIDE the optimizer (load_state_dict,
# a copy_) bumps its version counter; the next lookup then re-casts into the same buffers.  The
# optimizer writes through raw pointers (no version bump) and calls ``persistent_casts_fresh``
# whenever it rewrites the copies itself.
_PERSIST = {}


def register_persistent_casts(groups, w16s, wt16s, owner=None) -> None:
    """Serve ``groups``' bf16 copies from ``w16s`` / ``wt16s`` (kept current by ``owner``, the
    optimizer that writes them).  A later registration of the same weights takes over."""
    for ws, w16, wt16 in zip(groups, w16s, wt16s):
        _PERSIST[_wkey(ws)] = [tuple(w._version for w in ws), w16, wt16, list(ws), owner]


def unregister_persistent_casts(groups, owner=None) -> None:
    """Stop serving ``groups``' copies -- only the entries ``owner`` registered (None: any)."""
    for ws in groups:
        e = _PERSIST.get(_wkey(ws))
        if e is not None and (owner is None or e[4] is owner):
            del _PERSIST[_wkey(ws)]


def release_persistent_casts(params) -> None:
    """Drop every registered group holding one of ``params`` (an optimizer that now updates them
    without writing those copies takes them over: the copies would go stale)."""
    ids = {p.data_ptr() for p in params}
    for key in [k for k, e in _PERSIST.items() if any(w.data_ptr() in ids for w in e[3])]:
        del _PERSIST[key]


def persistent_casts_stale(groups) -> bool:
    """True when a weight of a registered group was changed in place since its copies were
    written (load_state_dict, copy_: the version counter moved)."""
    for ws in groups:
        e = _PERSIST.get(_wkey(ws))
        if e is not None and e[0] != tuple(w._version for w in e[3]):
            return True
    return False


def persistent_casts_fresh(groups) -> None:
    """The copies of ``groups`` match their fp32 weights as of now."""
    for ws in groups:
        e = _PERSIST.get(_wkey(ws))
        if e is not None:
            e[0] = tuple(w._version for w in ws)


def _cast_items(ws, w16, wt16):
    K, N = ws[0].shape[0], w16.shape[1]
    items, col = [], 0
    for w in ws:
        items.append(L.WeightCastItem(w.data_ptr(), w16.data_ptr(), wt16.data_ptr(), K, w.shape[1], N, K, col))
        col += w.shape[1]
    return items


def recast_persistent(groups) -> None:
    """Re-cast the registered copies of ``groups`` from their fp32 weights (one launch)."""
    items = []
    for ws in groups:
        e = _PERSIST.get(_wkey(ws))
        if e is not None:
            items += _cast_items(e[3], e[1], e[2])
            e[0] = tuple(w._version for w in e[3])
    if items:
        arr = (L.WeightCastItem * len(items))(*items)
        L.check(L.load().sae_weight_cast_multi(_stream(groups[0][0]), len(items), arr))


def _cast_lookup(ws):
    key = _wkey(ws)
    e = _PERSIST.get(key)
    if e is not None:
        if e[0] != tuple(w._version for w in ws):
            recast_persistent([ws])
        return e[1], e[2]
    e = _WCACHE.get(key)
    if e is not None and e[0] == tuple(w._version for w in ws):
        return e[1], e[2]
    return None


def _cast(ws, dt):
    """bf16 [K, N] and [N, K] of the column-stacked fp32 weights ``ws`` (cached, or one launch)."""
    hit = _cast_lookup(ws) if dt == torch.bfloat16 else None
    if hit is not None:
        return hit
    w = ws[0] if len(ws) == 1 else torch.cat(ws, dim=1)
    if dt == torch.bfloat16 and w.dtype == torch.float32 and w.is_cuda:
        return weight_cast(w)
    return w.to(dt), None


class _Dense(torch.autograd.Function):
    """y = x @ W (+ b): Flax ``Dense`` / ``DenseGeneral`` semantics (input and fp32 kernel cast to
    the compute dtype).  ``W`` may be given as column blocks (the queries / keys / values kernels of
    one stacked projection): their gradients come back as the matching column slices.  Backward:
    dX = dY W^T, dW / db straight into fp32 by the split-token MFMA kernel (``sae_gemm_dw``) when
    the compute dtype is bf16."""

    @staticmethod
    def forward(ctx, x, b, dt, *ws):
        I = ws[0].shape[0]
        J = sum(w.shape[1] for w in ws)
        x2 = x.to(dt).reshape(-1, I)
        wd, wt = _cast(ws, dt)
        if dt == torch.float32 and _f32_operand_ok(x2) and _f32_operand_ok(wd):
            y = gemm_f32(x2, wd, b)                       # exact fp32 on the f32 MFMA, bias in the epilogue
        elif wt is not None and (use_gemm_nt(I, J) or x2.shape[0] <= SMALL_M) and _nt_ok(x2, J):
            y = gemm_nt(x2, wt, b)                        # bias in the epilogue
        else:
            # bias rides in the library GEMM's epilogue (addmm) instead of a separate pass
            y = torch.addmm(b.to(dt), x2, wd) if b is not None else x2 @ wd
        # bf16 W^T [J, I] is kept only for the one input gradient that reads it (below: a small-M
        # call whose J is not a multiple of 8), through save_for_backward (version-checked)
        keep_wt = wt is not None and J % 8 != 0 and x2.shape[0] <= SMALL_M
        ctx.save_for_backward(x2, wd, wt if keep_wt else None)
        ctx.has_b, ctx.xshape, ctx.xdtype = b is not None, x.shape, x.dtype
        ctx.wmeta = [(w.shape[1], w.dtype) for w in ws]
        ctx.sinks_w, ctx.sink_b = [_sink(w) for w in ws], _sink(b)
        return y.view(*x.shape[:-1], J)

    @staticmethod
    @_sinking
    def backward(ctx, dy):
        x2, wd, wt = ctx.saved_tensors
        I, J = wd.shape
        dy2 = dy.reshape(-1, J)
        if dy2.stride(1) != 1 or dy2.stride(0) % 8:
            dy2 = dy2.contiguous()
        if wd.dtype == torch.float32 and _f32_operand_ok(dy2) and _f32_operand_ok(x2) and _f32_operand_ok(wd):
            return _Dense._backward_f32(ctx, x2, wd, dy2)
        if use_gemm_nt(J, I) and _nt_ok(dy2, I) and wd.dtype == torch.bfloat16:
            dx = gemm_nt(dy2, wd).view(ctx.xshape).to(ctx.xdtype)
        else:
            dyt = dy2.t().contiguous() if (wd.dtype == torch.bfloat16 and wt is not None) else None
            if dyt is not None and _dw_ok(dyt, wt):
                # K = J not a multiple of 8 (a classifier head with e.g. 10 classes) -- the reduction
                # runs over the ROWS of dY^T [J, M] and W^T [J, I], i.e. on the weight-gradient
                # kernel: dx[m][i] = sum_j dY^T[j][m] W^T[j][i], fp32 then the activation dtype
                dxf = torch.empty((dy2.shape[0], I), dtype=torch.float32, device=dy2.device)
                gemm_dw(dyt, wt, dxf)
                dx = dxf.view(ctx.xshape).to(ctx.xdtype)
            else:
                dx = (dy2 @ wd.t()).view(ctx.xshape).to(ctx.xdtype)
        widths = [n for n, _ in ctx.wmeta]
        blocked = len(widths) > 1 and len(set(widths)) == 1 and widths[0] % 4 == 0
        sw, sb = ctx.sinks_w, ctx.sink_b
        if _dw_ok(x2, dy2) and (blocked or len(widths) == 1):
            # flat-buffer sinks (multi-rank step): dW / db written in place, autograd gets None
            db = _claim(sb) if sb is not None else (
                torch.empty((J,), dtype=torch.float32, device=x2.device) if ctx.has_b else None)
            rdb = None if sb is not None else db
            if blocked:   # one contiguous [I, n] gradient per column block: no slice copies
                n = widths[0]
                s0 = sw[0]
                if s0 is not None and all(t is not None and t.data_ptr() == s0.data_ptr() + k * I * n * 4
                                          for k, t in enumerate(sw)):   # adjacent sinks: one [nb, I, n] block
                    for t in sw:
                        _claim(t)
                    gemm_dw(x2, dy2, s0.as_strided((len(widths), I, n), (I * n, n, 1)), db, jblock=n,
                            offload=sb is not None or not ctx.has_b)
                    return (dx, rdb, None, *[None] * len(widths))
                dwb = torch.empty((len(widths), I, n), dtype=torch.float32, device=x2.device)
                gemm_dw(x2, dy2, dwb, db, jblock=n)
                return (dx, rdb, None, *[dwb[k].to(wdt) for k, (_, wdt) in enumerate(ctx.wmeta)])
            if sw[0] is not None:
                gemm_dw(x2, dy2, _claim(sw[0]), db, offload=sb is not None or not ctx.has_b)
                return dx, rdb, None, None
            dw = torch.empty((I, J), dtype=torch.float32, device=x2.device)
            gemm_dw(x2, dy2, dw, db)
            db = rdb
        elif _dw_ok(x2, dy2):
            dw = torch.empty((I, J), dtype=torch.float32, device=x2.device)
            db = torch.empty((J,), dtype=torch.float32, device=x2.device) if ctx.has_b else None
            gemm_dw(x2, dy2, dw, db)
        else:
            dw = (x2.t() @ dy2).float()
            db = dy2.sum(0, dtype=torch.float32) if ctx.has_b else None
        dws, col = [], 0
        for n, wdt in ctx.wmeta:
            dws.append(dw[:, col:col + n].to(wdt))
            col += n
        return (dx, db, None, *dws)

    @staticmethod
    def _backward_f32(ctx, x2, wd, dy2):
        """fp32 compute dtype: dX = dY W^T, then per column block dW_k = X^T dY[:, block] with that
        block's db slice as the ones-row column sum, all on sae_gemm_f32; sinks written in place."""
        I, J = wd.shape
        dx = gemm_f32(dy2, wd.t()).view(ctx.xshape).to(ctx.xdtype)
        sb = ctx.sink_b
        db = _claim(sb) if sb is not None else (
            torch.empty((J,), dtype=torch.float32, device=x2.device) if ctx.has_b else None)
        dws, col = [], 0
        for (n, wdt), sw in zip(ctx.wmeta, ctx.sinks_w):
            dst = _claim(sw) if sw is not None else torch.empty((I, n), dtype=torch.float32, device=x2.device)
            dyb = dy2[:, col:col + n]
            if not _f32_operand_ok(dyb):
                dyb = dyb.contiguous()
            gemm_f32(x2.t(), dyb, out=dst, colsum=db[col:col + n] if db is not None else None)
            dws.append(None if sw is not None else dst.to(wdt))
            col += n
        return (dx, None if sb is not None else db, None, *dws)


def dense(x: torch.Tensor, w, b: Optional[torch.Tensor], dtype: torch.dtype) -> torch.Tensor:
    """Projection of the hot path: ``x @ w (+ b)`` in ``dtype`` with fp32 parameter gradients.
    ``w`` is a 2-D kernel [in, out] or a list of them stacked along the output axis."""
    ws = list(w) if isinstance(w, (list, tuple)) else [w]
    return _Dense.apply(x, b, dtype, *ws)


# ------------------------------------------------------------------------- patch embedding
def _patch_desc(images: torch.Tensor, patch: Tuple[int, int], embed: int, layout: str) -> L.SaePatchDesc:
    if layout == "NHWC":
        B, H, W, C = images.shape
        code = L.SAE_LAYOUT_NHWC
    elif layout == "HWCN":
        H, W, C, B = images.shape
        code = L.SAE_LAYOUT_HWCN
    else:
        raise ValueError(f"patch_embed: layout must be 'NHWC' or 'HWCN', got {layout!r}")
    return L.SaePatchDesc(B, H, W, C, int(patch[0]), int(patch[1]), int(embed), code, dtype_code(images.dtype))


# HWCN images (the train-step feed): write the patch matrix once (sae_patch_gather) and run the
# embedding and its weight gradient on the LDS-DMA GEMMs -- DeiT-S 59 + 56 us of fused HWCN
# gathers against the gather + gemm8 + gemm_dw8 (profiles/r05af_patch_gather_ab.txt).  False: the
# fused loaders (no patch copy; A/B runs).
PATCH_GATHER = os.environ.get("SAE_PATCH_GATHER", "1") != "0"


class _PatchEmbed(torch.autograd.Function):
    """patch_embed.py:15-26 in bf16: the patch gather fused into the GEMM's operand staging
    (``sae_patch_embed_fwd``), weight / bias gradients by the same gather (``sae_patch_embed_bwd``);
    for HWCN images the patch matrix is written once (``sae_patch_gather``) and both products run on
    ``sae_gemm_nt`` / ``sae_gemm_dw``.  The images take no gradient (they are the batch,
    train.py:80-82)."""

    @staticmethod
    def forward(ctx, images, w, b, patch, layout):
        lib = L.load()
        E = w.shape[1]
        desc = _patch_desc(images, patch, E, layout)
        _, wt = _cast([w], torch.bfloat16)
        Lp = (desc.height // desc.patch_h) * (desc.width // desc.patch_w)
        K = desc.patch_h * desc.patch_w * desc.channels
        bias = b.float().contiguous() if b is not None else None
        tok = _TIMER.begin("patch_embed") if _TIMER is not None else None
        gathered = layout == "HWCN" and PATCH_GATHER and E % 8 == 0
        if gathered:
            pm = torch.empty((desc.batch * Lp, K), dtype=torch.bfloat16, device=images.device)
            L.check(lib.sae_patch_gather(_stream(images), ctypes.byref(desc), _ptr(images), _ptr(pm)))
            out = gemm_nt(pm, wt, bias).view(desc.batch, Lp, E)
            ctx.save_for_backward(pm)
        else:
            out = torch.empty((desc.batch, Lp, E), dtype=torch.bfloat16, device=images.device)
            L.check(lib.sae_patch_embed_fwd(_stream(images), ctypes.byref(desc), _ptr(images), _ptr(wt),
                                            _ptr(bias), _ptr(out)))
            ctx.save_for_backward(images)
        if tok is not None:
            _TIMER.end(tok, (desc.batch * Lp, w.shape[0], E))
        ctx.desc, ctx.wshape, ctx.wdtype, ctx.has_b = desc, tuple(w.shape), w.dtype, b is not None
        ctx.gathered = gathered
        ctx.sinks = (_sink(w), _sink(b))
        return out

    @staticmethod
    @_sinking
    def backward(ctx, dout):
        lib = L.load()
        (saved,) = ctx.saved_tensors
        desc = ctx.desc
        dout = dout.to(torch.bfloat16).contiguous()
        sw, sb = ctx.sinks   # flat-buffer sinks (multi-rank step): written in place
        dw = _claim(sw) if sw is not None else torch.empty(ctx.wshape, dtype=torch.float32, device=dout.device)
        db = _claim(sb) if sb is not None else (
            torch.empty((ctx.wshape[1],), dtype=torch.float32, device=dout.device) if ctx.has_b else None)
        if ctx.gathered:   # dW = P^T dY, db = colsum(dY) on the weight-gradient kernel
            gemm_dw(saved, dout.view(-1, ctx.wshape[1]), dw, db)
        else:
            ws = torch.empty(lib.sae_patch_embed_bwd_workspace_bytes(ctypes.byref(desc)), dtype=torch.uint8,
                             device=dout.device)
            L.check(lib.sae_patch_embed_bwd(_stream(dout), ctypes.byref(desc), _ptr(saved), _ptr(dout), _ptr(dw),
                                            _ptr(db), 0, _ptr(ws)))
        return None, None if sw is not None else dw.to(ctx.wdtype), _unsunk(db, sb), None, None


def patch_embed(images: torch.Tensor, w: torch.Tensor, b: Optional[torch.Tensor], patch: Tuple[int, int],
                layout: str = "NHWC") -> torch.Tensor:
    """``PatchEmbedBlock`` (patch_embed.py:15-26) in bf16: tokens [B, L, E] of ``images`` (bf16 or
    fp32; ``layout`` "NHWC" [B, H, W, C] or the train-step feed "HWCN" [H, W, C, B], train.py:80)
    times the fp32 Dense kernel ``w`` [ph * pw * C, E] (+ ``b``).  The images take no gradient."""
    _require_gpu(images, w)
    if images.requires_grad:
        raise NotImplementedError("patch_embed: the images take no gradient on this path (train.py:80-82)")
    if images.dtype not in (torch.bfloat16, torch.float32):
        images = images.float()
    if not images.is_contiguous() or images.data_ptr() % 16:
        images = images.contiguous()
    if w.dtype != torch.float32 or w.dim() != 2:
        raise ValueError("patch_embed: w must be the fp32 Dense kernel [ph * pw * C, E]")
    return _PatchEmbed.apply(images, w, b, tuple(int(p) for p in patch), layout)


def patch_embed_ok(images: torch.Tensor, w: torch.Tensor, patch: Tuple[int, int], layout: str = "NHWC") -> bool:
    """Shapes the fused kernel takes (sae_patch_embed_fwd's requirements, include/sae_attn.h)."""
    if images.dim() != 4 or not images.is_cuda:
        return False
    H, W, C, B = images.shape if layout == "HWCN" else (images.shape[1], images.shape[2], images.shape[3],
                                                        images.shape[0])
    ph, pw = patch
    K = ph * pw * C
    return (H % ph == 0 and W % pw == 0 and K % 64 == 0 and (pw * C) % 8 == 0 and w.shape[1] % 8 == 0
            and w.shape[0] == K and (layout != "HWCN" or B % 8 == 0))


# ------------------------------------------------- forward / input-gradient GEMMs (sae_gemm_nt)
EPI_NONE, EPI_GELU, EPI_DGELU = 0, 1, 2
# the FF block's pair (include/sae_attn.h): the forward saves g = gelu'(h) instead of h, the
# input-gradient epilogue multiplies by it
EPI_GELU_GRAD, EPI_MUL_AUX = 3, 4
FF_GELU_GRAD = os.environ.get("SAE_FF_GELU_GRAD", "1") != "0"   # (False: save h, GELU' epilogue; A/B)


# Every bf16 forward / input-gradient projection whose widths are multiples of 8 runs on
# sae_gemm_nt (round 5): the C ABI picks the kernel by tile fill and reduction depth (capi.hip,
# g8x_route / g8_route: the persistent gemm8, the ping-pong gemm8x, or the 128-row kernel, which
# also takes K not a multiple of 64).  That covers every width in create_model.py:6-215 (ViT-B/L,
# DeiT, CaiT 192-768, CeiT, CvT 64/192/368/1024, TNT 24/40/384/640); tests/test_routing_cpu.py
# pins it.  GEMM_LIB = True sends them to the library GEMM instead (A/B runs only).
GEMM_LIB = False
SMALL_M = 4096   # Dense calls on at most this many rows (classifier heads, CLS-token projections)


def use_gemm_nt(K: int, N: int) -> bool:
    """Route a forward / input-gradient GEMM (reduction depth K, N output features) to sae_gemm_nt."""
    return not GEMM_LIB and K % 8 == 0 and N % 8 == 0


def _nt_ok(a2: torch.Tensor, N: int) -> bool:
    K = a2.shape[1]
    return (a2.is_cuda and a2.dtype == torch.bfloat16 and K % 8 == 0 and N % 8 == 0 and a2.stride(1) == 1
            and a2.stride(0) % 8 == 0 and a2.data_ptr() % 16 == 0)


def weight_cast(w: torch.Tensor, plain: bool = True, transposed: bool = True):
    """fp32 Dense kernel [K, N] -> (bf16 [K, N] or None, bf16 [N, K] or None) in one HIP pass."""
    lib = L.load()
    _require_gpu(w)
    K, N = w.shape
    w = w.contiguous()
    w16 = torch.empty((K, N), dtype=torch.bfloat16, device=w.device) if plain else None
    wt16 = torch.empty((N, K), dtype=torch.bfloat16, device=w.device) if transposed else None
    L.check(lib.sae_weight_cast(_stream(w), K, N, _ptr(w), _ptr(w16), _ptr(wt16)))
    return w16, wt16


def gemm_nt(a2: torch.Tensor, bt: torch.Tensor, bias: Optional[torch.Tensor] = None, epilogue: int = EPI_NONE,
            aux: Optional[torch.Tensor] = None, out: Optional[torch.Tensor] = None):
    """``epi(a2 @ bt^T (+ bias))`` through ``sae_gemm_nt``: a2 [M, K], bt [N, K] bf16.  Returns c,
    or (c, h) for the GELU epilogue (c = gelu(h), h = the bf16 pre-activation), or (c, g) for
    EPI_GELU_GRAD (g = bf16(gelu'(h)), the aux of a later EPI_MUL_AUX call)."""
    lib = L.load()
    _require_gpu(a2, bt)
    M, K = a2.shape
    N = bt.shape[0]
    if bt.shape[1] != K:
        raise ValueError(f"gemm_nt: a2 {tuple(a2.shape)} and bt {tuple(bt.shape)} disagree on K")
    if bt.stride(1) != 1:
        bt = bt.contiguous()
    if out is not None:
        if out.dtype != torch.bfloat16 or out.dim() != 2 or tuple(out.shape) != (M, N) or out.stride(1) != 1:
            raise ValueError(f"gemm_nt: out must be bf16 [{M}, {N}] with unit column stride")
        c = out
    else:
        c = torch.empty((M, N), dtype=torch.bfloat16, device=a2.device)
    # the kernel writes c2 with c's row stride (ldc): give it the same layout
    two = epilogue in (EPI_GELU, EPI_GELU_GRAD)
    c2 = torch.empty_strided((M, N), (c.stride(0), 1), dtype=torch.bfloat16, device=a2.device) if two else None
    if epilogue in (EPI_DGELU, EPI_MUL_AUX):
        if aux is None or aux.dtype != torch.bfloat16 or tuple(aux.shape) != (M, N):
            raise ValueError(f"gemm_nt: the GELU-derivative epilogue needs a bf16 aux [{M}, {N}]")
    if aux is not None and aux.stride(1) != 1:
        aux = aux.contiguous()
    if bias is not None:
        bias = bias.float().contiguous()
    L.check(lib.sae_gemm_nt(_stream(a2), M, N, K, _ptr(a2), a2.stride(0), _ptr(bt), bt.stride(0), _ptr(bias),
                            _ptr(c), c.stride(0), int(epilogue), _ptr(aux), aux.stride(0) if aux is not None else 0,
                            _ptr(c2)))
    return (c, c2) if two else c


class _FFBlock(torch.autograd.Function):
    """ff.py:8-34 in bf16: ``Dense_1(gelu(Dense_0(x)))`` with the GELU fused into Dense_0's GEMM
    epilogue (saving gelu'(h) of the pre-activation h, EPI_GELU_GRAD) and the product with it fused
    into the epilogue of Dense_1's input-gradient GEMM (EPI_MUL_AUX); weight / bias gradients
    through ``sae_gemm_dw``."""

    @staticmethod
    def forward(ctx, x, w0, b0, w1, b1):
        I, Hd = w0.shape
        x2 = x.to(torch.bfloat16).reshape(-1, I)
        if x2.stride(1) != 1 or x2.stride(0) % 8 or x2.data_ptr() % 16:
            x2 = x2.contiguous()
        w0p, w0t = _cast([w0], torch.bfloat16)
        w1p, w1t = _cast([w1], torch.bfloat16)
        gg = FF_GELU_GRAD
        a, h = gemm_nt(x2, w0t, b0, EPI_GELU_GRAD if gg else EPI_GELU)   # h: gelu'(pre-activation)
        y = gemm_nt(a, w1t, b1)                                   # Dense_1 forward
        ctx.save_for_backward(x2, h, a, w0p, w1p)
        ctx.gg = gg
        ctx.xshape, ctx.xdtype, ctx.has_b = x.shape, x.dtype, (b0 is not None, b1 is not None)
        ctx.sinks = [_sink(t) for t in (w0, b0, w1, b1)]
        return y.view(*x.shape[:-1], w1.shape[1])

    @staticmethod
    @_sinking
    def backward(ctx, dy):
        x2, h, a, w0p, w1p = ctx.saved_tensors
        I, Hd = w0p.shape
        O = w1p.shape[1]
        dy2 = dy.to(torch.bfloat16).reshape(-1, O)
        if dy2.stride(1) != 1 or dy2.stride(0) % 8 or dy2.data_ptr() % 16:
            dy2 = dy2.contiguous()
        dh = gemm_nt(dy2, w1p, None, EPI_MUL_AUX if ctx.gg else EPI_DGELU, aux=h)   # dA W1^T, times gelu'(h)
        sw0, sb0, sw1, sb1 = ctx.sinks   # flat-buffer sinks (multi-rank step): written in place
        dev = dy2.device
        dw1 = _claim(sw1) if sw1 is not None else torch.empty((Hd, O), dtype=torch.float32, device=dev)
        db1 = _claim(sb1) if sb1 is not None else (
            torch.empty((O,), dtype=torch.float32, device=dev) if ctx.has_b[1] else None)
        gemm_dw(a, dy2, dw1, db1, offload=sw1 is not None and (sb1 is not None or not ctx.has_b[1]))
        dx = gemm_nt(dh, w0p)                                     # dH W0^T
        dw0 = _claim(sw0) if sw0 is not None else torch.empty((I, Hd), dtype=torch.float32, device=dev)
        db0 = _claim(sb0) if sb0 is not None else (
            torch.empty((Hd,), dtype=torch.float32, device=dev) if ctx.has_b[0] else None)
        gemm_dw(x2, dh, dw0, db0, offload=sw0 is not None and (sb0 is not None or not ctx.has_b[0]))
        ret = [None if sk is not None else g for sk, g in zip(ctx.sinks, (dw0, db0, dw1, db1))]
        return (dx.view(ctx.xshape).to(ctx.xdtype), *ret)


FF_FUSED = True   # tools/ab_step.py flips this to A/B against the library GEMM + torch GELU path


def ff_block_ok(x: torch.Tensor, w0: torch.Tensor, w1: torch.Tensor) -> bool:
    if not FF_FUSED:
        return False
    I, Hd = w0.shape
    O = w1.shape[1]
    return (x.is_cuda and w0.dtype == w1.dtype == torch.float32 and I % 8 == 0 and Hd % 8 == 0 and O % 8 == 0
            and w1.shape[0] == Hd)


def ff_block(x: torch.Tensor, w0: torch.Tensor, b0: Optional[torch.Tensor], w1: torch.Tensor,
             b1: Optional[torch.Tensor]) -> torch.Tensor:
    """Flax FFBlock (ff.py:8-34, dropout 0) in bf16 with fp32 params: x [.., I] -> [.., O]."""
    _require_gpu(x, w0, w1)
    return _FFBlock.apply(x, w0, b0, w1, b1)


# ------------------------------------------------------------------ residual add + LayerNorm
LN_EPS = 1e-6   # Flax nn.LayerNorm default (models/vit.py:19,26,57)


def layer_norm_ok(x: torch.Tensor) -> bool:
    """The fused kernels cover the encoder's fp32 residual stream with C % 4 == 0, C <= 1024."""
    C = x.shape[-1]
    return x.is_cuda and x.dtype == torch.float32 and C % 4 == 0 and C <= 1024 and x.is_contiguous()


def _f32c(t: torch.Tensor, what: str) -> torch.Tensor:
    """fp32 contiguous view/copy of a LayerNorm operand (the kernels read raw fp32)."""
    if t.dtype != torch.float32:
        t = t.float()
    return t if t.is_contiguous() else t.contiguous()


def _bf16c(t: torch.Tensor) -> torch.Tensor:
    """bf16 contiguous copy of a LayerNorm operand (the kernels read raw bf16)."""
    if t.dtype != torch.bfloat16:
        t = t.to(torch.bfloat16)
    return t if t.is_contiguous() else t.contiguous()


def _ln_fwd(x, delta, gamma, beta, eps):
    lib = L.load()
    x, gamma, beta = _f32c(x, "x"), _f32c(gamma, "gamma"), _f32c(beta, "beta")
    if delta is not None:
        delta = _bf16c(delta)
    C = x.shape[-1]
    M = x.numel() // C
    y = torch.empty(x.shape, dtype=torch.bfloat16, device=x.device)
    mean = torch.empty(M, dtype=torch.float32, device=x.device)
    rstd = torch.empty(M, dtype=torch.float32, device=x.device)
    xout = torch.empty_like(x) if delta is not None else None
    L.check(lib.sae_layernorm_fwd(_stream(x), M, C, _ptr(x), _ptr(delta), _ptr(xout), _ptr(gamma), _ptr(beta),
                                  _ptr(y), _ptr(mean), _ptr(rstd), float(eps)))
    return xout, y, mean, rstd


def _ln_bwd(xs, mean, rstd, gamma, dy, dxin, want_ddelta, sinks=(None, None)):
    lib = L.load()
    C = xs.shape[-1]
    M = xs.numel() // C
    xs, gamma = _f32c(xs, "x"), _f32c(gamma, "gamma")
    dy = _bf16c(dy)
    dx = torch.empty_like(xs)
    ddelta = torch.empty(xs.shape, dtype=torch.bfloat16, device=xs.device) if want_ddelta else None
    dg = _claim(sinks[0]) if sinks[0] is not None else torch.empty(C, dtype=torch.float32, device=xs.device)
    db = _claim(sinks[1]) if sinks[1] is not None else torch.empty(C, dtype=torch.float32, device=xs.device)
    ws = torch.empty(lib.sae_layernorm_bwd_workspace_bytes(M, C), dtype=torch.uint8, device=xs.device)
    if dxin is not None:
        dxin = _f32c(dxin, "dxin")
    L.check(lib.sae_layernorm_bwd(_stream(xs), M, C, _ptr(xs), _ptr(mean), _ptr(rstd), _ptr(gamma), _ptr(dy),
                                  _ptr(dxin), _ptr(dx), _ptr(ddelta), _ptr(dg), _ptr(db), _ptr(ws)))
    return dx, ddelta, dg, db


def _unsunk(g, sink):
    """The gradient autograd should see: None when it went into a sink."""
    return None if sink is not None else g


class _LayerNorm(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, gamma, beta, eps):
        _, y, mean, rstd = _ln_fwd(x, None, gamma, beta, eps)
        ctx.save_for_backward(x, mean, rstd, gamma)
        ctx.sinks = (_sink(gamma), _sink(beta))
        return y

    @staticmethod
    @_sinking
    def backward(ctx, dy):
        x, mean, rstd, gamma = ctx.saved_tensors
        dx, _, dg, db = _ln_bwd(x, mean, rstd, gamma, dy, None, False, ctx.sinks)
        return dx, _unsunk(dg, ctx.sinks[0]), _unsunk(db, ctx.sinks[1]), None


class _AddLayerNorm(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, delta, gamma, beta, eps):
        xout, y, mean, rstd = _ln_fwd(x, delta, gamma, beta, eps)
        ctx.save_for_backward(xout, mean, rstd, gamma)
        ctx.delta_dtype = delta.dtype
        ctx.sinks = (_sink(gamma), _sink(beta))
        return xout, y

    @staticmethod
    @_sinking
    def backward(ctx, dxout, dy):
        xout, mean, rstd, gamma = ctx.saved_tensors
        if dy is None:
            dy = torch.zeros(xout.shape, dtype=torch.bfloat16, device=xout.device)
        dx, ddelta, dg, db = _ln_bwd(xout, mean, rstd, gamma, dy, dxout, True, ctx.sinks)
        return dx, ddelta.to(ctx.delta_dtype), _unsunk(dg, ctx.sinks[0]), _unsunk(db, ctx.sinks[1]), None


class _AddLayerNormScaled(torch.autograd.Function):
    """x + delta * layerscale[c] * rowscale[sample] and its LayerNorm (CaiT blocks)."""

    @staticmethod
    def forward(ctx, x, delta, gamma, beta, ls, rowscale, rpb, eps):
        lib = L.load()
        C = x.shape[-1]
        M = x.numel() // C
        x, gamma, beta = _f32c(x, "x"), _f32c(gamma, "gamma"), _f32c(beta, "beta")
        delta_dtype = delta.dtype
        delta = _bf16c(delta)
        # the reference casts the LayerScale parameter to the compute dtype (layerscale.py:22): the
        # kernels round the fp32 parameter to bf16 as they load it (no cast launches here)
        lsf = _f32c(ls.detach(), "layerscale")
        y = torch.empty(x.shape, dtype=torch.bfloat16, device=x.device)
        mean = torch.empty(M, dtype=torch.float32, device=x.device)
        rstd = torch.empty(M, dtype=torch.float32, device=x.device)
        xout = torch.empty_like(x)
        L.check(lib.sae_layernorm_fwd_scaled(_stream(x), M, C, _ptr(x), _ptr(delta), _ptr(xout), _ptr(gamma),
                                             _ptr(beta), _ptr(y), _ptr(mean), _ptr(rstd), float(eps), _ptr(lsf),
                                             _ptr(rowscale), int(rpb)))
        ctx.save_for_backward(xout, mean, rstd, gamma, delta, lsf, rowscale)
        ctx.rpb, ctx.delta_dtype, ctx.ls_dtype = int(rpb), delta_dtype, ls.dtype
        ctx.sinks = (_sink(gamma), _sink(beta), _sink(ls) if ls.dtype == torch.float32 else None)
        return xout, y

    @staticmethod
    @_sinking
    def backward(ctx, dxout, dy):
        xout, mean, rstd, gamma, delta, lsf, rowscale = ctx.saved_tensors
        lib = L.load()
        C = xout.shape[-1]
        M = xout.numel() // C
        if dy is None:
            dy = torch.zeros(xout.shape, dtype=torch.bfloat16, device=xout.device)
        dy = _bf16c(dy)
        gamma = _f32c(gamma, "gamma")
        dxin = _f32c(dxout, "dxin") if dxout is not None else None
        dx = torch.empty_like(xout)
        ddelta = torch.empty(xout.shape, dtype=torch.bfloat16, device=xout.device)
        sg, sbt, sls = ctx.sinks
        dg = _claim(sg) if sg is not None else torch.empty(C, dtype=torch.float32, device=xout.device)
        db = _claim(sbt) if sbt is not None else torch.empty(C, dtype=torch.float32, device=xout.device)
        dls = _claim(sls) if sls is not None else torch.empty(C, dtype=torch.float32, device=xout.device)
        ws = torch.empty(lib.sae_layernorm_bwd_workspace_bytes(M, C), dtype=torch.uint8, device=xout.device)
        L.check(lib.sae_layernorm_bwd_scaled(_stream(xout), M, C, _ptr(xout), _ptr(mean), _ptr(rstd), _ptr(gamma),
                                             _ptr(dy), _ptr(dxin), _ptr(dx), _ptr(ddelta), _ptr(dg), _ptr(db),
                                             _ptr(ws), _ptr(delta), _ptr(lsf), _ptr(rowscale), ctx.rpb, _ptr(dls)))
        return (dx, ddelta.to(ctx.delta_dtype), _unsunk(dg, sg), _unsunk(db, sbt),
                None if sls is not None else dls.to(ctx.ls_dtype), None, None, None)


def add_layer_norm_scaled(x: torch.Tensor, delta: torch.Tensor, gamma: torch.Tensor, beta: torch.Tensor,
                          layerscale: torch.Tensor, rowscale: Optional[torch.Tensor] = None,
                          eps: float = LN_EPS):
    """CaiT residual add ``x + delta * layerscale * rowscale[sample]`` (layerscale.py:21-23 and the
    stochastic-depth factor mask / keep, stochastic_depth.py:19-28) with its LayerNorm, one kernel;
    returns ``(x_out, LN(x_out))``.  ``rowscale`` [B] fp32 or None; x [B, N, C] fp32."""
    _require_gpu(x, delta)
    if rowscale is not None:
        rowscale = rowscale.float().contiguous()
    return _AddLayerNormScaled.apply(x, delta, gamma, beta, layerscale, rowscale, x.shape[1], eps)


def layer_norm(x: torch.Tensor, gamma: torch.Tensor, beta: torch.Tensor, eps: float = LN_EPS) -> torch.Tensor:
    """Flax ``nn.LayerNorm(dtype=bfloat16)`` of an fp32 residual stream: bf16 output (HIP kernel)."""
    _require_gpu(x)
    return _LayerNorm.apply(x, gamma, beta, eps)


def add_layer_norm(x: torch.Tensor, delta: torch.Tensor, gamma: torch.Tensor, beta: torch.Tensor,
                   eps: float = LN_EPS):
    """``x + delta`` (fp32 residual add, models/vit.py:24,31) and its LayerNorm in bf16, one kernel;
    returns ``(x + delta, LN(x + delta))``."""
    _require_gpu(x, delta)
    return _AddLayerNorm.apply(x, delta, gamma, beta, eps)


# ------------------------------------------------------------------------------ training loss
class _SmoothedCE(torch.autograd.Function):
    """Label-smoothed softmax cross entropy, mean over rows (train.py:77-90: optax.smooth_labels +
    jnp.mean(optax.softmax_cross_entropy)) in three HIP launches (sae_smoothed_ce_fwd / _bwd);
    dlogits come back in the logits' dtype."""

    @staticmethod
    def forward(ctx, logits, labels, alpha):
        lib = L.load()
        R, K = logits.shape
        lse = torch.empty(R, dtype=torch.float32, device=logits.device)
        row_loss = torch.empty(R, dtype=torch.float32, device=logits.device)
        loss = torch.empty((), dtype=torch.float32, device=logits.device)
        L.check(lib.sae_smoothed_ce_fwd(_stream(logits), R, K, _ptr(logits), logits.stride(0), dtype_code(logits.dtype),
                                        _ptr(labels), float(alpha), _ptr(lse), _ptr(row_loss), _ptr(loss)))
        ctx.save_for_backward(logits, labels, lse)
        ctx.alpha = float(alpha)
        return loss

    @staticmethod
    @_sinking
    def backward(ctx, gloss):
        lib = L.load()
        logits, labels, lse = ctx.saved_tensors
        R, K = logits.shape
        g = gloss.float().contiguous()
        dx = torch.empty((R, K), dtype=logits.dtype, device=logits.device)
        L.check(lib.sae_smoothed_ce_bwd(_stream(logits), R, K, _ptr(logits), logits.stride(0), dtype_code(logits.dtype),
                                        _ptr(labels), ctx.alpha, _ptr(lse), _ptr(g), _ptr(dx), dx.stride(0)))
        return dx, None, None


def smoothed_cross_entropy(logits: torch.Tensor, labels: torch.Tensor, alpha: float = 0.1) -> torch.Tensor:
    """mean_r [lse_r - (1 - alpha) x[r, y_r] - (alpha / K) sum_c x[r, c]] of [R, K] GPU logits (bf16 or
    fp32) against int64 labels [R]; the HIP kernels, or an error when they cannot take the input."""
    _require_gpu(logits, labels)
    if logits.dim() != 2 or logits.stride(1) != 1:
        logits = logits.reshape(-1, logits.shape[-1]).contiguous()
    return _SmoothedCE.apply(logits, labels.to(torch.int64).contiguous(), alpha)


# ------------------------------------------------------------------------ encoder input tokens
class _EncoderTokens(torch.autograd.Function):
    """concat(cls, float(tokens)) + pos (models/vit.py:82-85,46; position_embed.py:48) in one HIP
    pass each way (sae_tokens_fwd / _bwd); cls / pos gradients go into their sinks when the
    multi-rank step registered them."""

    @staticmethod
    def forward(ctx, tokens, cls, pos):
        lib = L.load()
        B, Lt, E = tokens.shape
        x = torch.empty((B, Lt + 1, E), dtype=torch.float32, device=tokens.device)
        L.check(lib.sae_tokens_fwd(_stream(tokens), B, Lt, E, _ptr(tokens), _ptr(cls), _ptr(pos), _ptr(x)))
        ctx.shape = (B, Lt, E)
        ctx.sinks = (_sink(cls), _sink(pos))
        ctx.meta = (cls.shape, pos.shape)
        return x

    @staticmethod
    @_sinking
    def backward(ctx, dx):
        lib = L.load()
        B, Lt, E = ctx.shape
        dx = _f32c(dx, "dx")
        dtok = torch.empty((B, Lt, E), dtype=torch.bfloat16, device=dx.device)
        scls, spos = ctx.sinks
        dcls = _claim(scls) if scls is not None else torch.empty(ctx.meta[0], dtype=torch.float32, device=dx.device)
        dpos = _claim(spos) if spos is not None else torch.empty(ctx.meta[1], dtype=torch.float32, device=dx.device)
        L.check(lib.sae_tokens_bwd(_stream(dx), B, Lt, E, _ptr(dx), _ptr(dtok), _ptr(dcls), _ptr(dpos)))
        return dtok, _unsunk(dcls, scls), _unsunk(dpos, spos)


def encoder_tokens_ok(tokens: torch.Tensor, cls: torch.Tensor, pos: torch.Tensor) -> bool:
    """Inputs sae_tokens_fwd takes: bf16 [B, L, E] tokens, fp32 contiguous cls [.., E] and pos [1, L+1, E]."""
    if not (tokens.is_cuda and tokens.dtype == torch.bfloat16 and tokens.dim() == 3 and tokens.is_contiguous()):
        return False
    B, Lt, E = tokens.shape
    return (E % 4 == 0 and E <= 4096 and tokens.data_ptr() % 8 == 0
            and cls.dtype == torch.float32 and cls.is_contiguous() and cls.numel() == E and cls.data_ptr() % 16 == 0
            and pos.dtype == torch.float32 and pos.is_contiguous() and pos.numel() == (Lt + 1) * E
            and pos.data_ptr() % 16 == 0)


def encoder_tokens(tokens: torch.Tensor, cls: torch.Tensor, pos: torch.Tensor) -> torch.Tensor:
    """fp32 [B, L+1, E] encoder input = concat(cls, float(tokens)) + pos (see _EncoderTokens)."""
    _require_gpu(tokens, cls, pos)
    if not encoder_tokens_ok(tokens, cls, pos):
        raise ValueError("encoder_tokens: needs bf16 contiguous tokens [B, L, E] (E % 4 == 0) and fp32 "
                         "contiguous cls [E] / pos [L+1, E]")
    return _EncoderTokens.apply(tokens, cls, pos)


class _LayerNormPass(torch.autograd.Function):
    """(x, LN(x)): the encoder's first LayerNorm, returning its input as the residual stream so that
    the backward adds the residual gradient in the LayerNorm backward kernel (dx = dxout + LN'^T dy)
    instead of autograd summing the two paths in a separate pass."""

    @staticmethod
    def forward(ctx, x, gamma, beta, eps):
        _, y, mean, rstd = _ln_fwd(x, None, gamma, beta, eps)
        ctx.save_for_backward(x, mean, rstd, gamma)
        ctx.sinks = (_sink(gamma), _sink(beta))
        return x, y

    @staticmethod
    @_sinking
    def backward(ctx, dxout, dy):
        x, mean, rstd, gamma = ctx.saved_tensors
        if dy is None:
            dy = torch.zeros(x.shape, dtype=torch.bfloat16, device=x.device)
        dx, _, dg, db = _ln_bwd(x, mean, rstd, gamma, dy, dxout, False, ctx.sinks)
        return dx, _unsunk(dg, ctx.sinks[0]), _unsunk(db, ctx.sinks[1]), None


def layer_norm_pass(x: torch.Tensor, gamma: torch.Tensor, beta: torch.Tensor, eps: float = LN_EPS):
    """(x, LayerNorm(x)) -- see _LayerNormPass."""
    _require_gpu(x, gamma, beta)
    return _LayerNormPass.apply(x, gamma, beta, eps)


class _ClsAddLayerNorm(torch.autograd.Function):
    """LayerNorm(x[:, 0] + delta[:, 0]) -> bf16 [B, E]: the encoder's final residual add and
    LayerNorm on the class-token rows only (ViT's head reads token 0, vit.py:95; the LayerNorm is
    row-wise, so those rows' values equal the full pass's).  The backward writes the class rows of
    dx (fp32) and ddelta (bf16); the other rows take no gradient from here."""

    @staticmethod
    def forward(ctx, x, delta, gamma, beta, eps):
        xout, y, mean, rstd = _ln_fwd(x[:, 0], delta[:, 0], gamma, beta, eps)
        ctx.save_for_backward(xout, mean, rstd, gamma)
        ctx.meta = (x.shape, delta.dtype)
        ctx.sinks = (_sink(gamma), _sink(beta))
        return y

    @staticmethod
    @_sinking
    def backward(ctx, dy):
        xout, mean, rstd, gamma = ctx.saved_tensors
        shape, ddt = ctx.meta
        dxc, ddc, dg, db = _ln_bwd(xout, mean, rstd, gamma, dy, None, True, ctx.sinks)
        dx = torch.zeros(shape, dtype=torch.float32, device=dxc.device)
        dx[:, 0] = dxc
        dd = torch.zeros(shape, dtype=ddt, device=dxc.device)
        dd[:, 0] = ddc
        return dx, dd, _unsunk(dg, ctx.sinks[0]), _unsunk(db, ctx.sinks[1]), None


def cls_add_layer_norm(x: torch.Tensor, delta: torch.Tensor, gamma: torch.Tensor, beta: torch.Tensor,
                       eps: float = LN_EPS) -> torch.Tensor:
    """bf16 LayerNorm(x[:, 0] + delta[:, 0]) of the [B, N, E] residual stream -- see _ClsAddLayerNorm."""
    _require_gpu(x, delta, gamma, beta)
    return _ClsAddLayerNorm.apply(x, delta, gamma, beta, eps)
