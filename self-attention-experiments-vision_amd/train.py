"""Data-parallel training step (train.py:77-109 of the reference, rebuilt for MI355X).

One process per GPU, ``torch.distributed`` with backend ``nccl`` (= RCCL on ROCm) over
xGMI.  The reference's ``jax.pmap(train_step)`` + ``lax.pmean(grads)`` (train.py:94-96,230)
becomes: every parameter's gradient is a 16-byte-aligned view into ONE flat fp32 buffer, cut
into buckets along parameter boundaries in the order the backward finishes them; the backward
kernels write the gradients straight into their views (gradient sinks, ops.set_grad_sinks), and
as soon as the last gradient of a bucket is written its SUM all-reduce (of the gradients of
loss / world = the global-batch mean) is launched on a communication stream, overlapping the
rest of the backward; the compute stream joins that stream before the one-launch AdamW.  On the
GPU the whole step -- forward, loss, backward with the overlapped bucket all-reduces, AdamW -- is
ONE HIP graph (RCCL collectives are graph-capturable: tools/probe/rccl_graph.py), so a step costs
one host call.  Survey D9 decisions: standard descent (the reference's optax chain ascends), the
gradient is the global batch mean (the reference divides the loss by device_count *and*
pmean's), no wandb call inside the step.

Collective modes (``TrainStep.collective``): "overlap" (default whenever there is a process group:
bucket all-reduces launched from inside the backward), "between" (``two_graphs=True``: forward +
backward graph, the bucket all-reduces, optimizer graph), "host" (gloo with CUDA tensors, the
multi-rank rehearsal on one GPU: an explicit host round trip between two graphs), "none" (no
process group).  ``SAE_WORLD1_RCCL=1`` (bench.py ``--world1-rccl``) creates a world-size-1 RCCL
group so the overlapped collective path runs on a one-GPU box.

Loss: one-hot -> optax.smooth_labels(0.1) -> softmax cross-entropy, mean (train.py:83-92).
Optimizer: Adam + decoupled weight decay 1e-4, lr 5e-4 * batch/512 (train.py:25-27,229-233;
constant schedule: the warmup-cosine value does not change the work per step).
"""
from __future__ import annotations

import os
from typing import Optional

import torch
import torch.distributed as dist
import torch.nn.functional as F

__all__ = ["smoothed_cross_entropy", "TrainStep", "init_distributed", "FusedAdamW"]


def smoothed_cross_entropy(logits: torch.Tensor, labels: torch.Tensor, smoothing: float = 0.1) -> torch.Tensor:
    """train.py:77-90 (optax.smooth_labels + mean softmax cross entropy): on the GPU the two-launch
    HIP loss (ops.smoothed_cross_entropy); CPU tensors (the multi-process gloo tests' small
    models) take torch's cross entropy, which computes the same quantity."""
    if logits.is_cuda:
        from . import ops
        return ops.smoothed_cross_entropy(logits, labels, smoothing)
    return F.cross_entropy(logits.float(), labels, label_smoothing=smoothing)


def init_distributed():
    """Initialise the process group from torchrun's env (RANK/WORLD_SIZE/LOCAL_RANK/MASTER_*).
    ``SAE_WORLD1_RCCL=1`` at world size 1 (GPU): a one-rank RCCL group, so the training step's
    collective path (the overlapped bucket all-reduces captured in the step's HIP graph) runs."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # SAE_DIST_BACKEND=gloo rehearses the multi-rank path on fewer GPUs than ranks (ranks share
    # devices round-robin; gloo all-reduces the CUDA gradients through host memory)
    backend = os.environ.get("SAE_DIST_BACKEND") or ("nccl" if torch.cuda.is_available() else "gloo")
    if torch.cuda.is_available():
        local = local % max(1, torch.cuda.device_count()) if backend == "gloo" else local
    world1 = world == 1 and os.environ.get("SAE_WORLD1_RCCL", "0") == "1" and torch.cuda.is_available()
    if backend == "nccl" or world1:
        # Peer connections at communicator creation, not at a communicator's first collective:
        # RCCL (2.26 bundled with torch, 2.27 in /opt/rocm; both read NCCL_RUNTIME_CONNECT) by
        # default connects the ring / tree peers lazily, inside the first collective that needs
        # them -- for the gradient group that first collective is issued INSIDE the step's graph
        # capture (TrainStep._cpg), where the connection setup's allocations and host handshakes
        # would run in a capturing context.  With 0 every communicator -- the default one created
        # by init_process_group(device_id=) and the gradient group's by new_group(device_id=) --
        # is fully connected when its creation returns, so the captured collectives only enqueue
        # kernels.  A value the user exported wins.
        os.environ.setdefault("NCCL_RUNTIME_CONNECT", "0")
    if (world > 1 or world1) and not dist.is_initialized():
        if torch.cuda.is_available():
            torch.cuda.set_device(local)
        if world1:
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            if "MASTER_PORT" not in os.environ:
                import socket
                with socket.socket() as sk:
                    sk.bind(("127.0.0.1", 0))
                    os.environ["MASTER_PORT"] = str(sk.getsockname()[1])
            dist.init_process_group(backend="nccl", rank=0, world_size=1, device_id=torch.device("cuda", local))
        elif backend == "nccl":
            # device_id: the communicator is created now (eagerly), not by the first collective
            dist.init_process_group(backend=backend, device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend=backend)
    elif torch.cuda.is_available():
        torch.cuda.set_device(local)
    return rank, world, local


def agree_all_ranks(ok: bool, group) -> bool:
    """True iff ``ok`` holds on every rank of ``group`` (a MIN all-reduce of one flag over a
    host-side gloo group).  TrainStep decides with it whether the captured graph is used: at
    world > 1 one rank's capture failure turns the graph off on every rank, so that all ranks
    issue the same collectives in the same order."""
    flag = torch.tensor([1 if ok else 0], dtype=torch.int32)
    dist.all_reduce(flag, op=dist.ReduceOp.MIN, group=group)
    return bool(flag.item())


def flat_layout(params, align: int = 4):
    """Offsets of ``params`` in one flat fp32 buffer, each rounded up to ``align`` elements (16
    bytes): every gradient view starts 16-byte aligned, as the vector stores of the kernels that
    write them in place (gemm_dw, patch_embed_bwd, tokens_bwd) require.  Returns (offsets, total)."""
    offs, off = [], 0
    for p in params:
        offs.append(off)
        off += -(-p.numel() // align) * align
    return offs, off


class FusedAdamW:
    """AdamW (optax.adamw of train.py:25-27,229-233, torch.optim.AdamW's update order) for fp32 GPU
    parameters whose gradients live in one flat buffer: every parameter in one HIP launch
    (``sae_adamw_step``, csrc/adamw.h) instead of torch's multi-tensor launches.  The moments are
    two more flat buffers laid out like the gradients; the step counter stays on the device, so the
    update can be captured in a HIP graph and replayed.

    ``cast_groups``: column-stacked groups of 2-D fp32 Dense kernels (the ``ops.cast_weights``
    groups; each kernel a whole parameter, possibly reshaped) whose bf16 compute copies the
    update writes as it goes (``sae_adamw_step_cast``): the forward then reads persistent copies
    (``ops.register_persistent_casts``) instead of casting every weight at its start.  Parameter
    values are bit-identical either way."""

    def __init__(self, params, flat_grad: torch.Tensor, lr: float, betas=(0.9, 0.999), eps: float = 1e-8,
                 weight_decay: float = 0.0, cast_groups=None):
        import ctypes
        from . import _lib as L
        from . import ops
        self.lib = L.load()
        self.params = list(params)
        self.lr, self.betas, self.eps, self.weight_decay = float(lr), tuple(betas), float(eps), float(weight_decay)
        dev = flat_grad.device
        self.m = torch.zeros_like(flat_grad)
        self.v = torch.zeros_like(flat_grad)
        self.step_count = torch.zeros(1, dtype=torch.int32, device=dev)
        # copies an earlier optimizer over these parameters registered would go stale under this
        # one (it updates the weights through raw pointers): they stop being served
        ops.release_persistent_casts(self.params)
        slot = {}
        for i, p in enumerate(self.params):
            g = p.grad
            if (p.dtype != torch.float32 or not p.is_contiguous() or g is None or g.dtype != torch.float32
                    or not g.is_contiguous() or g.data_ptr() < flat_grad.data_ptr()):
                raise ValueError("FusedAdamW: fp32 contiguous parameters with views of the flat gradient buffer")
            off = (g.data_ptr() - flat_grad.data_ptr()) // 4
            slot[p.data_ptr()] = (i, p, g.data_ptr(), self.m.data_ptr() + 4 * off, self.v.data_ptr() + 4 * off)
        # the Dense kernels whose copies the update writes: whole parameters, shapes / alignment
        # the tile path takes (K, N, column offsets multiples of 4)
        self.cast_groups, self.copies = [], []
        tiles_in = []
        claimed = set()
        for ws in (cast_groups or []):
            K = ws[0].shape[0]
            ent = [slot.get(w.data_ptr()) for w in ws]
            if (any(e is None or e[1].numel() != w.numel() for e, w in zip(ent, ws))
                    or any(e[0] in claimed for e in ent)          # a parameter is updated once
                    or len({e[0] for e in ent}) != len(ent)
                    or any(w.dim() != 2 or w.shape[0] != K for w in ws)
                    or K % 4 or any(w.shape[1] % 4 for w in ws)
                    or any(e[2] % 16 or e[3] % 16 or e[4] % 16 or e[1].data_ptr() % 16 for e in ent)):
                continue
            claimed.update(e[0] for e in ent)
            N = sum(w.shape[1] for w in ws)
            w16 = torch.empty((K, N), dtype=torch.bfloat16, device=dev)
            wt16 = torch.empty((N, K), dtype=torch.bfloat16, device=dev)
            col = 0
            for e, w in zip(ent, ws):
                tiles_in.append((e, K, w.shape[1], w16, wt16, N, col))
                col += w.shape[1]
            self.cast_groups.append(list(ws))
            self.copies.append((w16, wt16))
        in_tiles = {e[0] for e, *_ in tiles_in}
        flat_idx = [i for i in range(len(self.params)) if i not in in_tiles]
        n = len(flat_idx)
        P = (ctypes.c_void_p * max(1, n))()
        G, M, V = (ctypes.c_void_p * max(1, n))(), (ctypes.c_void_p * max(1, n))(), (ctypes.c_void_p * max(1, n))()
        Nn = (ctypes.c_int64 * max(1, n))()
        for j, i in enumerate(flat_idx):
            p = self.params[i]
            _, _, G[j], M[j], V[j] = slot[p.data_ptr()]
            P[j], Nn[j] = p.data_ptr(), p.numel()
        cap = sum((self.params[i].numel() + L.SAE_ADAMW_CHUNK - 1) // L.SAE_ADAMW_CHUNK for i in flat_idx)
        table = (L.AdamwChunk * max(1, cap))()
        cnt = ctypes.c_int64(0)
        L.check(self.lib.sae_adamw_plan(n, P, G, M, V, Nn, table, cap, ctypes.byref(cnt)))
        self.n_chunks = int(cnt.value)
        self.table = torch.frombuffer(bytearray(table), dtype=torch.uint8).to(dev)   # device copy, built once
        self.n_tiles = 0
        self.tiles = None
        if tiles_in:
            k = len(tiles_in)
            arr = lambda t: (t * k)()
            P, G, M, V, W16, WT = (arr(ctypes.c_void_p) for _ in range(6))
            Kx, Nx, LD, LT, C0 = (arr(ctypes.c_int32) for _ in range(5))
            for j, (e, K, Nw, w16, wt16, Ntot, col) in enumerate(tiles_in):
                P[j], G[j], M[j], V[j] = e[1].data_ptr(), e[2], e[3], e[4]
                W16[j], WT[j] = w16.data_ptr(), wt16.data_ptr()
                Kx[j], Nx[j], LD[j], LT[j], C0[j] = K, Nw, Ntot, K, col
            cap = sum(-(-K // 64) * -(-Nw // 64) for _, K, Nw, *_ in tiles_in)
            ttab = (L.AdamwCastTile * cap)()
            L.check(self.lib.sae_adamw_cast_plan(k, P, G, M, V, Kx, Nx, W16, LD, WT, LT, C0, ttab, cap,
                                                 ctypes.byref(cnt)))
            self.n_tiles = int(cnt.value)
            self.tiles = torch.frombuffer(bytearray(ttab), dtype=torch.uint8).to(dev)
            # the owner token: unregistering (close, finalizer) removes only this optimizer's entries
            self._owner = object()
            ops.register_persistent_casts(self.cast_groups, [c[0] for c in self.copies], [c[1] for c in self.copies],
                                          self._owner)
            ops.recast_persistent(self.cast_groups)   # the copies of the initial weights
            # the registry holds the weights (their addresses cannot be reused while registered);
            # it lets go of them with the optimizer
            import weakref
            weakref.finalize(self, ops.unregister_persistent_casts, list(self.cast_groups), self._owner)

    def step(self):
        from . import _lib as L
        b1, b2 = self.betas
        st = torch.cuda.current_stream(self.m.device).cuda_stream
        if self.n_tiles:
            L.check(self.lib.sae_adamw_step_cast(st, self.n_chunks, self.table.data_ptr(), self.n_tiles,
                                                 self.tiles.data_ptr(), self.step_count.data_ptr(), self.lr, b1, b2,
                                                 self.eps, self.weight_decay))
        else:
            L.check(self.lib.sae_adamw_step(st, self.n_chunks, self.table.data_ptr(), self.step_count.data_ptr(),
                                            self.lr, b1, b2, self.eps, self.weight_decay))

    def refresh_casts(self):
        """Re-cast the copies after the parameters were overwritten outside the update."""
        if self.cast_groups:
            from . import ops
            ops.recast_persistent(self.cast_groups)

    def refresh_if_stale(self):
        """Re-cast the copies if a weight was changed in place since they were written: a replayed
        step graph does not contain the cast, so a load_state_dict / copy_ after the capture would
        otherwise reach the forward only after the next update.  Host-side version check."""
        if self.cast_groups:
            from . import ops
            if ops.persistent_casts_stale(self.cast_groups):
                ops.recast_persistent(self.cast_groups)

    def close(self):
        """Stop serving the copies (the forward casts per call again)."""
        if self.cast_groups:
            from . import ops
            ops.unregister_persistent_casts(self.cast_groups, self._owner)
            self.cast_groups = []

    def state_tensors(self):
        return [self.m, self.v, self.step_count]


class TrainStep:
    """``step(images, labels)`` = forward (bf16 compute) + loss + backward (+ bucketed all-reduce of
    the flat gradient when there is a process group) + optimizer update.  No host sync.

    graph=True (GPU): the whole step is one HIP graph (collective "overlap" or "none"); with
    ``two_graphs=True`` (collective "between") or the gloo rehearsal ("host"): graph 1 = forward +
    loss + backward, the bucket all-reduces, graph 2 = AdamW."""

    def __init__(self, model: torch.nn.Module, global_batch: int, lr: float = 5e-4, weight_decay: float = 1e-4,
                 label_smoothing: float = 0.1, bucket_cap_mb: float = 25.0, device: Optional[torch.device] = None,
                 graph: bool = False, input_layout: str = "NHWC", flat_grads: Optional[bool] = None,
                 grad_sinks: bool = True, two_graphs: Optional[bool] = None, persistent_casts: bool = True,
                 wgrad_stream: Optional[bool] = None):
        # input_layout "HWCN": the batch arrives as the reference's train-step feed [H, W, C, N]
        # (train.py:80, input_pipeline.py:187-191) and the model's patch GEMM gathers from it
        self.input_layout = input_layout
        self.pg = dist.is_initialized()
        self.world = dist.get_world_size() if self.pg else 1
        self.graph = bool(graph) and torch.cuda.is_available()
        self._g = self._g_opt = None
        self.model = model
        params = [p for p in model.parameters() if p.requires_grad]
        self._params = params
        if self.world > 1:
            self._broadcast_from_rank0([t for t in model.state_dict().values() if torch.is_tensor(t)])
        # flat_grads (default: on the GPU, and whenever there is a process group): one flat gradient
        # buffer written in place by the backward kernels (gradient sinks), stepped by the one-launch
        # FusedAdamW
        on_gpu = all(p.is_cuda for p in params)
        self.flat = (self.pg or on_gpu) if flat_grads is None else bool(flat_grads)
        if not self.pg:
            self.collective = "none"
        elif on_gpu and dist.get_backend() == "gloo":
            self.collective = "host"
        elif two_graphs:
            self.collective = "between"
        else:
            self.collective = "overlap"
        if self.collective != "none" and not self.flat:
            raise ValueError("TrainStep: the collective path needs the flat gradient buffer")
        # the gradient all-reduces run on a process group of their own, created with an eager
        # communicator (device_id) and given no eager work before the capture: RCCL's watchdog
        # thread then never holds an event recorded on that group's internal stream, which joins
        # the step's capture (an event query on a capturing stream is hipErrorCapturedEvent,
        # fatal in the watchdog).  The warm-up steps before the capture run without collectives.
        self._cpg = None
        self._comm_on = True
        # "flagged" (graph steps with the overlapped collective, default on the GPU): the captured
        # forward + backward stays ONE linear kernel chain -- at each bucket's ready point it bumps a
        # device flag (sae_flag_bump) instead of forking the all-reduce onto the communication stream
        # inside the graph -- and after each replay the host enqueues, on the communication stream,
        # every bucket's wait for its flag (hipStreamWaitValue32) followed by its RCCL all-reduce,
        # so the rings still run beside the rest of the backward.  A branch inside a replayed HIP graph
        # costs the whole replay 0.13-0.4 ms on this runtime (the multi-queue launch path, measured
        # with one-rank RCCL + a stand-in kernel per bucket: profiles/r06e_graph_fork.txt,
        # r06d_rccl_emulation.txt); a linear graph keeps the single-queue fast path.  SAE_FLAGGED=0:
        # the round-3 structure (the all-reduces forked inside the one graph).
        self._flagged = False
        # one-GPU contention emulation of an N-GPU node (bench.py --emulate-rccl, env
        # SAE_EMULATE_RCCL="channels,busbw_GBps,world[,lds_KiB[,threads]]"): beside each bucket's
        # (one-rank) all-reduce, `channels` workgroups of `threads` threads holding `lds_KiB` of LDS
        # (default 64 KiB, 256) occupy CUs on the communication stream for the ring time the bucket
        # would take at `world` GPUs, 2 (world - 1) / world x bytes / busbw -- the CU footprint of
        # RCCL's ring channels on the compute units the backward is using
        self._emulate = None
        em = os.environ.get("SAE_EMULATE_RCCL", "")
        if em:
            f = [float(x) for x in em.split(",")] + [64.0, 256.0][max(0, len(em.split(",")) - 3):]
            self._emulate = (int(f[0]), f[1], int(f[2]), int(f[3] * 1024), int(f[4]))
        if self.collective in ("overlap", "between") and on_gpu:
            self._cpg = dist.new_group(backend="nccl", device_id=params[0].device)
        # world > 1: whether the step runs as a graph is decided by ALL ranks together (a host-side
        # gloo group carries the one flag all-reduce): a rank whose capture fails must not run the
        # eager step while its peers replay graphs -- their collective sequences would differ
        self._flag_pg = dist.new_group(backend="gloo") if self.world > 1 and self.graph else None
        self._flagged = (self.collective == "overlap" and self.graph and on_gpu
                         and os.environ.get("SAE_FLAGGED", "1") != "0")
        self.two_graphs = (self.collective in ("between", "host") or (self.collective == "none" and bool(two_graphs))
                           or self._flagged)
        if self.flat:
            # one flat fp32 gradient buffer, every .grad a 16-byte-aligned view into it (autograd
            # accumulates into the views in place), cut into buckets of ~bucket_cap_mb along
            # parameter boundaries in reverse registration order (the order the backward finishes
            # them; a bucket closes once it holds >= cap elements)
            offs, n = flat_layout(params)
            self._offs = offs
            dev = params[0].device
            self._flat = torch.zeros(n, dtype=torch.float32, device=dev)
            for p, off in zip(params, offs):
                p.grad = self._flat[off:off + p.numel()].view_as(p)
            cap = max(1, int(bucket_cap_mb * 2 ** 20 / 4))
            self._buckets, self._bucket_params = [], []
            hi, members = n, []
            for i in reversed(range(len(params))):
                members.append(i)
                lo = offs[i]
                if hi - lo >= cap:
                    self._buckets.append((lo, hi))
                    self._bucket_params.append(members)
                    hi, members = lo, []
            if members:
                self._buckets.append((0, hi))
                self._bucket_params.append(members)
            self._bucket_of = {i: b for b, ms in enumerate(self._bucket_params) for i in ms}
            # the backward kernels write each parameter's gradient straight into its flat view
            # (ops.set_grad_sinks) instead of autograd adding a fresh gradient tensor into it
            self._sinks = bool(grad_sinks)
            if self._sinks:
                from . import ops
                ops.set_grad_sinks(params, [p.grad for p in params])
            if self.collective == "overlap":
                self._arm_overlap_hooks()
            if self._flagged:
                # one int32 counter per bucket, bumped once per replay of the forward + backward graph
                self._flags = torch.zeros(len(self._buckets), dtype=torch.int32, device=dev)
                self._flag_order = []   # bucket order of the captured bumps (the host's issue order)
                self._epoch = 0
        # the sink-bound weight-gradient GEMMs run on a side stream beside the input-gradient chain
        # (ops.set_weight_grad_stream), opt-in: SAE_WG_STREAM=1 or wgrad_stream=True.  Off by default: the
        # concurrent dW kernels push the persistent gemm8 tiles into a tail (DeiT-S 15,381 vs
        # 15,619 img/s, profiles/r05i_wgstream_rejected.txt)
        if wgrad_stream is None:
            wgrad_stream = os.environ.get("SAE_WG_STREAM", "0") == "1"
        self._wg = (torch.cuda.Stream(device=params[0].device)
                    if wgrad_stream and self.flat and self._sinks and on_gpu else None)
        base_lr = lr * (global_batch / 512)
        kw = dict(lr=base_lr, betas=(0.9, 0.999), eps=1e-8, weight_decay=weight_decay)
        self.opt = None
        if self.flat and on_gpu and all(p.dtype == torch.float32 and p.is_contiguous() for p in params):
            # the bf16 Dense copies written by the update (models that name them, bf16 compute)
            groups = model.cast_groups() if persistent_casts and hasattr(model, "cast_groups") else None
            self.opt = FusedAdamW(params, self._flat, cast_groups=groups, **kw)
        else:
            if self.graph:
                kw["capturable"] = True   # step counters on the device: replayable
            try:
                self.opt = torch.optim.AdamW(params, fused=True, **kw)
            except (RuntimeError, TypeError):
                self.opt = torch.optim.AdamW(params, foreach=True, **kw)
        self.smoothing = label_smoothing

    @staticmethod
    def _broadcast_from_rank0(tensors):
        """Once, at construction: every replica starts from rank 0's parameters and buffers (the
        reference's pmap replicates one host-initialised state, train.py:226-228), whatever seed
        each rank used.  One flat broadcast per dtype, not one per tensor."""
        by_dtype = {}
        for t in tensors:
            by_dtype.setdefault(t.dtype, []).append(t)
        for ts in by_dtype.values():
            flat = torch.cat([t.detach().reshape(-1) for t in ts])
            if flat.is_cuda and dist.get_backend() == "gloo":
                host = flat.cpu()
                dist.broadcast(host, src=0)
                flat.copy_(host)
            else:
                dist.broadcast(flat, src=0)
            off = 0
            with torch.no_grad():
                for t in ts:
                    t.copy_(flat[off:off + t.numel()].view_as(t))
                    off += t.numel()

    # ---- the overlapped bucket all-reduce
    def _arm_overlap_hooks(self):
        """A parameter's gradient is final when the kernel writing its sink has been enqueued
        (ops.set_sink_listener) or, for gradients autograd accumulates, after its accumulation
        (post-accumulate-grad hook); the bucket holding it is launched once all of its parameters
        are final."""
        from . import ops
        self._armed = False
        self._ptr_to_idx = {p.grad.data_ptr(): i for i, p in enumerate(self._params)}
        ops.set_sink_listener(self._on_sink)
        for i, p in enumerate(self._params):
            p.register_post_accumulate_grad_hook(lambda _p, i=i: self._on_ready(i))
        if self._flat.is_cuda:
            self._comm = torch.cuda.Stream(device=self._flat.device)

    def _on_sink(self, ptr):
        i = self._ptr_to_idx.get(ptr)
        if i is not None:
            self._on_ready(i)

    def _on_ready(self, i):
        if not self._armed or i in self._ready:
            return
        self._ready.add(i)
        b = self._bucket_of[i]
        self._remaining[b] -= 1
        if self._remaining[b] == 0:
            self._launch_bucket(b)

    def _launch_bucket(self, b):
        lo, hi = self._buckets[b]
        t = self._flat[lo:hi]
        self._launched[b] = True
        if not self._comm_on:   # the capture's warm-up steps: no collective
            return
        if self._flagged and torch.cuda.is_current_stream_capturing():
            # flagged graph: a mark on the captured chain; the collective is issued after the replay
            from . import ops
            ops.flag_bump(self._flags, b)
            self._flag_order.append(b)
            return
        if t.is_cuda:
            # the comm stream picks up everything enqueued so far on the compute stream (this
            # bucket's gradient kernels included) and runs the RCCL all-reduce beside the rest of
            # the backward; inside a graph capture this is a fork of the captured graph
            self._comm.wait_stream(torch.cuda.current_stream(t.device))
            with torch.cuda.stream(self._comm):
                dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self._cpg)
                if self._emulate is not None:
                    from . import ops
                    ch, bw, wd, lds, thr = self._emulate
                    usec = 2.0 * (wd - 1) / wd * t.numel() * 4 / (bw * 1e3)
                    ops.occupy_cus(self._comm, ch, usec, threads=thr, lds_bytes=lds)
        else:
            self._works.append(dist.all_reduce(t, op=dist.ReduceOp.SUM, async_op=True))

    def _begin_overlap(self):
        self._ready = set()
        self._remaining = [len(ms) for ms in self._bucket_params]
        self._launched = [False] * len(self._buckets)
        self._works = []
        self._armed = True

    def _end_overlap(self):
        self._armed = False
        for b in range(len(self._buckets)):   # buckets holding a parameter that got no gradient
            if not self._launched[b]:
                self._launch_bucket(b)
        if self._flat.is_cuda:
            if not (self._flagged and torch.cuda.is_current_stream_capturing()):
                torch.cuda.current_stream(self._flat.device).wait_stream(self._comm)   # the join
        else:
            for w in self._works:
                w.wait()
        self._works = []

    # ---- pieces of one step
    def _zero_grad(self):
        if self.flat:
            ranges = getattr(self, "_zero_ranges", None)
            if ranges is None:
                self._flat.zero_()
            else:   # only the gradients autograd accumulates (every sink is overwritten)
                for lo, hi in ranges:
                    self._flat[lo:hi].zero_()
        else:
            self.opt.zero_grad(set_to_none=True)

    def _note_sunk(self):
        """After a graph-mode backward: the flat ranges of the parameters whose gradients did NOT
        go through a sink (autograd adds into those, so they need zeroing before the next
        backward).  Graph mode only: the captured step writes the same sinks on every replay."""
        from . import ops
        written = set(ops._SINK_WRITTEN)
        ranges = []
        for p, off in zip(self._params, self._offs):
            n = p.numel()
            if p.grad is None or p.grad.data_ptr() not in written:
                if ranges and ranges[-1][1] == off:
                    ranges[-1] = (ranges[-1][0], off + n)
                else:
                    ranges.append((off, off + n))
        # many scattered ranges would cost more launches than the one full fill saves
        self._zero_ranges = ranges if len(ranges) <= 8 else None

    def _fwd_bwd(self, images: torch.Tensor, labels: torch.Tensor) -> torch.Tensor:
        from . import ops
        self._zero_grad()
        sinks = self.flat and self._sinks
        overlap = self.collective == "overlap"
        if sinks:
            ops.begin_backward_sinks()   # the sink window: this step's forward + backward only
            ops.set_weight_grad_stream(self._wg)
        try:
            if overlap:
                self._begin_overlap()
            if self.input_layout == "NHWC":
                logits = self.model(images, is_training=True)
            else:
                logits = self.model(images, is_training=True, layout=self.input_layout)
            loss = smoothed_cross_entropy(logits, labels, self.smoothing)
            # world > 1: the SUM all-reduce of the per-rank gradients of loss / world is the
            # gradient of the global-batch mean (survey D9)
            (loss / self.world if self.world > 1 else loss).backward()
            if sinks:
                ops.join_weight_grad_stream()   # every weight gradient written before the update
            if overlap:
                self._end_overlap()
        finally:
            if sinks:
                ops.end_backward_sinks()
                ops.set_weight_grad_stream(None)
            if overlap:
                self._armed = False
        if sinks and self.graph and not torch.cuda.is_current_stream_capturing():
            self._note_sunk()
        return loss.detach()

    def _allreduce(self):
        """The all-reduce between two graphs ("between" / "host"); "overlap" runs it inside the
        backward and "none" has none."""
        if self.collective in ("none", "overlap") or not self._comm_on:
            return
        if self.collective == "host":
            # rehearsal of the multi-rank step on fewer GPUs (SAE_DIST_BACKEND=gloo): one explicit
            # host round trip (gloo's own CUDA path stalled for seconds behind the graph replays)
            host = self._flat.cpu()
            dist.all_reduce(host, op=dist.ReduceOp.SUM)
            self._flat.copy_(host)
            return
        # every bucket in flight at once on the process group's stream; the optimizer's graph
        # replay waits for them on the compute stream (no host synchronisation)
        works = [dist.all_reduce(self._flat[lo:hi], op=dist.ReduceOp.SUM, group=self._cpg, async_op=True)
                 for lo, hi in self._buckets]
        for w in works:
            w.wait()

    def _issue_flagged(self):
        """After a replay of the flagged forward + backward graph: on the communication stream, each
        bucket's wait for its flag (bumped by this replay) and its all-reduce, in the captured order;
        the compute stream joins the communication stream before the optimizer's graph."""
        from . import ops
        self._epoch += 1
        dev = self._flat.device
        for b in self._flag_order:
            lo, hi = self._buckets[b]
            t = self._flat[lo:hi]
            ops.stream_wait_flag(self._comm, self._flags, b, self._epoch)
            with torch.cuda.stream(self._comm):
                dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self._cpg)
                if self._emulate is not None:
                    ch, bw, wd, lds, thr = self._emulate
                    usec = 2.0 * (wd - 1) / wd * t.numel() * 4 / (bw * 1e3)
                    ops.occupy_cus(self._comm, ch, usec, threads=thr, lds_bytes=lds)
        torch.cuda.current_stream(dev).wait_stream(self._comm)

    def _eager(self, images: torch.Tensor, labels: torch.Tensor) -> torch.Tensor:
        loss = self._fwd_bwd(images, labels)
        self._allreduce()
        self.opt.step()
        return loss

    def _capture(self, images: torch.Tensor, labels: torch.Tensor):
        self._images = images.clone()
        self._labels = labels.clone()
        params = self._params
        snap = [p.detach().clone() for p in params]
        fused = isinstance(self.opt, FusedAdamW)
        snap_fused = [t.clone() for t in self.opt.state_tensors()] if fused else None
        had_state = set() if fused else {id(p) for p in params if p in self.opt.state and self.opt.state[p]}
        snap_state = {id(p): {k: (v.clone() if torch.is_tensor(v) else v) for k, v in self.opt.state[p].items()}
                      for p in params if id(p) in had_state}
        s = torch.cuda.Stream(device=images.device)
        s.wait_stream(torch.cuda.current_stream(images.device))
        # warm-up on a side stream (allocator, library and optimizer state), collectives off: the
        # gradient group stays free of eager work until its collectives are captured (above)
        self._comm_on = False
        try:
            with torch.cuda.stream(s):
                for _ in range(2):
                    self._eager(self._images, self._labels)
        finally:
            self._comm_on = True
        torch.cuda.current_stream(images.device).wait_stream(s)
        # the warm-up steps were only for the allocator and the optimizer's lazily created state:
        # put parameters and optimizer state back, so that the first call performs exactly ONE
        # update (the reference's one update per batch, train.py:94-100)
        with torch.no_grad():
            for p, v in zip(params, snap):
                p.copy_(v)
            if fused:
                for t, v in zip(self.opt.state_tensors(), snap_fused):
                    t.copy_(v)
                self.opt.refresh_casts()   # the bf16 copies of the restored weights
            for p in ([] if fused else params):
                st = self.opt.state.get(p)
                if not st:
                    continue
                old = snap_state.get(id(p))
                for k, v in st.items():
                    if not torch.is_tensor(v):
                        continue
                    if old is not None and torch.is_tensor(old.get(k)):
                        v.copy_(old[k])
                    else:   # state created by the warm-up: a fresh optimizer's zeros
                        v.zero_()
        if not self.flat:
            self.opt.zero_grad(set_to_none=True)
        # thread_local: RCCL's watchdog thread keeps querying the events of the default group's
        # eager work (the parameter broadcast) while the capture runs; a "global" capture would
        # refuse those queries (hipErrorStreamCaptureUnsupported, fatal in the watchdog)
        mode = "thread_local" if self.pg else "global"
        try:
            if not self.two_graphs:     # the whole step (with the overlapped collectives) in one graph
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g, capture_error_mode=mode):
                    self._loss = self._eager(self._images, self._labels)
                self._g = g
            else:                 # the collectives stay outside: two graphs around them
                g, go = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
                if self._flagged:
                    self._flag_order = []
                with torch.cuda.graph(g, capture_error_mode=mode):
                    self._loss = self._fwd_bwd(self._images, self._labels)
                with torch.cuda.graph(go, capture_error_mode=mode):
                    self.opt.step()
                self._g, self._g_opt = g, go
            ok = True
        except RuntimeError as e:   # an op that cannot be captured: stay eager, say so once
            import sys
            print(f"[train] HIP-graph capture failed ({e}); running the eager step", file=sys.stderr)
            ok = False
        self._settle_capture(ok)

    def _settle_capture(self, ok: bool):
        """Keep the captured graph(s) or go eager -- at world > 1 on every rank alike (one MIN flag
        all-reduce over the gloo group): a rank whose capture failed would otherwise run the eager
        step's collectives while its peers replay graphs."""
        if self._flag_pg is not None:
            ok = agree_all_ranks(ok, self._flag_pg)
        if not ok:
            self.graph = False
            self._g = self._g_opt = None
            if torch.cuda.is_available():
                torch.cuda.synchronize()

    def close(self):
        """Release the captured graphs and the optimizer's persistent bf16 copies.  With a process
        group, call it BEFORE destroy_process_group: a graph whose capture holds RCCL collectives
        keeps communicator resources that its destruction releases, so it must not outlive the
        communicator (left to the garbage collector, it was destroyed at an arbitrary later point)."""
        if self._g is not None or self._g_opt is not None:
            torch.cuda.synchronize()
        self._g = self._g_opt = None
        if self.collective == "overlap":
            from . import ops
            ops.set_sink_listener(None)
        if dist.is_initialized():
            for attr in ("_cpg", "_flag_pg"):
                if getattr(self, attr) is not None:
                    dist.destroy_process_group(getattr(self, attr))
                    setattr(self, attr, None)
        if isinstance(self.opt, FusedAdamW):
            self.opt.close()

    def input_buffers(self):
        """(images, labels): the captured graph's static input buffers, once the first call has
        captured it (None otherwise).  A loader that writes each batch into them saves the copy a
        call with other tensors makes before the replay."""
        if self._g is None:
            return None
        return self._images, self._labels

    def __call__(self, images: torch.Tensor, labels: torch.Tensor) -> torch.Tensor:
        if not self.graph:
            return self._eager(images, labels)
        if self._g is None:
            self._capture(images, labels)
            if not self.graph:
                return self._eager(images, labels)
        if images.data_ptr() != self._images.data_ptr():
            self._images.copy_(images)
        if labels.data_ptr() != self._labels.data_ptr():
            self._labels.copy_(labels)
        if isinstance(self.opt, FusedAdamW):
            self.opt.refresh_if_stale()
        self._g.replay()
        if self._g_opt is not None:
            if self._flagged:
                self._issue_flagged()
            else:
                self._allreduce()
            self._g_opt.replay()
        return self._loss
