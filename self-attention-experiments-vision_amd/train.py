"""Data-parallel training step (train.py:77-109 of the reference, rebuilt for MI355X).

One process per GPU, ``torch.distributed`` with backend ``nccl`` (= RCCL on ROCm) over
xGMI.  The reference's ``jax.pmap(train_step)`` + ``lax.pmean(grads)`` (train.py:94-96,230)
becomes DistributedDataParallel: fp32 gradients are all-reduced in size-capped buckets in
reverse layer order on RCCL's own stream while the backward pass is still running (the
overlap the reference lacks, survey §3.2).  Survey D9 decisions: standard descent (the
reference's optax chain ascends), the gradient is the global batch mean (the reference
divides the loss by device_count *and* pmean's), no wandb call inside the step.

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

__all__ = ["smoothed_cross_entropy", "TrainStep", "init_distributed"]


def smoothed_cross_entropy(logits: torch.Tensor, labels: torch.Tensor, smoothing: float = 0.1) -> torch.Tensor:
    return F.cross_entropy(logits.float(), labels, label_smoothing=smoothing)


def init_distributed():
    """Initialise the process group from torchrun's env (RANK/WORLD_SIZE/LOCAL_RANK/MASTER_*)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # SAE_DIST_BACKEND=gloo rehearses the multi-rank path on fewer GPUs than ranks (ranks share
    # devices round-robin; gloo all-reduces the CUDA gradients through host memory)
    backend = os.environ.get("SAE_DIST_BACKEND") or ("nccl" if torch.cuda.is_available() else "gloo")
    if torch.cuda.is_available():
        local = local % max(1, torch.cuda.device_count()) if backend == "gloo" else local
    if world > 1 and not dist.is_initialized():
        if torch.cuda.is_available():
            torch.cuda.set_device(local)
        dist.init_process_group(backend=backend)
    elif torch.cuda.is_available():
        torch.cuda.set_device(local)
    return rank, world, local


class TrainStep:
    """``step(images, labels)`` = forward (bf16 compute) + loss + backward (+ bucketed RCCL
    all-reduce overlapped with it when world > 1) + optimizer update.  No host sync."""

    def __init__(self, model: torch.nn.Module, global_batch: int, lr: float = 5e-4, weight_decay: float = 1e-4,
                 label_smoothing: float = 0.1, bucket_cap_mb: float = 25.0, device: Optional[torch.device] = None,
                 graph: bool = False, input_layout: str = "NHWC"):
        # input_layout "HWCN": the batch arrives as the reference's train-step feed [H, W, C, N]
        # (train.py:80, input_pipeline.py:187-191) and the model's patch GEMM gathers from it
        self.input_layout = input_layout
        self.world = dist.get_world_size() if dist.is_initialized() else 1
        # One HIP graph for the whole step (forward, loss, backward, AdamW): the eager step spends
        # ~10 ms/step of host time submitting ~600 launches (tools/ab_step.py), as long as the GPU
        # needs to run them.  Single-process only: with world > 1 the DDP step stays eager so the
        # RCCL all-reduce keeps overlapping the backward through DDP's bucket hooks.
        self.graph = bool(graph) and self.world == 1 and torch.cuda.is_available()
        self._g = None
        self.model = model
        if self.world > 1:
            self.ddp = torch.nn.parallel.DistributedDataParallel(
                model, device_ids=[device.index] if (device is not None and device.type == "cuda") else None,
                bucket_cap_mb=bucket_cap_mb, gradient_as_bucket_view=True, static_graph=True)
        else:
            self.ddp = model
        base_lr = lr * (global_batch / 512)
        params = [p for p in model.parameters() if p.requires_grad]
        kw = dict(lr=base_lr, betas=(0.9, 0.999), eps=1e-8, weight_decay=weight_decay)
        if self.graph:
            kw["capturable"] = True   # step counters on the device: replayable
        try:
            self.opt = torch.optim.AdamW(params, fused=True, **kw)
        except (RuntimeError, TypeError):
            self.opt = torch.optim.AdamW(params, foreach=True, **kw)
        self.smoothing = label_smoothing

    def _eager(self, images: torch.Tensor, labels: torch.Tensor) -> torch.Tensor:
        self.opt.zero_grad(set_to_none=True)
        if self.input_layout == "NHWC":
            logits = self.ddp(images, is_training=True)
        else:
            logits = self.ddp(images, is_training=True, layout=self.input_layout)
        loss = smoothed_cross_entropy(logits, labels, self.smoothing)
        loss.backward()
        self.opt.step()
        return loss.detach()

    def _capture(self, images: torch.Tensor, labels: torch.Tensor):
        self._images = images.clone()
        self._labels = labels.clone()
        params = [p for p in self.model.parameters() if p.requires_grad]
        snap = [p.detach().clone() for p in params]
        had_state = {id(p) for p in params if p in self.opt.state and self.opt.state[p]}
        snap_state = {id(p): {k: (v.clone() if torch.is_tensor(v) else v) for k, v in self.opt.state[p].items()}
                      for p in params if id(p) in had_state}
        s = torch.cuda.Stream(device=images.device)
        s.wait_stream(torch.cuda.current_stream(images.device))
        with torch.cuda.stream(s):   # warm-up on a side stream (allocator / library state)
            for _ in range(2):
                self._eager(self._images, self._labels)
        torch.cuda.current_stream(images.device).wait_stream(s)
        # the warm-up steps were only for the allocator and the optimizer's lazily created state:
        # put parameters and optimizer state back, so that the first call performs exactly ONE
        # update (the reference's one update per batch, train.py:94-100)
        with torch.no_grad():
            for p, v in zip(params, snap):
                p.copy_(v)
            for p in params:
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
        g = torch.cuda.CUDAGraph()
        self.opt.zero_grad(set_to_none=True)
        try:
            with torch.cuda.graph(g):
                self._loss = self._eager(self._images, self._labels)
        except RuntimeError as e:   # an op that cannot be captured: stay eager, say so once
            import sys
            print(f"[train] HIP-graph capture failed ({e}); running the eager step", file=sys.stderr)
            self.graph = False
            torch.cuda.synchronize()
            return
        self._g = g

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
        self._g.replay()
        return self._loss
