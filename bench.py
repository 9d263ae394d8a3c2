#!/usr/bin/env python3
"""Benchmark: DeiT-S/16 224px bf16 data-parallel training on MI355X (BASELINE.json configs[1]
at N=1; the same per-GPU workload at N>1, weak scaling) with the fused HIP attention on the hot path.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    torchrun --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N ...

One process per GPU; each rank holds 128 synthetic N(0,1) images (fed as the reference's train step
receives them: HWCN fp32, train.py:80-81) + uniform labels, resident in HBM.  The step is forward,
smoothed cross-entropy, backward and AdamW, replayed as ONE HIP graph (train.TrainStep): every
gradient is written in place into a flat fp32 buffer, and at N>1 each ~25 MB bucket of it is
all-reduced on RCCL (backend nccl) on a communication stream as soon as its last gradient is
written, inside the captured backward (overlapped with the rest of it; the compute stream joins
before AdamW).  ``--world1-rccl`` runs that collective path at N=1 with a one-rank RCCL group;
``--two-graphs`` puts the all-reduce between a forward+backward graph and an AdamW graph;
``--eager`` launches the step op by op.  W untimed warm-up steps, then exactly K steps bracketed
by a barrier + device synchronisation on both sides; the max elapsed time over ranks is used.
Rank 0 prints ONE JSON line:
  value        = whole-job training images/s (all ranks)
  roofline     = the fused attention op of this workload: one call = 2 launches (attn_fwd2 +
                 the single-pass attn_bwd3 at DeiT-S), timed with HIP events on the launch stream
                 around a HIP graph of 10 back-to-back calls at the workload's layer shape (packed
                 [B, N, 3, H, D] q/k/v), median of 20 replays, after the timed region (events
                 inside a captured step cannot be read); algorithmic FLOPs / bytes per call
                 (DESIGN.md §4); traffic = HBM bytes per call from profiles/pmc_traffic.json
                 (rocprofv3 PMC, gfx950 FETCH_SIZE correction)
  cpu_baseline = the numpy port (oracle/vit_ref.py) of the same training step on a bounded
                 sample, on this host's cores (rank 0, N=1 only); .configs0 = BASELINE configs[0]
                 (DeiT-Ti forward + loss, batch 8); .attention = the unfused attention core fwd+bwd
                 as C + OpenMP (oracle/attn_cpu.c), TFLOP/s
  attention_headline = the fused fwd+bwd core alone at ViT-B/16@384 shape (B=64, N=577, H=12,
                 D=64), TFLOP/s and fraction of the 2.5 PF bf16 MFMA peak (N>=577 target), timed
                 on HIP graphs of back-to-back launches (no host gaps)
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "attention fwd+bwd TFLOP/s (% MFMA peak); DeiT-S/16 train img/s at 1/8 GPUs"
PEAK_BF16_TFLOPS = 2500.0     # MI355X_MICROARCH.md: dense bf16 MFMA
PEAK_F32_TFLOPS = 157.3       # MI355X_MICROARCH.md: dense fp32 MFMA
PEAK_HBM_GBS = 8000.0         # MI355X_MICROARCH.md: HBM3E spec
TIMER_STEPS = 3               # graph mode: eager steps timed with HIP events after the timed region
RIDGE = PEAK_BF16_TFLOPS * 1e12 / (PEAK_HBM_GBS * 1e9)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def attn_work(B, Nq, Nk, H, D, elt=2):
    """Algorithmic FLOPs / HBM bytes of one fused attention call."""
    f_fwd = 4.0 * B * H * Nq * Nk * D
    f_bwd = 8.0 * B * H * Nq * Nk * D
    b_fwd = elt * B * H * D * (2 * Nq + 2 * Nk) + 4.0 * B * H * Nq
    b_bwd = elt * B * H * D * (4 * Nq + 4 * Nk) + 8.0 * B * H * Nq
    return f_fwd, f_bwd, b_fwd, b_bwd


def roofline_entry(flops, nbytes, seconds, traffic=None, bound=None):
    ai = flops / nbytes
    if bound == "mfma" or (bound is None and ai >= RIDGE):
        ach, peak, unit, bound = flops / seconds / 1e12, PEAK_BF16_TFLOPS, "TFLOP/s", "mfma"
    else:
        ach, peak, unit, bound = nbytes / seconds / 1e9, PEAK_HBM_GBS, "GB/s", "hbm"
    return {"bound": bound, "achieved": round(ach, 2), "peak": peak, "unit": unit, "frac": round(ach / peak, 4),
            "traffic": traffic, "algorithmic_flops": flops, "algorithmic_bytes": nbytes,
            "arith_intensity": round(ai, 1), "tflops": round(flops / seconds / 1e12, 2),
            "gbs": round(nbytes / seconds / 1e9, 1), "ms_per_call": round(seconds * 1e3, 4)}


def load_pmc(name, key):
    """A per-call figure from the committed rocprofv3 PMC summary (profiles/pmc_traffic.json,
    tools/pmc_traffic.py), or None."""
    p = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(p) as f:
            return json.load(f).get(name, {}).get(key)
    except (OSError, ValueError):
        return None


def load_traffic(name):
    """HBM bytes per call (FETCH_SIZE / WRITE_SIZE, gfx950-corrected), or None."""
    return load_pmc(name, "hbm_bytes_per_call")


def cpu_baseline(model_name, seconds_budget=15.0):
    """numpy port of the training step (oracle/vit_ref.py) on a bounded sample."""
    import numpy as np
    import torch
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import vit_ref
    from sae_vision_amd import vit
    L, H, C, p = vit.MODEL_CONFIGS[model_name]
    cpu_model = vit.create_model(model_name, 1000, torch.float32, device="cpu")
    params = {k: v.detach().numpy().astype(np.float32).copy() for k, v in cpu_model.named_parameters()}
    rng = np.random.default_rng(0)
    bs = 2
    images = rng.standard_normal((bs, 224, 224, 3)).astype(np.float32)
    labels = rng.integers(0, 1000, size=bs)
    state = {}
    try:
        from threadpoolctl import threadpool_info
        cores = max([i.get("num_threads", 1) for i in threadpool_info()] or [1])
    except Exception:
        cores = len(os.sched_getaffinity(0))
    n_img, t0 = 0, time.perf_counter()
    while True:
        _, _, grads = vit_ref.vit_loss_and_grads(params, images, labels, L, H, p)
        vit_ref.adam_update(params, grads, state)
        n_img += bs
        if time.perf_counter() - t0 > seconds_budget or n_img >= 16:
            break
    dt = time.perf_counter() - t0
    out = {"value": round(n_img / dt, 3), "unit": "img/s", "cores": int(cores), "kind": "port",
           "affinity_cpus": len(os.sched_getaffinity(0)), "cores_note": CORES_NOTE,
           "sample": f"{model_name} fp32 numpy train step (fwd+loss+bwd+AdamW), batch {bs} x {n_img // bs} steps, "
                     f"{dt:.1f} s"}
    # BASELINE configs[0]: DeiT-Tiny/16 forward + loss on a 224 px batch of 8, the CPU reference path
    Lt, Ht, Ct, pt = vit.MODEL_CONFIGS["deit_ti_patch16"]
    ti = vit.create_model("deit_ti_patch16", 1000, torch.float32, device="cpu")
    pti = {k: v.detach().numpy().astype(np.float32).copy() for k, v in ti.named_parameters()}
    im8 = rng.standard_normal((8, 224, 224, 3)).astype(np.float32)
    lb8 = rng.integers(0, 1000, size=8)
    vit_ref.vit_loss(pti, im8, lb8, Lt, pt)   # warm-up (allocations, BLAS thread pool)
    n, t1 = 0, time.perf_counter()
    while n < 3 and time.perf_counter() - t1 < seconds_budget / 3:
        vit_ref.vit_loss(pti, im8, lb8, Lt, pt)
        n += 1
    d1 = (time.perf_counter() - t1) / n
    out["configs0"] = {"value": round(8 / d1, 3), "unit": "img/s", "ms_per_batch": round(d1 * 1e3, 1),
                       "cores": int(cores), "affinity_cpus": len(os.sched_getaffinity(0)), "kind": "port",
                       "sample": f"deit_ti_patch16 224px fp32 numpy forward+loss, batch 8 x {n}"}
    out["attention"] = cpu_attention_baseline(seconds_budget / 3)
    return out


# why `cores` is below `affinity_cpus`: the GPU box gives one GPU's job a 16-CPU share of the host
# (OMP_NUM_THREADS / MAX_JOBS are set to 16 there and worker pools must stay within it); the
# affinity mask still lists every CPU of the 8-GPU machine, which the other GPUs' jobs use
CORES_NOTE = ("threads = OMP_NUM_THREADS, the box's CPU share for one GPU (16 of the machine's CPUs; "
              "affinity_cpus counts all of them, shared with the other GPUs' jobs)")


def cpu_attention_baseline(seconds_budget=5.0, B=16, N=197, H=6, D=64):
    """SURVEY §8d's CPU baseline of metric (1): the unfused reference attention core (S and P
    materialised, softmax, AV; backward through dP / dS) as C + OpenMP over (batch, head), fp32
    (oracle/attn_cpu.c), fwd + bwd on a DeiT-S-shaped sample, TFLOP/s by the same algorithmic count
    as the GPU line (12 B H N^2 D)."""
    import numpy as np
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import attn_cpu
    rng = np.random.default_rng(0)
    q, k, v, do = (rng.standard_normal((B, N, H, D)).astype(np.float32) for _ in range(4))
    o, lse = attn_cpu.attn_fwd(q, k, v)   # warm-up (thread pool, page faults)
    n, t0 = 0, time.perf_counter()
    while n < 1 or time.perf_counter() - t0 < seconds_budget:
        o, lse = attn_cpu.attn_fwd(q, k, v)
        attn_cpu.attn_bwd(q, k, v, o, lse, do)
        n += 1
    dt = (time.perf_counter() - t0) / n
    f_fwd, f_bwd, _, _ = attn_work(B, N, N, H, D)
    return {"value": round((f_fwd + f_bwd) / dt / 1e12, 5), "unit": "TFLOP/s", "ms_per_call": round(dt * 1e3, 2),
            "cores": attn_cpu.threads(), "affinity_cpus": len(os.sched_getaffinity(0)), "cores_note": CORES_NOTE,
            "kind": "port",
            "sample": f"unfused fp32 attention core fwd+bwd (C + OpenMP, oracle/attn_cpu.c), B={B} N={N} H={H} "
                      f"D={D}, {n} calls"}


def attn_graph_ms(dev, B, N, H, D, dt, iters=20, reps=10):
    """Kernel time of one fused attention fwd and one bwd call at [B, N, H, D] (packed [B, N, 3, H, D]
    q/k/v as the models feed it): each captured as a HIP graph of `reps` back-to-back C-ABI
    launches, HIP events around each replay on the replay stream, median over `iters` replays.
    No host gaps inside a replay, so the per-launch time is the kernels' own (what rocprofv3's
    kernel trace reports for the same launches)."""
    import math
    import torch
    import sae_vision_amd.ops as ops
    g = torch.Generator(device=dev).manual_seed(0)
    qkv = torch.randn(B, N, 3, H, D, device=dev, generator=g).to(dt)
    do = torch.randn(B, N, H, D, device=dev, generator=g).to(dt)
    dqkv = torch.empty_like(qkv)
    sc = 1.0 / math.sqrt(D)
    q, k, v = qkv[:, :, 0], qkv[:, :, 1], qkv[:, :, 2]
    o, lse = ops._fwd(q, k, v, sc)
    bwd = lambda: ops._bwd(q, k, v, o, lse, do, dqkv[:, :, 0], dqkv[:, :, 1], dqkv[:, :, 2], sc)
    side = torch.cuda.Stream(dev)
    side.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(side):
        for _ in range(3):
            ops._fwd(q, k, v, sc)
            bwd()
    torch.cuda.current_stream(dev).wait_stream(side)
    gf, gb = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
    with torch.cuda.graph(gf):
        for _ in range(reps):
            ops._fwd(q, k, v, sc)
    with torch.cuda.graph(gb):
        for _ in range(reps):
            bwd()
    tf, tb = [], []
    for _ in range(iters):
        e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
        e[0].record()
        gf.replay()
        e[1].record()
        gb.replay()
        e[2].record()
        torch.cuda.synchronize()
        tf.append(e[0].elapsed_time(e[1]) / reps)
        tb.append(e[1].elapsed_time(e[2]) / reps)
    return sorted(tf)[iters // 2], sorted(tb)[iters // 2]


def headline(dev, iters=20, reps=10, f32=False):
    """Fused attention fwd+bwd alone at the ViT-B/16@384 shape, timed by attn_graph_ms.
    f32: the fp32 kernels (v_mfma_f32_32x32x2_f32) at batch 16 against the 157.3 TF fp32 MFMA peak."""
    import torch
    B, N, H, D = (16 if f32 else 64), 577, 12, 64
    dt = torch.float32 if f32 else torch.bfloat16
    fwd_ms, bwd_ms = attn_graph_ms(dev, B, N, H, D, dt, iters, reps)
    f_fwd, f_bwd, b_fwd, b_bwd = attn_work(B, N, N, H, D, elt=4 if f32 else 2)
    sec = (fwd_ms + bwd_ms) / 1e3
    peak = PEAK_F32_TFLOPS if f32 else PEAK_BF16_TFLOPS
    if f32:
        tf = (f_fwd + f_bwd) / sec / 1e12
        return {"shape": {"B": B, "N": N, "H": H, "D": D}, "dtype": "f32", "fwd_ms": round(fwd_ms, 4),
                "bwd_ms": round(bwd_ms, 4), "tflops": round(tf, 2), "peak": PEAK_F32_TFLOPS,
                "frac_mfma_peak": round(tf / peak, 4), "timing": f"HIP graphs of {reps} launches, median of {iters}"}
    # BASELINE states the N >= 577 target against the bf16 MFMA peak (AI 286 sits at the ridge)
    r = roofline_entry(f_fwd + f_bwd, b_fwd + b_bwd, sec, load_traffic("vitb384"), bound="mfma")
    busy = load_pmc("vitb384", "mfma_busy_frac")
    if busy is not None:
        r["mfma_busy_frac"] = busy
    return {"shape": {"B": B, "N": N, "H": H, "D": D}, "fwd_ms": round(fwd_ms, 4), "bwd_ms": round(bwd_ms, 4),
            "fwd_tflops": round(f_fwd / fwd_ms / 1e9, 1), "bwd_tflops": round(f_bwd / bwd_ms / 1e9, 1),
            "tflops": r["tflops"], "frac_mfma_peak": round(r["tflops"] / PEAK_BF16_TFLOPS, 4),
            "timing": f"HIP graphs of {reps} launches, median of {iters} replays", "roofline": r}


def step_label(step, use_graph):
    """What the timed step ran, named by the collective path that actually executed (train.py)."""
    if not (use_graph and step.graph):
        base = "eager"
    elif step.two_graphs:
        base = "hip_graphs(fwd+bwd, adamw)"
    else:
        base = "hip_graph_replay"
    coll = {"none": "no collective", "overlap": "rccl_allreduce overlapped with the backward",
            "between": "rccl_allreduce between the graphs", "host": "gloo host all-reduce between the graphs"}
    if getattr(step, "_flagged", False) and use_graph and step.graph:
        return f"{base} + rccl_allreduce per bucket on the comm stream, gated by device flags the backward sets"
    return f"{base} + {coll[step.collective]}"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--batch", type=int, default=128, help="images per GPU")
    ap.add_argument("--model", default="deit_s_patch16",
                    help="ViT/DeiT (vit.MODEL_CONFIGS) or CaiT (cait.CAIT_CONFIGS, e.g. cait_s_24: configs[4])")
    ap.add_argument("--img-size", type=int, default=224,
                    help="input resolution (384 with --model vit_b_patch16 --batch 32: BASELINE configs[2])")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-headline", action="store_true")
    ap.add_argument("--profile", action="store_true", help="training loop only (for rocprofv3 runs)")
    ap.add_argument("--eager", action="store_true", help="N=1: eager step instead of the HIP-graph replay")
    ap.add_argument("--two-graphs", action="store_true",
                    help="N=1: the multi-rank step structure (forward+backward graph, the all-reduce point, AdamW "
                         "graph) without the collective, to rehearse the N > 1 step's GPU time")
    ap.add_argument("--no-flat-grads", action="store_true",
                    help="autograd's per-parameter gradients and torch's fused AdamW (the round-1 step) instead of "
                         "the flat gradient buffer, in-place gradient sinks and the one-launch AdamW")
    ap.add_argument("--input-layout", default="HWCN", choices=["HWCN", "NHWC"],
                    help="HWCN: the reference's train-step feed [H, W, C, N] fp32 (train.py:80-81, "
                         "input_pipeline.py:187-191), gathered by the fused patch GEMM; NHWC: the model call")
    ap.add_argument("--no-grad-sinks", action="store_true",
                    help="flat gradient buffer without the in-place gradient sinks (autograd adds into it)")
    ap.add_argument("--world1-rccl", action="store_true",
                    help="N=1: a one-rank RCCL process group, so the overlapped bucket all-reduces run (captured "
                         "in the step's HIP graph) as they do at N > 1")
    ap.add_argument("--bucket-mb", type=float, default=25.0, help="gradient all-reduce bucket size")
    ap.add_argument("--no-persistent-casts", action="store_true",
                    help="cast every Dense kernel to bf16 at the start of each forward instead of the optimizer "
                         "writing the bf16 copies in its update")
    ap.add_argument("--emulate-rccl", default="",
                    help="CHANNELS,BUSBW_GBPS,WORLD: one-GPU contention emulation of a WORLD-GPU node -- beside "
                         "each bucket's all-reduce, CHANNELS workgroups hold CUs for the bucket's ring time at "
                         "BUSBW_GBPS (implies --world1-rccl; a diagnostic, never the bench line)")
    args = ap.parse_args()
    if args.emulate_rccl:
        os.environ["SAE_EMULATE_RCCL"] = args.emulate_rccl
        args.world1_rccl = True
    if args.world1_rccl:
        os.environ["SAE_WORLD1_RCCL"] = "1"
    # stdout carries exactly ONE line, the JSON result: everything else written to fd 1 by the
    # libraries underneath (RCCL prints its version banner at communicator creation) goes to stderr
    sys.stdout.flush()
    out_fd = os.dup(1)
    os.dup2(2, 1)

    import torch
    import torch.distributed as dist
    import sae_vision_amd
    from sae_vision_amd import cait, ops, train, vit

    rank, world, local = train.init_distributed()
    if world != args.gpus:
        log(f"[bench] note: --gpus {args.gpus} but WORLD_SIZE={world}; using {world}")
    dev = torch.device("cuda", local)
    sae_vision_amd.load_library()

    torch.manual_seed(0)
    is_cait = args.model in cait.CAIT_CONFIGS
    if is_cait:   # BASELINE configs[4]; stochastic depth at its config rate (a real training step)
        model = cait.create_cait(args.model, 1000, torch.bfloat16, img_size=args.img_size, device=dev)
    else:
        model = vit.create_model(args.model, 1000, torch.bfloat16, img_size=args.img_size, device=dev)
    B = args.batch
    # the whole step (forward, loss, backward with the overlapped bucket all-reduces at N > 1, AdamW)
    # replayed as one HIP graph
    use_graph = not args.eager
    step = train.TrainStep(model, global_batch=B * world, device=dev, graph=use_graph, input_layout=args.input_layout,
                           flat_grads=False if args.no_flat_grads else None, grad_sinks=not args.no_grad_sinks,
                           two_graphs=True if args.two_graphs else None, bucket_cap_mb=args.bucket_mb,
                           persistent_casts=not args.no_persistent_casts)
    g = torch.Generator(device=dev).manual_seed(1234 + rank)
    images = torch.randn(B, args.img_size, args.img_size, 3, device=dev, generator=g)
    if args.input_layout == "HWCN":
        images = images.permute(1, 2, 3, 0).contiguous()
    labels = torch.randint(0, 1000, (B,), device=dev, generator=g)

    for _ in range(args.warmup):
        step(images, labels)
    # the synthetic batch lives in the step graph's static input buffers (as a loader writing each
    # batch there would put it), so a replay reads it in place instead of copying it in first
    bufs = step.input_buffers()
    if bufs is not None:
        images, labels = bufs
    torch.cuda.synchronize()
    timer = ops.KernelTimer()
    if not use_graph:   # eager launches: the attention events sit inside the timed region
        ops.set_kernel_timer(timer)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    host = 0.0
    for _ in range(args.steps):
        h0 = time.perf_counter()
        loss = step(images, labels)
        host += time.perf_counter() - h0
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    ops.set_kernel_timer(None)
    if use_graph:
        # graph replays carry no host-side events: time the same kernels with HIP events on their
        # launch stream over eager steps of the same workload, right after the timed region
        ops.set_kernel_timer(timer)
        for _ in range(TIMER_STEPS):
            step._eager(images, labels)
        ops.set_kernel_timer(None)
    if world > 1:
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    final_loss = float(loss.item())

    ksum = timer.summary()
    timed_steps = TIMER_STEPS if use_graph else args.steps
    if is_cait:   # the dominant attention: the talking-heads self-attention trunk (no CLS token)
        L, _, Hh, C, _, _ = cait.CAIT_CONFIGS[args.model]
        N = (args.img_size // 16) ** 2
        kf, kb = "th_attn_fwd", "th_attn_bwd"
    else:
        L, Hh, C, p = vit.MODEL_CONFIGS[args.model]
        N = (args.img_size // p) ** 2 + 1
        kf, kb = "attn_fwd", "attn_bwd"
    D = C // Hh
    f_fwd, f_bwd, b_fwd, b_bwd = attn_work(B, N, N, Hh, D)
    if is_cait:   # + the two H x H head mixes, fwd and bwd
        f_fwd += 2 * 2.0 * B * Hh * Hh * N * N
        f_bwd += 2 * 4.0 * B * Hh * Hh * N * N
    ev_fwd_ms, ev_bwd_ms = ksum[kf]["mean_ms"], ksum[kb]["mean_ms"]
    if is_cait:   # the talking-heads op: HIP events around its launches in the eager steps
        fwd_ms, bwd_ms, how = ev_fwd_ms, ev_bwd_ms, "HIP events around each launch, eager steps after the timed region"
    else:         # the same kernels at the workload's layer shape, replayed from a HIP graph
        fwd_ms, bwd_ms = attn_graph_ms(dev, B, N, Hh, D, torch.bfloat16)
        how = ("the workload's attention call ([B, N, 3, H, D] packed q/k/v) as a HIP graph of 10 launches "
               "after the timed region, median of 20 replays (kernel time, as rocprofv3 reports it)")
    is_deit_s = (args.model, args.img_size, B) == ("deit_s_patch16", 224, 128)
    roof = roofline_entry(f_fwd + f_bwd, b_fwd + b_bwd, (fwd_ms + bwd_ms) / 1e3,
                          load_traffic("deit_s") if is_deit_s else None)
    roof["timing"] = how
    roof["eager_step_events_ms_per_call"] = round(ev_fwd_ms + ev_bwd_ms, 4)
    if is_deit_s and load_pmc("deit_s", "mfma_busy_frac") is not None:
        roof["mfma_busy_frac"] = load_pmc("deit_s", "mfma_busy_frac")
    img_s = B * world * args.steps / elapsed
    flop_img = 3 * (cait.cait_flops_per_image(args.model, args.img_size) if is_cait
                    else vit.vit_flops_per_image(args.model, args.img_size))

    if rank != 0:
        if world > 1:
            dist.barrier()
        step.close()   # the graph's RCCL resources go before the communicator does
        dist.destroy_process_group()
        return
    out = {
        "metric": METRIC, "value": round(img_s, 2), "unit": "img/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 3), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "bf16", "data": "synthetic",
        "config": {"workload": f"{args.model} {args.img_size}px bf16 data-parallel training step (fused attention fwd+bwd)",
                   "model": args.model, "global_batch": B * world, "per_gpu_batch": B, "seq_len": N,
                   "heads": Hh, "head_dim": D, "layers": L, "parallelism": f"dp{world}",
                   "input": f"{args.input_layout} fp32 images (patch gather fused into the embedding GEMM)",
                   # what actually ran: a capture that failed leaves the step eager (train.py)
                   "step": step_label(step, use_graph),
                   "collective": {"mode": step.collective, "process_group": dist.get_backend() if step.pg else None,
                                  "emulated_rccl": args.emulate_rccl or None,
                                  "buckets": len(getattr(step, "_buckets", [])), "bucket_cap_mb": args.bucket_mb}},
        "host_submit_ms_per_step": round(host / args.steps * 1e3, 3),
        "roofline": roof,
        "attention": {"kernel": kf.replace("_fwd", ""), "calls_per_step": ksum[kf]["launches"] // timed_steps,
                      "fwd_ms": round(fwd_ms, 4), "bwd_ms": round(bwd_ms, 4), "tflops": roof["tflops"],
                      "share_of_step": round((fwd_ms + bwd_ms) * ksum[kf]["launches"] / timed_steps
                                             / (elapsed / args.steps * 1e3), 4)},
        "e2e": {"train_flop_per_img": flop_img, "tflops": round(img_s * flop_img / 1e12, 1),
                "mfma_frac": round(img_s * flop_img / 1e12 / (world * PEAK_BF16_TFLOPS), 4),
                "final_loss": round(final_loss, 4)},
    }
    if not args.profile and not args.no_headline:
        out["attention_headline"] = headline(dev)
        out["attention_headline_f32"] = headline(dev, iters=5, reps=3, f32=True)
    if not args.profile and not args.no_cpu_baseline and world == 1 and args.img_size == 224 and not is_cait:
        out["cpu_baseline"] = cpu_baseline(args.model)
    os.write(out_fd, (json.dumps(out) + "\n").encode())
    if world > 1:
        dist.barrier()
    step.close()   # the graph's RCCL resources go before the communicator does
    if dist.is_initialized():
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
