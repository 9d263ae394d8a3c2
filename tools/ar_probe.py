#!/usr/bin/env python3
"""All-reduce probe for the N>1 rehearsal on a 1-GPU box: times dist.all_reduce of a flat fp32
gradient-sized CUDA buffer (whole, and in buckets, sync / async) on the active backend.
usage: torchrun --nproc-per-node 2 tools/ar_probe.py [MB]"""
import os
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from sae_vision_amd import train  # noqa: E402

rank, world, local = train.init_distributed()
mb = float(sys.argv[1]) if len(sys.argv) > 1 else 88.0
n = int(mb * 2 ** 20 / 4)
x = torch.ones(n, device=f"cuda:{local}")
for label, buckets, asyn in (("whole", 1, False), ("2 buckets async", 2, True), ("4 buckets sync", 4, False)):
    step = (n + buckets - 1) // buckets
    for it in range(3):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        works = [dist.all_reduce(x[i:i + step], async_op=asyn) for i in range(0, n, step)]
        if asyn:
            for w in works:
                w.wait()
        torch.cuda.synchronize()
        if rank == 0 and it == 2:
            print(f"{dist.get_backend()} {label}: {mb:.0f} MB in {(time.perf_counter() - t0) * 1e3:.1f} ms", flush=True)
dist.destroy_process_group()
