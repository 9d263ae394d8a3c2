#!/usr/bin/env python3
"""Host-side cost of the eager DeiT-S training step: cProfile over a few steps (the GPU runs
behind; the step is launch-bound when host time per step approaches the GPU time)."""
import cProfile
import os
import pstats
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    from sae_vision_amd import train, vit
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    model = vit.create_model("deit_s_patch16", 1000, torch.bfloat16, device=dev)
    step = train.TrainStep(model, global_batch=128, device=dev)
    g = torch.Generator(device=dev).manual_seed(1234)
    images = torch.randn(128, 224, 224, 3, device=dev, generator=g)
    labels = torch.randint(0, 1000, (128,), device=dev, generator=g)
    for _ in range(3):
        step(images, labels)
    torch.cuda.synchronize()
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(5):
        step(images, labels)
    pr.disable()
    torch.cuda.synchronize()
    st = pstats.Stats(pr)
    st.sort_stats("tottime").print_stats(35)


if __name__ == "__main__":
    main()
