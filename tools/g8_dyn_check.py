#!/usr/bin/env python3
"""gemm8's work-stealing tile walk (DYN) against its static walk: bitwise-equal outputs on the
multi-round shapes of the DeiT-S / ViT-B / CaiT steps (dev library, SAE_G8_DYN toggles the walk
per call: SAE_G8_DYN=1 takes the work-stealing walk), every epilogue; run back to back many times so the counter slot's reset is exercised.

    SAE_ATTN_LIB=<pkg>/libsae_attn_dev.so python tools/g8_dyn_check.py
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import sae_vision_amd.ops as ops
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    shapes = [  # (M, N, K, epilogue): multi-round gemm8 launches of the benchmark steps
        (25216, 1152, 384, ops.EPI_NONE),        # DeiT-S QKV forward (678 tiles)
        (25216, 1536, 384, ops.EPI_GELU_GRAD),   # DeiT-S FF Dense_0 + GELU (256 x 128 tiles)
        (25216, 1536, 384, ops.EPI_MUL_AUX),     # DeiT-S Dense_1 input gradient x gelu'
        (18464, 2304, 768, ops.EPI_NONE),        # ViT-B QKV forward
        (4116, 1152, 384, ops.EPI_NONE),         # CaiT-width QKV at M 4,116
    ]
    bad = 0
    for M, N, K, epi in shapes:
        a = torch.randn(M, K, device=dev, generator=g).to(torch.bfloat16)
        bt = (torch.randn(N, K, device=dev, generator=g) * 0.05).to(torch.bfloat16)
        bias = torch.randn(N, device=dev, generator=g) if epi != ops.EPI_MUL_AUX else None
        aux = torch.randn(M, N, device=dev, generator=g).to(torch.bfloat16) if epi == ops.EPI_MUL_AUX else None
        outs = {}
        for mode in ("0", "1", "1", "0", "1"):   # static, dynamic, dynamic, static, dynamic
            os.environ["SAE_G8_DYN"] = mode
            r = ops.gemm_nt(a, bt, bias, epi, aux=aux)
            r = r if isinstance(r, tuple) else (r,)
            outs.setdefault(mode, []).append([x.clone() for x in r])
        torch.cuda.synchronize()
        ref = outs["0"][0]
        same = all(torch.equal(x, y) for runs in outs.values() for run in runs for x, y in zip(run, ref))
        ref_f = (a.float() @ bt.float().t()) + (bias if bias is not None else 0)
        err = float((ref[0].float() - (ref_f if epi == ops.EPI_NONE else ref[0].float())).abs().max())
        print(f"M={M} N={N} K={K} epi={epi}: bitwise static == dynamic over 5 calls: {same}; "
              f"max |c - fp32| {err:.3g}", flush=True)
        bad += not same
    os.environ.pop("SAE_G8_DYN", None)
    print("G8_DYN_CHECK", "OK" if bad == 0 else f"FAILED {bad}")
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
