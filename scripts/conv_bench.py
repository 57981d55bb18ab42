#!/usr/bin/env python
"""Causal depthwise conv (dna_causal_conv1d_fwd / _bwd) at config E's shape (Caduceus d_inner 512,
L 131072, bf16, K 4, SiLU): HIP-event time per launch and the rate over the algorithmic bytes
(fwd: x + out, bwd: x + dout + dx). Run once per library (DNA_AMD_LIB) for an A/B.

    python scripts/conv_bench.py [--B 1] [--C 512] [--L 131072] [--iters 50]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=1)
    ap.add_argument("--C", type=int, default=512)
    ap.add_argument("--L", type=int, default=131072)
    ap.add_argument("--K", type=int, default=4)
    ap.add_argument("--iters", type=int, default=50)
    a = ap.parse_args()
    from dna_amd.mamba import CausalConv1d
    dev = torch.device("cuda", 0)
    x = torch.randn(a.B, a.C, a.L, device=dev).bfloat16().requires_grad_(True)
    w = (torch.randn(a.C, 1, a.K, device=dev) * 0.5).requires_grad_(True)
    b = (torch.randn(a.C, device=dev) * 0.1).requires_grad_(True)
    dy = torch.randn(a.B, a.C, a.L, device=dev).bfloat16()
    nb = a.B * a.C * a.L * 2
    for name, fn, byt in (("fwd", lambda: CausalConv1d.apply(x, w, b, True), 2 * nb),
                          ("fwd+bwd", lambda: CausalConv1d.apply(x, w, b, True).backward(dy), 5 * nb)):
        for _ in range(5):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.iters):
            fn()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / a.iters
        print(f"{os.path.basename(os.environ.get('DNA_AMD_LIB', 'libdna_amd.so'))} {name}: "
              f"{ms * 1e3:.1f} us  {byt / ms / 1e9:.2f} TB/s (algorithmic)")


if __name__ == "__main__":
    main()
