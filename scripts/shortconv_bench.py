#!/usr/bin/env python
"""HyenaDNA short conv + split (dna_hyena_shortconv_fwd / _bwd) at config D's shape (B 2, L 65536,
d 256, order 2, K 3, bf16): HIP-event time per launch. For A/Bs and PMC passes.

    python scripts/shortconv_bench.py [--B 2] [--L 65536] [--d 256] [--iters 20]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=2)
    ap.add_argument("--L", type=int, default=65536)
    ap.add_argument("--d", type=int, default=256)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    from dna_amd.hyena import ShortConvSplit
    dev = torch.device("cuda", 0)
    order, K, C = 2, 3, 3 * a.d
    u = torch.randn(a.B, a.L, C, device=dev).bfloat16().requires_grad_(True)
    w = (torch.randn(C, 1, K, device=dev) * 0.5).requires_grad_(True)
    b = (torch.randn(C, device=dev) * 0.1).requires_grad_(True)
    dxs = torch.randn(a.B, order - 1, a.d, a.L, device=dev).bfloat16()
    dvx = torch.randn(a.B, a.d, a.L, device=dev).bfloat16()

    def fb():
        xs, vx = ShortConvSplit.apply(u, w, b, order, a.d)
        torch.autograd.backward((xs, vx), (dxs, dvx))
    for name, fn in (("fwd", lambda: ShortConvSplit.apply(u, w, b, order, a.d)), ("fwd+bwd", fb)):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.iters):
            fn()
        e1.record()
        torch.cuda.synchronize()
        print(f"{os.path.basename(os.environ.get('DNA_AMD_LIB', 'libdna_amd.so'))} {name}: "
              f"{e0.elapsed_time(e1) / a.iters * 1e3:.1f} us", flush=True)


if __name__ == "__main__":
    main()
