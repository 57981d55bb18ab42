#!/usr/bin/env python
"""Weight-gradient A/B at the bench shapes (b=256, M=131072 tokens): the step's split-K batched
GEMM + dna_sum_slices_accum vs one hipBLASLt GEMM with fp32 output accumulated in place
(torch.addmm(..., out_dtype=float32)). Prints per-shape times and the max difference."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dna_amd import functional as DF  # noqa: E402

M = 131072
SHAPES = {"Wqkv": (2304, 768), "Wo": (768, 768), "Wg": (6144, 768), "Wwo": (768, 3072)}


def timed(fn, iters=10):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


def main():
    torch.manual_seed(0)
    for name, (m, n) in SHAPES.items():
        dy = (torch.rand(M, m, device="cuda") - 0.5).bfloat16()
        x = (torch.rand(M, n, device="cuda") - 0.5).bfloat16()
        g1 = torch.zeros(m, n, device="cuda")
        g2 = torch.zeros(m, n, device="cuda")
        t1 = timed(lambda: DF.wgrad_accumulate(dy, x, g1))
        try:
            def f2():
                torch.addmm(g2, dy.t(), x, out_dtype=torch.float32, out=g2)
            t2 = timed(f2)
            g1.zero_(); g2.zero_()
            DF.wgrad_accumulate(dy, x, g1)
            f2()
            diff = (g1 - g2).abs().max().item() / g1.abs().max().item()
            flop = 2.0 * M * m * n
            print(f"{name:5s} split-K+sum {t1:8.1f} us {flop / t1 / 1e6:6.0f} TF | addmm fp32-out {t2:8.1f} us "
                  f"{flop / t2 / 1e6:6.0f} TF | rel diff {diff:.2e}", flush=True)
        except Exception as e:  # noqa: BLE001
            print(f"{name:5s} split-K+sum {t1:8.1f} us | addmm out_dtype failed: {str(e).splitlines()[0][:160]}", flush=True)


if __name__ == "__main__":
    main()
