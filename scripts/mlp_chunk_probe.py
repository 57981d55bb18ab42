#!/usr/bin/env python
"""Does row-chunking the GeGLU MLP keep its intermediates in the 256 MB Infinity Cache (MALL)?

Times fwd (Wg GEMM -> dna_geglu_fwd -> Wwo GEMM) and bwd (Wwo dgrad -> dna_geglu_bwd -> Wg dgrad)
over the full b*512 rows, issued as row chunks of several sizes (GPU, HIP events)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dna_amd import _native as N  # noqa: E402

H, F = 768, 3072


def timeit(fn, iters=10):
    for _ in range(2):
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
    T = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
    torch.manual_seed(0)
    x = torch.rand(T, H, device="cuda").sub_(0.5).bfloat16()
    wg = torch.rand(2 * F, H, device="cuda").sub_(0.5).mul_(0.1).bfloat16()
    bg = torch.randn(2 * F, device="cuda").bfloat16()
    wo = torch.rand(H, F, device="cuda").sub_(0.5).mul_(0.1).bfloat16()
    bo = torch.randn(H, device="cuda").bfloat16()
    g = torch.empty(T, 2 * F, device="cuda", dtype=torch.bfloat16)
    a = torch.empty(T, F, device="cuda", dtype=torch.bfloat16)
    y = torch.empty(T, H, device="cuda", dtype=torch.bfloat16)
    dy = torch.rand(T, H, device="cuda").sub_(0.5).bfloat16()
    da = torch.empty(T, F, device="cuda", dtype=torch.bfloat16)
    dg = torch.empty(T, 2 * F, device="cuda", dtype=torch.bfloat16)
    dx = torch.empty(T, H, device="cuda", dtype=torch.bfloat16)
    st = torch.cuda.current_stream().cuda_stream

    def fwd(c, gemm2=True):
        for r0 in range(0, T, c):
            r1 = min(T, r0 + c)
            torch.addmm(bg, x[r0:r1], wg.t(), out=g[r0:r1])
            N.call("dna_geglu_fwd", g[r0:r1].data_ptr(), 1, r1 - r0, F, 0.1, 7, r0 * F, a[r0:r1].data_ptr(), st)
            if gemm2:
                torch.addmm(bo, a[r0:r1], wo.t(), out=y[r0:r1])

    def bwd(c, gemm2=True):
        for r0 in range(0, T, c):
            r1 = min(T, r0 + c)
            torch.mm(dy[r0:r1], wo, out=da[r0:r1])
            N.call("dna_geglu_bwd", da[r0:r1].data_ptr(), g[r0:r1].data_ptr(), 1, r1 - r0, F, 0.1, 7, r0 * F,
                   dg[r0:r1].data_ptr(), st)
            if gemm2:
                torch.mm(dg[r0:r1], wg, out=dx[r0:r1])

    for c in (T, 32768, 16384, 8192, 4096):
        if c > T:
            continue
        print(f"chunk {c:6d}: fwd {timeit(lambda: fwd(c)):8.1f} us  (Wg+geglu {timeit(lambda: fwd(c, False)):8.1f})"
              f"   bwd {timeit(lambda: bwd(c)):8.1f} us  (dgrad+geglu' {timeit(lambda: bwd(c, False)):8.1f})",
              flush=True)


if __name__ == "__main__":
    main()
