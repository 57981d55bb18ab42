#!/usr/bin/env python
"""hipBLASLt weight-gradient sweep at the bench shape (GPU): dW[n,k] = dy[M,n]^T x[M,k] as one
fp32-output GEMM (s=1, the library's own split/stream-K) and as s-way split-K batched GEMMs
(fp32 or bf16 partials) + the sum, for the four DNABERT-2 projection shapes."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from scripts.gemm_bench import SHAPES, timeit  # noqa: E402


def main(M=131072, iters=10):
    torch.manual_seed(0)
    for name, (n, k) in SHAPES.items():
        dy = torch.rand(M, n, device="cuda").sub_(0.5).bfloat16()
        x = torch.rand(M, k, device="cuda").sub_(0.5).bfloat16()
        fl = 2.0 * M * n * k
        res = []
        t = timeit(lambda: torch.mm(dy.t(), x, out_dtype=torch.float32), iters)
        res.append(f"s1:{t:.0f}")
        for s in (4, 8, 16, 32, 64):
            a = dy.view(s, M // s, n).transpose(1, 2)
            b = x.view(s, M // s, k)
            t32 = timeit(lambda: torch.bmm(a, b, out_dtype=torch.float32).sum(0), iters)
            t16 = timeit(lambda: torch.bmm(a, b).float().sum(0), iters)
            res.append(f"s{s}:{t32:.0f}/{t16:.0f}")
        best = min(float(r.split(":")[1].split("/")[0]) for r in res)
        print(f"{name:5s} n={n} k={k}  (us; s: fp32-part/bf16-part incl. sum)  " + "  ".join(res) +
              f"  best {fl / best / 1e6:.0f} TF", flush=True)


if __name__ == "__main__":
    main()
