#!/usr/bin/env python
"""K-sweep of csrc/gemm.hip (fwd: both operands K-major; dgrad: B stored [K][N]) against
hipBLASLt at fixed M x N, to separate the per-tile fixed cost from the main-loop rate
(time = tiles/CUs * (K/64 * t_step + t_tile)). Random uniform [-0.5, 0.5) operands."""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from scripts.gemm_bench import ours_dgrad, ours_fwd, timeit  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--M", type=int, default=65536)
    ap.add_argument("--N", type=int, default=768)
    ap.add_argument("--Ks", default="768,1536,3072,6144")
    ap.add_argument("--iters", type=int, default=15)
    ap.add_argument("--modes", default="fwd,dgrad")
    ap.add_argument("--only-ours", action="store_true")
    a = ap.parse_args()
    M, N = a.M, a.N
    for K in (int(k) for k in a.Ks.split(",")):
        fl = 2.0 * M * N * K
        for mode in a.modes.split(","):
            if mode == "fwd":
                x = torch.rand(M, K, device="cuda").sub_(0.5).bfloat16()
                w = torch.rand(N, K, device="cuda").sub_(0.5).bfloat16()
                y = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
                fo, ft = (lambda: ours_fwd(x, w, None, y)), (lambda: torch.mm(x, w.t()))
            else:  # out[M, N] = dy[M, K] . W[K, N]  (dgrad shape: W stored [K][N])
                dy = torch.rand(M, K, device="cuda").sub_(0.5).bfloat16()
                w = torch.rand(K, N, device="cuda").sub_(0.5).bfloat16()
                dx = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
                fo, ft = (lambda: ours_dgrad(dy, w, dx)), (lambda: torch.mm(dy, w))
            to = timeit(fo, a.iters)
            line = f"{mode:5s} M={M} N={N} K={K:5d} ours {to:8.1f} us {fl / to / 1e6:6.0f} TF"
            if not a.only_ours:
                tt = timeit(ft, a.iters)
                line += f" | hipBLASLt {tt:8.1f} us {fl / tt / 1e6:6.0f} TF"
            print(line, flush=True)
            del fo, ft


if __name__ == "__main__":
    main()
