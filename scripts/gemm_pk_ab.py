#!/usr/bin/env python
"""Packed-weight persistent GEMM (SCH 3: weight fragments loaded straight into registers from the
dna_pack_frag_bf16 copy) vs the LDS-staged lean kernel (SCH 2), interleaved in one process, at
the DNABERT-2 forward / data-gradient shapes (M = b*512 tokens). Checks bit-identity first."""
import argparse
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dna_amd import _native as N  # noqa: E402

H, F = 768, 3072
# name: (rows N of the weight operand, reduction K, trans) -- dgrad packs W^T from W [K_out][N_in]
SHAPES = {"Wqkv.fwd": (3 * H, H, 0), "Wo.fwd": (H, H, 0), "Wg.fwd": (2 * F, H, 0),
          "Wwo.fwd": (H, F, 0), "Wqkv.dgrad": (H, 3 * H, 1), "Wo.dgrad": (H, H, 1),
          "Wg.dgrad": (H, 2 * F, 1), "Wwo.dgrad": (F, H, 1)}


def st():
    return torch.cuda.current_stream().cuda_stream


def timed(fn, iters):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) * 1e3 / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--M", type=int, default=262144)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--only", default="")
    a = ap.parse_args()
    torch.manual_seed(0)
    tot = {"lds": 0.0, "pk": 0.0}
    for name, (n, k, trans) in SHAPES.items():
        if a.only and a.only not in name:
            continue
        M = a.M
        x = torch.rand(M, k, device="cuda").sub_(0.5).bfloat16()
        # the operand [n][k]; for dgrad it is W^T of the stored weight W [k][n]
        w_stored = torch.rand((k, n) if trans else (n, k), device="cuda").sub_(0.5).bfloat16()
        w = w_stored.t().contiguous() if trans else w_stored
        wp = torch.empty(n * k, device="cuda", dtype=torch.bfloat16)
        N.call("dna_pack_frag_bf16", w_stored.data_ptr(), n, k, trans, wp.data_ptr(), st())
        b = torch.randn(n, device="cuda") if not trans else None
        y0 = torch.empty(M, n, device="cuda", dtype=torch.bfloat16)
        y1 = torch.empty_like(y0)
        bp = b.data_ptr() if b is not None else None
        f0 = lambda: N.call("dna_linear_fwd", x.data_ptr(), w.data_ptr(), bp, M, n, k, y0.data_ptr(), st())  # noqa
        f1 = lambda: N.call("dna_linear_fwd_pk", x.data_ptr(), w.data_ptr(), wp.data_ptr(), bp, M, n, k,  # noqa
                            y1.data_ptr(), st())
        f0()
        f1()
        torch.cuda.synchronize()
        same = bool(torch.equal(y0, y1))
        r0, r1 = [], []
        for _ in range(a.rounds):
            r0.append(timed(f0, a.iters))
            r1.append(timed(f1, a.iters))
        m0, m1 = statistics.median(r0), statistics.median(r1)
        tot["lds"] += m0
        tot["pk"] += m1
        fl = 2.0 * M * n * k
        print(f"{name:12s} M={M} bit-identical={same}  lds {m0:8.1f} us {fl / m0 / 1e6:6.0f} TF | "
              f"packed {m1:8.1f} us {fl / m1 / 1e6:6.0f} TF  ({(m0 / m1 - 1) * 100:+.1f} %)", flush=True)
        if not same:
            d = (y0.float() - y1.float()).abs()
            print("   max diff", d.max().item(), "rows with diffs", int((d.amax(1) > 0).sum()))
    print("total", {k: round(v, 1) for k, v in tot.items()})


if __name__ == "__main__":
    main()
