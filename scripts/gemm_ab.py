#!/usr/bin/env python
"""Interleaved in-process A/B of GEMM kernel variants selected by environment variables (read by
the C ABI at every launch), at the DNABERT-2 projection shapes. Random uniform [-0.5, 0.5).

  python scripts/gemm_ab.py --variants "DNA_GEMM_ROT=0;DNA_GEMM_ROT=1" --shapes fwd:2304x768
Shapes: MODE:NxK with MODE fwd (x[M,K] . W[N,K]^T) or geglu (F x K, fused GeGLU epilogue)."""
import argparse
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dna_amd import _native as N  # noqa: E402


def st():
    return torch.cuda.current_stream().cuda_stream


def timed(fn, iters=10):
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
    ap.add_argument("--M", type=int, default=131072)
    ap.add_argument("--variants", required=True, help="';'-separated, each ','-separated K=V")
    ap.add_argument("--shapes", default="fwd:2304x768,fwd:768x768,geglu:3072x768,fwd:768x3072")
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--torch", action="store_true", help="also time torch.mm (hipBLASLt)")
    a = ap.parse_args()
    variants = [dict(kv.split("=") for kv in v.split(",") if kv) for v in a.variants.split(";")]
    M = a.M
    torch.manual_seed(0)
    for shape in a.shapes.split(","):
        mode, nk = shape.split(":")
        n, k = (int(t) for t in nk.split("x"))
        x = torch.rand(M, k, device="cuda").sub_(0.5).bfloat16()
        if mode == "fwd":
            w = torch.rand(n, k, device="cuda").sub_(0.5).bfloat16()
            b = torch.randn(n, device="cuda")
            y = torch.empty(M, n, device="cuda", dtype=torch.bfloat16)
            fl = 2.0 * M * n * k
            fn = lambda: N.call("dna_linear_fwd", x.data_ptr(), w.data_ptr(), b.data_ptr(), M, n, k,  # noqa
                                y.data_ptr(), st())
            ref = lambda: torch.addmm(b.bfloat16(), x, w.t())  # noqa
        else:
            w = torch.rand(2 * n, k, device="cuda").sub_(0.5).mul_(0.1).bfloat16()
            b = torch.randn(2 * n, device="cuda")
            g = torch.empty(M, 2 * n, device="cuda", dtype=torch.bfloat16)
            out = torch.empty(M, n, device="cuda", dtype=torch.bfloat16)
            fl = 2.0 * M * 2 * n * k
            fn = lambda: N.call("dna_geglu_linear_fwd", x.data_ptr(), w.data_ptr(), b.data_ptr(), M, n,  # noqa
                                k, 0.1, 7, 3, g.data_ptr(), out.data_ptr(), st())
            ref = lambda: torch.addmm(b.bfloat16(), x, w.t())  # noqa
        res = {i: [] for i in range(len(variants) + (1 if a.torch else 0))}
        for _ in range(a.rounds):
            for i, env in enumerate(variants):
                saved = {kk: os.environ.get(kk) for kk in env}
                os.environ.update(env)
                res[i].append(timed(fn))
                for kk, vv in saved.items():
                    if vv is None:
                        os.environ.pop(kk, None)
                    else:
                        os.environ[kk] = vv
            if a.torch:
                res[len(variants)].append(timed(ref))
        names = [a.variants.split(";")[i] or "default" for i in range(len(variants))] + (["hipBLASLt"] if a.torch else [])
        line = " | ".join(f"{names[i]}: {statistics.median(v):7.1f} us {fl / statistics.median(v) / 1e6:5.0f} TF"
                          for i, v in res.items())
        print(f"{shape:16s} M={M}  {line}", flush=True)


if __name__ == "__main__":
    main()
