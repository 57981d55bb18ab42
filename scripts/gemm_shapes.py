#!/usr/bin/env python
"""Every projection GEMM of the DNABERT-2 training step at the bench shape (T = b*512 tokens),
timed with HIP events: forward (dna_linear_fwd), data gradient (dna_linear_fwd on the transposed
weight, as functional.Linear runs it), weight gradient (the default wgrad path and, when built,
the hand-written one), each beside hipBLASLt (torch.mm) on the same operands. Env variants
(name=ENV=VAL,...) are interleaved in one process (rule: A/B in one process).

    python scripts/gemm_shapes.py [--batch 512] [--iters 20] [--variants 'base;order=DNA_GEMM_ORDER=1']
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dna_amd import _native as N  # noqa: E402
from dna_amd import functional as DF  # noqa: E402

H, F = 768, 3072
SHAPES = {"Wqkv": (3 * H, H), "Wo": (H, H), "Wg": (2 * F, H), "Wwo": (H, F)}


def st():
    return torch.cuda.current_stream().cuda_stream


def timeit(fn, iters):
    for _ in range(2):
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
    ap.add_argument("--batch", type=int, default=512)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--variants", default="base")
    ap.add_argument("--only", default="")
    ap.add_argument("--kinds", default="fwd,dgrad,wgrad")
    ap.add_argument("--torch", action="store_true", help="also time hipBLASLt")
    a = ap.parse_args()
    T = a.batch * 512
    torch.manual_seed(0)
    variants = []
    for v in a.variants.split(";"):
        name, *kv = v.split(",")
        env = {}
        for item in kv:
            if "=" in item:
                k, val = item.split("=", 1)
                env[k] = val
        variants.append((name.split("=")[0], env))
    ops = []
    for name, (n, k) in SHAPES.items():
        if a.only and name not in a.only.split(","):
            continue
        x = torch.randn(T, k, device="cuda").bfloat16()
        w = (torch.randn(n, k, device="cuda") * 0.05).bfloat16()
        wt = w.t().contiguous()
        b = torch.randn(n, device="cuda")
        y = torch.empty(T, n, device="cuda", dtype=torch.bfloat16)
        dy = torch.randn(T, n, device="cuda").bfloat16()
        dx = torch.empty(T, k, device="cuda", dtype=torch.bfloat16)
        g = torch.zeros(n, k, device="cuda")
        fl = 2.0 * T * n * k
        ops.append((f"{name}.fwd", fl, lambda x=x, w=w, b=b, y=y, n=n, k=k: N.call(
            "dna_linear_fwd", x.data_ptr(), w.data_ptr(), b.data_ptr(), T, n, k, y.data_ptr(), st()),
            lambda x=x, w=w, b=b: torch.addmm(b.bfloat16(), x, w.t())))
        ops.append((f"{name}.dgrad", fl, lambda dy=dy, wt=wt, dx=dx, n=n, k=k: N.call(
            "dna_linear_fwd", dy.data_ptr(), wt.data_ptr(), None, T, k, n, dx.data_ptr(), st()),
            lambda dy=dy, w=w: torch.mm(dy, w)))
        ops.append((f"{name}.wgrad", fl, lambda dy=dy, x=x, g=g: DF.wgrad_accumulate(dy, x, g),
                    lambda dy=dy, x=x: torch.mm(dy.t(), x, out_dtype=torch.float32)))
    kinds = a.kinds.split(",")
    ops = [o for o in ops if o[0].split(".")[1] in kinds]
    res = {}
    for r in range(a.rounds):
        for vname, env in variants:
            old = {k: os.environ.get(k) for k in env}
            os.environ.update(env)
            for name, fl, ours, ref in ops:
                us = timeit(ours, a.iters)
                res.setdefault((vname, name), []).append(us)
            for k, v in old.items():
                if v is None:
                    os.environ.pop(k, None)
                else:
                    os.environ[k] = v
        if a.torch:
            for name, fl, ours, ref in ops:
                res.setdefault(("hipblaslt", name), []).append(timeit(ref, a.iters))
    tot = {}
    for (vname, name), ts in sorted(res.items(), key=lambda t: (t[0][1], t[0][0])):
        fl = next(f for n_, f, _, _ in ops if n_ == name)
        us = min(ts)
        tot[vname] = tot.get(vname, 0) + us
        print(json.dumps({"variant": vname, "op": name, "us": round(us, 1),
                          "tflops": round(fl / us / 1e6, 1), "frac": round(fl / us / 1e6 / 2500, 4),
                          "all_us": [round(t, 1) for t in ts]}), flush=True)
    print(json.dumps({"total_us": {k: round(v, 1) for k, v in tot.items()}}), flush=True)


if __name__ == "__main__":
    main()
