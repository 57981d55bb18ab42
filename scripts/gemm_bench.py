#!/usr/bin/env python
"""MFMA GEMM (dna_amd/csrc/gemm.hip) vs hipBLASLt (torch.mm) at the DNABERT-2 bench shapes (GPU).

Checks every entry point against an fp32 torch reference of the same bf16 operands at a small
row count, then times ours and torch's at M = b*512 rows with HIP events."""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dna_amd import _native as N  # noqa: E402
from dna_amd.functional import wgrad_splits  # noqa: E402

H, F = 768, 3072
SHAPES = {"Wqkv": (3 * H, H), "Wo": (H, H), "Wg": (2 * F, H), "Wwo": (H, F)}


def st():
    return torch.cuda.current_stream().cuda_stream


def ours_fwd(x, w, b, y):
    N.call("dna_linear_fwd", x.data_ptr(), w.data_ptr(), b.data_ptr() if b is not None else None,
           x.shape[0], w.shape[0], w.shape[1], y.data_ptr(), st())


def ours_dgrad(dy, w, dx):
    N.call("dna_linear_dgrad", dy.data_ptr(), w.data_ptr(), dy.shape[0], w.shape[0], w.shape[1],
           dx.data_ptr(), st())


def ours_wgrad(dy, x, splits, part):
    N.call("dna_linear_wgrad", dy.data_ptr(), x.data_ptr(), dy.shape[0], dy.shape[1], x.shape[1],
           splits, part.data_ptr(), st())


def geglu_ref(g, p=0.0):
    g1, g2 = g.float().chunk(2, dim=1)
    return torch.nn.functional.gelu(g1) * g2


def rel(a, b):
    return float((a.float() - b.float()).norm() / (b.float().norm() + 1e-30))


def timeit(fn, iters):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(iters):
        e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
        e0.record()
        fn()
        e1.record()
        e1.synchronize()
        ts.append(e0.elapsed_time(e1) * 1e3)
    ts.sort()
    return ts[len(ts) // 2]


def check(M=4096):
    torch.manual_seed(0)
    ok = True
    for name, (n, k) in SHAPES.items():
        x = torch.randn(M, k, device="cuda").bfloat16()
        w = (torch.randn(n, k, device="cuda") * 0.05).bfloat16()
        b = torch.randn(n, device="cuda")
        y = torch.empty(M, n, device="cuda", dtype=torch.bfloat16)
        ours_fwd(x, w, b, y)
        ref = x.float() @ w.float().t() + b
        e1 = rel(y, ref)
        dy = torch.randn(M, n, device="cuda").bfloat16()
        dx = torch.empty(M, k, device="cuda", dtype=torch.bfloat16)
        ours_dgrad(dy, w, dx)
        e2 = rel(dx, dy.float() @ w.float())
        s = 4
        part = torch.empty(s, n, k, device="cuda")
        ours_wgrad(dy, x, s, part)
        e3 = rel(part.sum(0), dy.float().t() @ x.float())
        sp = N.lib().dna_linear_wgrad_p_splits(M, n, k)
        partp = torch.empty(sp, n, k, device="cuda")
        N.call("dna_linear_wgrad_p", dy.data_ptr(), x.data_ptr(), M, n, k, sp, partp.data_ptr(), st())
        e4 = rel(partp.sum(0), dy.float().t() @ x.float())
        print(f"check {name}: wgrad_p (s={sp}) {e4:.2e}", flush=True)
        ok &= e4 < 1e-5
        print(f"check {name}: fwd {e1:.2e} dgrad {e2:.2e} wgrad {e3:.2e}", flush=True)
        ok &= max(e1, e2) < 1e-2 and e3 < 1e-5
    # odd M (tail rows)
    x = torch.randn(1000, H, device="cuda").bfloat16()
    w = (torch.randn(H, H, device="cuda") * 0.05).bfloat16()
    y = torch.empty(1000, H, device="cuda", dtype=torch.bfloat16)
    ours_fwd(x, w, None, y)
    e = rel(y, x.float() @ w.float().t())
    print(f"check tail M=1000: {e:.2e}", flush=True)
    ok &= e < 1e-2
    # the fused GeGLU epilogues: tests/test_gpu_kernels.py (fused == unfused bit for bit)
    print("CHECK", "PASS" if ok else "FAIL", flush=True)
    return ok


def bench(M, iters):
    torch.manual_seed(0)
    tot_o = tot_t = 0.0
    for name, (n, k) in SHAPES.items():
        x = torch.rand(M, k, device="cuda").sub_(0.5).bfloat16()
        w = torch.rand(n, k, device="cuda").sub_(0.5).bfloat16()
        b = torch.randn(n, device="cuda")
        y = torch.empty(M, n, device="cuda", dtype=torch.bfloat16)
        dy = torch.rand(M, n, device="cuda").sub_(0.5).bfloat16()
        dx = torch.empty(M, k, device="cuda", dtype=torch.bfloat16)
        fl = 2.0 * M * n * k
        s = wgrad_splits(M, n, k)
        part = torch.empty(s, n, k, device="cuda")
        sp = N.lib().dna_linear_wgrad_p_splits(M, n, k)
        partp = torch.empty(sp, n, k, device="cuda")
        bb = b.bfloat16()
        rows = [
            ("fwd", lambda: ours_fwd(x, w, b, y), lambda: torch.addmm(bb, x, w.t())),
            ("dgrad", lambda: ours_dgrad(dy, w, dx), lambda: torch.mm(dy, w)),
            (f"wgradP/s{sp}", lambda: N.call("dna_linear_wgrad_p", dy.data_ptr(), x.data_ptr(), M, n, k, sp,
                                            partp.data_ptr(), st()),
             lambda: torch.bmm(dy.view(s, M // s, n).transpose(1, 2), x.view(s, M // s, k),
                               out_dtype=torch.float32)),
            (f"wgrad/s{s}", lambda: ours_wgrad(dy, x, s, part),
             lambda: torch.bmm(dy.view(s, M // s, n).transpose(1, 2), x.view(s, M // s, k),
                               out_dtype=torch.float32)),
        ]
        for tag, fo, ft in rows:
            to = timeit(fo, iters)
            tt = timeit(ft, iters)
            tot_o += to
            tot_t += tt
            print(f"{name:5s} {tag:9s} ours {to:7.1f} us {fl / to / 1e6:6.0f} TF | hipBLASLt {tt:7.1f} us "
                  f"{fl / tt / 1e6:6.0f} TF", flush=True)
    # fused GeGLU
    x = torch.rand(M, H, device="cuda").sub_(0.5).bfloat16()
    wg = torch.rand(2 * F, H, device="cuda").sub_(0.5).mul_(0.1).bfloat16()
    bg = torch.randn(2 * F, device="cuda")
    g = torch.empty(M, 2 * F, device="cuda", dtype=torch.bfloat16)
    a = torch.empty(M, F, device="cuda", dtype=torch.bfloat16)
    fo = lambda: N.call("dna_geglu_linear_fwd", x.data_ptr(), wg.data_ptr(), bg.data_ptr(), M, F, H,  # noqa
                        0.1, 7, 3, g.data_ptr(), a.data_ptr(), st())
    fl = 2.0 * M * 2 * F * H
    to = timeit(fo, iters)
    print(f"Wg+GeGLU fused fwd  ours {to:7.1f} us {fl / to / 1e6:6.0f} TF", flush=True)
    dy = torch.rand(M, H, device="cuda").sub_(0.5).bfloat16()
    wo = torch.rand(H, F, device="cuda").sub_(0.5).mul_(0.1).bfloat16()
    dg = torch.empty(M, 2 * F, device="cuda", dtype=torch.bfloat16)
    fo = lambda: N.call("dna_geglu_linear_dgrad", dy.data_ptr(), wo.data_ptr(), g.data_ptr(), M, F, H,  # noqa
                        dg.data_ptr(), st())
    fl = 2.0 * M * F * H
    to = timeit(fo, iters)
    print(f"Wwo dgrad+GeGLU bwd ours {to:7.1f} us {fl / to / 1e6:6.0f} TF", flush=True)
    print(f"TOTAL plain GEMMs: ours {tot_o:.0f} us, hipBLASLt {tot_t:.0f} us", flush=True)


def only(M, iters, name, tag):
    n, k = SHAPES[name]
    x = torch.rand(M, k, device="cuda").sub_(0.5).bfloat16()
    w = torch.rand(n, k, device="cuda").sub_(0.5).bfloat16()
    y = torch.empty(M, n, device="cuda", dtype=torch.bfloat16)
    dy = torch.rand(M, n, device="cuda").sub_(0.5).bfloat16()
    dx = torch.empty(M, k, device="cuda", dtype=torch.bfloat16)
    s = wgrad_splits(M, n, k)
    part = torch.empty(s, n, k, device="cuda")
    sp = N.lib().dna_linear_wgrad_p_splits(M, n, k)
    partp = torch.empty(sp, n, k, device="cuda")
    fn = {"fwd": lambda: ours_fwd(x, w, None, y), "dgrad": lambda: ours_dgrad(dy, w, dx),
          "wgrad": lambda: ours_wgrad(dy, x, s, part),
          "wgradp": lambda: N.call("dna_linear_wgrad_p", dy.data_ptr(), x.data_ptr(), M, n, k, sp,
                                   partp.data_ptr(), st())}[tag]
    t = timeit(fn, iters)
    print(f"{name} {tag}: {t:.1f} us {2.0 * M * n * k / t / 1e6:.0f} TF", flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--M", type=int, default=65536)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--no-check", action="store_true")
    ap.add_argument("--only", default="", help="NAME:fwd|dgrad|wgrad -- run just our kernel (profiling)")
    a = ap.parse_args()
    if a.only:
        only(a.M, a.iters, *a.only.split(":"))
        return
    if not a.no_check and not check():
        sys.exit(1)
    bench(a.M, a.iters)


if __name__ == "__main__":
    main()
