#!/usr/bin/env python
"""Selective-scan micro-benchmark at BASELINE config E scale (Caduceus: d_inner = 2*d_model = 512,
d_state 16, L = 131072), GPU, HIP events. Algorithmic bytes: fwd reads u, delta, z [B,D,L] and
B, C [B,N,L], writes out [B,D,L]; bwd additionally reads dout, writes du, ddelta, dz and
accumulates dB, dC (fp32). HBM roofline 8 TB/s."""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dna_amd.mamba import selective_scan_fn  # noqa: E402


def timeit(fn, iters):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(iters):
        a, b = torch.cuda.Event(True), torch.cuda.Event(True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b) * 1e3)
    ts.sort()
    return ts[len(ts) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=2)
    ap.add_argument("--D", type=int, default=512)
    ap.add_argument("--L", type=int, default=131072)
    ap.add_argument("--N", type=int, default=16)
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--ab", default="", help="ENV=V1,V2: time the backward under each value, interleaved")
    a = ap.parse_args()
    B, D, L, N = a.B, a.D, a.L, a.N
    g = torch.Generator(device="cuda").manual_seed(0)
    dt = torch.bfloat16
    u = torch.randn(B, D, L, device="cuda", generator=g).to(dt)
    delta = (torch.randn(B, D, L, device="cuda", generator=g) * 0.5 - 1).to(dt)
    A = -torch.exp(torch.randn(D, N, device="cuda", generator=g) * 0.5)
    Bm = torch.randn(B, N, L, device="cuda", generator=g).to(dt)
    Cm = torch.randn(B, N, L, device="cuda", generator=g).to(dt)
    Dv = torch.randn(D, device="cuda", generator=g)
    z = torch.randn(B, D, L, device="cuda", generator=g).to(dt)
    bias = torch.randn(D, device="cuda", generator=g) * 0.1
    fwd = lambda: selective_scan_fn(u, delta, A, Bm, Cm, D=Dv, z=z, delta_bias=bias, delta_softplus=True)  # noqa
    t_f = timeit(fwd, a.iters)
    ins = [t.clone().requires_grad_(True) for t in (u, delta, A, Bm, Cm, Dv, z, bias)]
    dout = torch.randn(B, D, L, device="cuda", generator=g).to(dt)

    def fb():
        o = selective_scan_fn(*ins[:5], D=ins[5], z=ins[6], delta_bias=ins[7], delta_softplus=True)
        o.backward(dout)
    t_fb = timeit(fb, a.iters)
    if a.ab:
        var, vals = a.ab.split("=")
        res = {v: [] for v in vals.split(",")}
        for _ in range(3):
            for v in res:
                os.environ[var] = v
                res[v].append(timeit(fb, a.iters) - t_f)
        os.environ.pop(var, None)
        print("A/B bwd us:", {v: [round(x, 1) for x in ts] for v, ts in res.items()}, flush=True)
    s = 2
    fb_bytes = (4 * B * D * L + 2 * B * N * L) * s
    bb_bytes = (7 * B * D * L + 2 * B * N * L) * s + 2 * B * N * L * 4
    print(f"selective scan bf16 B={B} D={D} L={L} N={N}: fwd {t_f:.1f} us "
          f"({fb_bytes / t_f / 1e3:.0f} GB/s alg, {fb_bytes / t_f / 1e3 / 8000:.3f} of HBM) | "
          f"bwd {t_fb - t_f:.1f} us ({bb_bytes / (t_fb - t_f) / 1e3:.0f} GB/s alg)", flush=True)


if __name__ == "__main__":
    main()
