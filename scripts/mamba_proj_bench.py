#!/usr/bin/env python
"""Mamba in_proj / out_proj products at config-E scale (Caduceus d_model 256, d_inner 512,
L = 131,072, b = 1; reference modeling_caduceus.py:88-91 -> mamba_ssm Mamba.in_proj/out_proj):
hipBLASLt (torch) against the hand-written strided MFMA GEMM (dna_gemm_bf16_strided), same
operands, HIP events, plus the max abs difference of the two results.

  in_proj fwd     xz[b, 2E, L] = W[2E, d] . h[b, L, d]^T          (channel-major output)
  in_proj dgrad   dh[T, d]     = g_x^T . W_x + g_z^T . W_z          (g_* [E, T])
  out_proj fwd    out[T, d]    = y[b, E, L]^T . W_o[d, E]^T
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dna_amd.functional import strided_gemm  # noqa: E402


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
    ap.add_argument("--L", type=int, default=131072)
    ap.add_argument("--d", type=int, default=256)
    ap.add_argument("--E", type=int, default=512)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    L, d, E = a.L, a.d, a.E
    T, E2 = L, 2 * E
    dev = "cuda"
    bf = torch.bfloat16
    g = torch.Generator(device=dev).manual_seed(0)
    h = torch.randn(T, d, device=dev, dtype=bf, generator=g)
    W = (torch.randn(E2, d, device=dev, generator=g) / d ** 0.5).to(bf)
    gx = torch.randn(E, T, device=dev, dtype=bf, generator=g)
    gz = torch.randn(E, T, device=dev, dtype=bf, generator=g)
    y = torch.randn(1, E, L, device=dev, dtype=bf, generator=g)
    Wo = (torch.randn(d, E, device=dev, generator=g) / E ** 0.5).to(bf)
    res = {}

    # in_proj forward
    xz_t = torch.empty(E2, T, device=dev, dtype=bf)
    xz_s = torch.empty(1, E2, L, device=dev, dtype=bf)
    f_t = lambda: torch.mm(W, h.t(), out=xz_t)
    f_s = lambda: strided_gemm(W, (d, 1, 0), h, (1, d, L * d), xz_s, (L, E2 * L), E2, L, d, 1)
    res["in_proj_fwd"] = dict(torch_us=timeit(f_t, a.iters), hip_us=timeit(f_s, a.iters),
                              max_abs_diff=float((xz_t.float() - xz_s[0].float()).abs().max()),
                              bytes=(T * d + E2 * d + E2 * T) * 2)
    from dna_amd import _native as N
    xz_p = torch.empty(1, E2, L, device=dev, dtype=bf)
    f_p = lambda: N.call("dna_proj_cm_bf16", W.data_ptr(), h.data_ptr(), None, E2, L, d, 1, 0,
                         xz_p.data_ptr(), N.stream_ptr())
    res["in_proj_fwd_proj_cm"] = dict(torch_us=res["in_proj_fwd"]["torch_us"],
                                      hip_us=timeit(f_p, a.iters),
                                      max_abs_diff=float((xz_t.float() - xz_p[0].float()).abs().max()),
                                      bytes=(T * d + E2 * d + E2 * T) * 2)

    # the same product token-major (C[T, 2E] = h . W^T): how much of the time is the layout
    xz_k = torch.empty(T, E2, device=dev, dtype=bf)
    f_k = lambda: strided_gemm(h, (d, 1, 0), W, (1, d, 0), xz_k, (E2, T * E2), T, E2, d, 1)
    f_kt = lambda: torch.mm(h, W.t(), out=xz_k)
    res["in_proj_fwd_token_major"] = dict(torch_us=timeit(f_kt, a.iters), hip_us=timeit(f_k, a.iters),
                                          max_abs_diff=0.0, bytes=(T * d + E2 * d + E2 * T) * 2)

    # in_proj data gradient (both halves)
    dh_t = torch.empty(T, d, device=dev, dtype=bf)
    dh_s = torch.empty(T, d, device=dev, dtype=bf)
    from dna_amd import _native as N

    def f_t2():
        torch.mm(gx.t(), W[:E], out=dh_t)
        dh_t.addmm_(gz.t(), W[E:])

    # both halves in one pass: k < E from g_x, k >= E from g_z
    f_s2 = lambda: N.call("dna_gemm_bf16_strided_cat", gx.data_ptr(), gz.data_ptr(), E, 1, T, 0,
                          W.data_ptr(), d, 1, 0, dh_s.data_ptr(), d, T * d, 0, None, None, T, d,
                          E2, 1, 1, N.stream_ptr())
    res["in_proj_dgrad"] = dict(torch_us=timeit(f_t2, a.iters), hip_us=timeit(f_s2, a.iters),
                                max_abs_diff=float((dh_t.float() - dh_s.float()).abs().max()),
                                bytes=(E2 * T + E2 * d + T * d) * 2)

    # out_proj forward
    o_t = torch.empty(T, d, device=dev, dtype=bf)
    o_s = torch.empty(T, d, device=dev, dtype=bf)
    f_t3 = lambda: torch.mm(y[0].t(), Wo.t(), out=o_t)
    f_s3 = lambda: strided_gemm(y, (1, L, E * L), Wo, (1, E, 0), o_s, (d, T * d), T, d, E, 1)
    res["out_proj_fwd"] = dict(torch_us=timeit(f_t3, a.iters), hip_us=timeit(f_s3, a.iters),
                               max_abs_diff=float((o_t.float() - o_s.float()).abs().max()),
                               bytes=(E * T + E * d + T * d) * 2)
    for k, v in res.items():
        v["hip_tbs"] = round(v["bytes"] / v["hip_us"] / 1e6, 2)
        v["torch_tbs"] = round(v["bytes"] / v["torch_us"] / 1e6, 2)
        print(json.dumps({"op": k, **{kk: (round(vv, 2) if isinstance(vv, float) else vv)
                                      for kk, vv in v.items()}}), flush=True)


if __name__ == "__main__":
    main()
