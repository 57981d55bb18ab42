"""A/B of the fused wo-dgrad + GeGLU-backward kernel variants (DNA_GEGLU_BWD_VAR) at the bench
shape (T = 262,144, F = 3072, hidden 768), interleaved rounds, vs the separate pair; one JSON
line per (variant, round)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dna_amd import _native as N  # noqa: E402


def main():
    T, F, H = 512 * 512, 3072, 768
    gen = torch.Generator(device="cuda").manual_seed(1)
    dy = torch.randn(T, H, device="cuda", generator=gen).bfloat16()
    wt = (torch.randn(F, H, device="cuda", generator=gen) * 0.05).bfloat16()
    g = torch.randn(T, 2 * F, device="cuda", generator=gen).bfloat16()
    dg = torch.empty_like(g)
    da = torch.empty(T, F, device="cuda", dtype=torch.bfloat16)
    s = N.stream_ptr()

    pdrop = float(os.environ.get("P", "0.1"))

    def fused():
        N.call("dna_geglu_linear_dgrad_p", dy.data_ptr(), wt.data_ptr(), g.data_ptr(), T, F, H,
               dg.data_ptr(), s)

    def gemm():  # the same GEMM with the plain bf16 epilogue (da stored, no GeGLU)
        N.call("dna_linear_fwd", dy.data_ptr(), wt.data_ptr(), None, T, F, H, da.data_ptr(), s)

    def pair():
        N.call("dna_linear_fwd", dy.data_ptr(), wt.data_ptr(), None, T, F, H, da.data_ptr(), s)
        N.call("dna_geglu_bwd", da.data_ptr(), g.data_ptr(), 1, T, F, dg.data_ptr(), s)

    variants = [v for v in os.environ.get("VARS", "0").split(",") if v]
    iters = int(os.environ.get("ITERS", "20"))
    for rnd in range(int(os.environ.get("ROUNDS", "3"))):
        for v in variants + ["pair", "gemm"]:
            fn = {"pair": pair, "gemm": gemm}.get(v, fused)
            os.environ["DNA_GEMM_ABL"] = "0"
            os.environ["DNA_GEGLU_BWD_SCHED"] = "2"
            if v.startswith("s"):  # s4: the deferred-epilogue schedule
                os.environ["DNA_GEGLU_BWD_SCHED"] = v[1:]
            elif v not in ("pair", "gemm"):
                os.environ["DNA_GEMM_ABL"] = v  # 0 = the real kernel, 64 / 128 diagnostics
            for _ in range(3):
                fn()
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            a.record()
            for _ in range(iters):
                fn()
            b.record()
            torch.cuda.synchronize()
            ms = a.elapsed_time(b) / iters
            print(json.dumps({"variant": v, "p": pdrop, "round": rnd, "ms": round(ms, 4),
                              "tflops": round(2 * T * F * H / ms / 1e9, 1),
                              "hbm_gbs_min_bytes": round((T * H * 2 + 4 * T * F * 2) / ms / 1e6, 1)}),
                  flush=True)


if __name__ == "__main__":
    main()
