#!/usr/bin/env python
"""Where the GeGLU epilogue GEMMs' time goes, at the bench shape (T = 262,144 tokens, F = 3072,
hidden 768): the fused forward (gated_layers + GeGLU, dna_geglu_linear_fwd) at dropout p = 0.1
and p = 0 (p = 0 skips the keep-bit draws) and the fused backward (wo data gradient + GeGLU
backward, dna_geglu_linear_dgrad_p: dg = bf16(da) * fac, no draws since round 6), against the
same GEMMs with the plain bf16 epilogue.
Interleaved rounds, one JSON line per (kernel, round); DNA_AMD_LIB picks the library build.

    python scripts/geglu_epi_ab.py [ROUNDS]"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dna_amd import _native as N  # noqa: E402


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    T, F, H = 512 * 512, 3072, 768
    gen = torch.Generator(device="cuda").manual_seed(1)
    x = (torch.rand(T, H, device="cuda", generator=gen) - 0.5).bfloat16()
    wg = ((torch.rand(2 * F, H, device="cuda", generator=gen) - 0.5) * 0.1).bfloat16()
    bg = torch.randn(2 * F, device="cuda", generator=gen) * 0.1
    g = torch.empty(T, 2 * F, device="cuda", dtype=torch.bfloat16)
    a = torch.empty(T, F, device="cuda", dtype=torch.bfloat16)
    dy = torch.randn(T, H, device="cuda", generator=gen).bfloat16()
    wt = (torch.randn(F, H, device="cuda", generator=gen) * 0.05).bfloat16()
    dg = torch.empty_like(g)
    s = N.stream_ptr()
    kern = {
        "fwd_p0.1": lambda: N.call("dna_geglu_linear_fwd", x.data_ptr(), wg.data_ptr(), bg.data_ptr(),
                                   T, F, H, 0.1, 7, 3, g.data_ptr(), a.data_ptr(), s),
        "fwd_p0": lambda: N.call("dna_geglu_linear_fwd", x.data_ptr(), wg.data_ptr(), bg.data_ptr(),
                                 T, F, H, 0.0, 7, 3, g.data_ptr(), a.data_ptr(), s),
        "fwd_plain": lambda: N.call("dna_linear_fwd", x.data_ptr(), wg.data_ptr(), bg.data_ptr(),
                                    T, 2 * F, H, g.data_ptr(), s),
        "bwd_fac": lambda: N.call("dna_geglu_linear_dgrad_p", dy.data_ptr(), wt.data_ptr(),
                                  g.data_ptr(), T, F, H, dg.data_ptr(), s),
        "bwd_plain": lambda: N.call("dna_linear_fwd", dy.data_ptr(), wt.data_ptr(), None, T, F, H,
                                    a.data_ptr(), s),
    }
    lib = os.path.basename(os.environ.get("DNA_AMD_LIB", "libdna_amd.so"))
    for rnd in range(rounds):
        for name, fn in kern.items():
            for _ in range(3):
                fn()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            e0.record()
            for _ in range(20):
                fn()
            e1.record()
            torch.cuda.synchronize()
            print(json.dumps({"lib": lib, "kernel": name, "round": rnd,
                              "ms": round(e0.elapsed_time(e1) / 20, 4)}), flush=True)


if __name__ == "__main__":
    main()
