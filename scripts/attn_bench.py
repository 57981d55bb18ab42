#!/usr/bin/env python
"""Attention kernel micro-benchmark at the bench shape (GPU): HIP-event timing of dna_attn_fwd
and dna_attn_bwd on random bf16 data, TF/s of algorithmic FLOPs (fwd 4bHS^2D, bwd 10bHS^2D)."""
import argparse
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dna_amd import _native as N  # noqa: E402
from dna_amd.config import alibi_slopes  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--b", type=int, default=128)
    ap.add_argument("--S", type=int, default=512)
    ap.add_argument("--H", type=int, default=12)
    ap.add_argument("--iters", type=int, default=30)
    ap.add_argument("--which", default="fwd,bwd")
    ap.add_argument("--dbias", type=int, default=1, help="backward with the fused bias partials")
    a = ap.parse_args()
    b, S, H, D = a.b, a.S, a.H, 64
    T = b * S
    torch.manual_seed(0)
    qkv = torch.randn(T, 3 * H * D, device="cuda").to(torch.bfloat16)
    kv = torch.ones(T, dtype=torch.uint8, device="cuda")
    slopes = torch.tensor(alibi_slopes(H), device="cuda")
    out = torch.empty(T, H * D, device="cuda", dtype=torch.bfloat16)
    lse = torch.empty(b, H, S, device="cuda")
    dout = torch.randn(T, H * D, device="cuda").to(torch.bfloat16)
    dqkv = torch.empty_like(qkv)
    delta = torch.empty(b * H * S, device="cuda")
    st = torch.cuda.current_stream().cuda_stream
    sc = 1.0 / math.sqrt(D)

    def fwd():
        N.call("dna_attn_fwd", qkv.data_ptr(), kv.data_ptr(), slopes.data_ptr(), b, S, H, D, 1, sc,
               out.data_ptr(), lse.data_ptr(), st)

    # the training step runs the backward with the fused Wqkv bias-gradient partials
    part = torch.empty(N.lib().dna_attn_dbias_part_rows(b, S), 3 * H * D, device="cuda")

    def bwd():
        N.call("dna_attn_bwd_ex", qkv.data_ptr(), out.data_ptr(), dout.data_ptr(), lse.data_ptr(),
               kv.data_ptr(), slopes.data_ptr(), b, S, H, D, 1, sc, dqkv.data_ptr(),
               delta.data_ptr(), part.data_ptr() if a.dbias else None, st)

    fwd()
    for name, fn, fl in (("fwd", fwd, 4.0), ("bwd", bwd, 10.0)):
        if name not in a.which:
            continue
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        ts = []
        for _ in range(a.iters):
            e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
            e0.record()
            fn()
            e1.record()
            e1.synchronize()
            ts.append(e0.elapsed_time(e1))
        ts.sort()
        med = ts[len(ts) // 2]
        print(f"attn_{name} b={b} S={S} H={H}: median {med * 1e3:.1f} us min {ts[0] * 1e3:.1f} us "
              f"-> {fl * b * H * S * S * D / (med * 1e-3) / 1e12:.1f} TF/s", flush=True)


if __name__ == "__main__":
    main()
