#!/usr/bin/env python
"""Digest of the FFT long-conv gradients (du, dk, dbias) at the config-D shape, GPU. Run once
with DNA_FFT_BWD_SPLIT=1 (four row passes) and once without (the fused row_bwd_kernel); the two
digests must be equal (the fused pass computes the same fp32 values in the same order)."""
import argparse
import hashlib
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dna_amd.hyena import fftconv  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=2)
    ap.add_argument("--D", type=int, default=256)
    ap.add_argument("--L", type=int, default=65536)
    ap.add_argument("--bidirectional", type=int, default=0)
    a = ap.parse_args()
    g = torch.Generator(device="cuda").manual_seed(0)
    for dt in (torch.bfloat16, torch.float32):
        u = torch.randn(a.B, a.D, a.L, device="cuda", generator=g).to(dt).requires_grad_(True)
        k = (torch.randn(a.D, a.L, device="cuda", generator=g)
             * torch.exp(-torch.linspace(0, 6, a.L, device="cuda"))).requires_grad_(True)
        bias = torch.randn(a.D, 1, device="cuda", generator=g).requires_grad_(True)
        dy = torch.randn(a.B, a.D, a.L, device="cuda", generator=g).to(dt)
        y = fftconv(u, k, bias, bidirectional=bool(a.bidirectional))
        y.backward(dy)
        dig = []
        for t in (y, u.grad, k.grad, bias.grad):
            dig.append(hashlib.sha256(t.detach().contiguous().view(torch.uint8).cpu().numpy().tobytes()).hexdigest()[:10])
        # the backward alone, HIP events (median of 10)
        ts = []
        for _ in range(12):
            y = fftconv(u, k, bias, bidirectional=bool(a.bidirectional))
            e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
            torch.cuda.synchronize()
            e0.record()
            y.backward(dy)
            e1.record()
            e1.synchronize()
            ts.append(e0.elapsed_time(e1) * 1e3)
        ts = sorted(ts[2:])
        print(f"{str(dt)[6:]} B={a.B} D={a.D} L={a.L} bi={a.bidirectional} "
              f"split={os.environ.get('DNA_FFT_BWD_SPLIT', '0')} y/du/dk/db {' '.join(dig)} "
              f"bwd {ts[len(ts) // 2]:.1f} us", flush=True)


if __name__ == "__main__":
    main()
