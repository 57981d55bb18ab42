#!/usr/bin/env python
"""FFT long-conv micro-benchmark at BASELINE config D (HyenaDNA-small width D=256, L=65536), GPU.

Times dna_amd.hyena.fftconv (HIP four-step FFT kernels) and, for comparison, the same math
through torch.fft (rocFFT), with HIP events. Algorithmic bytes: fwd = u read + y write
(+ filter k read, amortised over the batch); bwd = dy, u read + du write (+ dk write).
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dna_amd import _native as N  # noqa: E402
from dna_amd.hyena import fftconv  # noqa: E402

PEAK_HBM = 8000.0  # GB/s
PEAK_FP32 = 157.3  # TFLOP/s, MI355X fp32 vector (MI355X_MICROARCH.md)


def timeit(fn, iters):
    for _ in range(2):
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


def torch_fftconv(u, k, bias, bidirectional):
    L = u.shape[-1]
    n = 2 * L
    kf = torch.fft.rfft(k, n=n) / n
    if bidirectional:
        pb = (L + 2 * (L // 2)) // 2 - L // 2
        u2 = torch.nn.functional.pad(u, (pb, n - L - pb))
        uf = torch.fft.rfft(u2.float(), n=n)
    else:
        uf = torch.fft.rfft(u.float(), n=n)
    y = torch.fft.irfft(uf * kf, n=n, norm="forward")[..., :L]
    return (y + u * bias).to(u.dtype)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=8)
    ap.add_argument("--D", type=int, default=256)
    ap.add_argument("--L", type=int, default=65536)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--dtype", default="bf16,fp32")
    ap.add_argument("--bidirectional", type=int, default=1)
    a = ap.parse_args()
    B, D, L, bi = a.B, a.D, a.L, bool(a.bidirectional)
    g = torch.Generator(device="cuda").manual_seed(0)
    for dn in a.dtype.split(","):
        dt = torch.bfloat16 if dn == "bf16" else torch.float32
        s = 2 if dt == torch.bfloat16 else 4
        u = torch.randn(B, D, L, device="cuda", generator=g).to(dt)
        k = torch.randn(D, L, device="cuda", generator=g) * torch.exp(-torch.linspace(0, 6, L, device="cuda"))
        bias = torch.randn(D, 1, device="cuda", generator=g)
        dy = torch.randn(B, D, L, device="cuda", generator=g).to(dt)
        ur = u.clone().requires_grad_(True)
        kr = k.clone().requires_grad_(True)
        br = bias.clone().requires_grad_(True)

        t_fwd = timeit(lambda: fftconv(u, k, bias, bidirectional=bi), a.iters)

        def fb():
            y = fftconv(ur, kr, br, bidirectional=bi)
            y.backward(dy)
        t_fb = timeit(fb, a.iters)
        t_bwd = t_fb - t_fwd
        t_torch = timeit(lambda: torch_fftconv(u, k, bias, bi), a.iters)
        fwd_bytes = 2 * B * D * L * s + D * L * 4
        bwd_bytes = 3 * B * D * L * s + 2 * D * L * 4
        # roofline: max(algorithmic bytes / HBM peak, FFT flops / fp32 VALU peak); flops of an
        # N-point complex transform = 5 N log2 N, per row pair a forward and an inverse transform
        # (the backward: dy forward, du inverse, plus one inverse per channel for dk)
        n = 2 * L
        lg = n.bit_length() - 1
        P = (B + 1) // 2 * D
        fwd_flop = P * 10 * n * lg
        bwd_flop = P * 10 * n * lg + D * 5 * n * lg
        b_fwd = max(fwd_bytes / (PEAK_HBM * 1e3), fwd_flop / (PEAK_FP32 * 1e6))
        b_bwd = max(bwd_bytes / (PEAK_HBM * 1e3), bwd_flop / (PEAK_FP32 * 1e6))
        print(f"{dn} B={B} D={D} L={L} bi={int(bi)}: fwd {t_fwd:8.1f} us ({fwd_bytes / t_fwd / 1e3:7.1f} GB/s alg, "
              f"{fwd_bytes / t_fwd / 1e3 / PEAK_HBM:.3f} of HBM, roofline frac {b_fwd / t_fwd:.3f}) | bwd {t_bwd:8.1f} us "
              f"({bwd_bytes / t_bwd / 1e3:7.1f} GB/s alg, roofline frac {b_bwd / t_bwd:.3f}) | torch.fft fwd {t_torch:8.1f} us "
              f"-> speedup {t_torch / t_fwd:.2f}x", flush=True)


if __name__ == "__main__":
    main()
