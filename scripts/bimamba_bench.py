#!/usr/bin/env python
"""BiMamba mixer fwd+bwd at BASELINE config E scale (Caduceus: d_model 256, d_inner 512,
d_state 16, L = 131072), bf16 activations/weights (A_log, D, dt bias fp32), GPU, HIP events.
Reports tokens/s of one mixer layer and the share of the HIP scan / conv kernels (OpTimer)."""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dna_amd.functional import OpTimer  # noqa: E402
from dna_amd.mamba import BiMambaWrapper  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=2)
    ap.add_argument("--L", type=int, default=131072)
    ap.add_argument("--d", type=int, default=256)
    ap.add_argument("--iters", type=int, default=3)
    a = ap.parse_args()
    torch.manual_seed(0)
    w = BiMambaWrapper(d_model=a.d, d_state=16).cuda()
    for n, p in w.named_parameters():
        if not (n.endswith("A_log") or n.endswith(".D") or "dt_proj.bias" in n):
            p.data = p.data.bfloat16()
    x = torch.randn(a.B, a.L, a.d, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    dy = torch.randn(a.B, a.L, a.d, device="cuda", dtype=torch.bfloat16)

    def step():
        w(x).backward(dy)

    step()
    torch.cuda.synchronize()
    timer = OpTimer()
    e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
    timer.__enter__()
    e0.record()
    for _ in range(a.iters):
        step()
    e1.record()
    e1.synchronize()
    timer.__exit__()
    ms = e0.elapsed_time(e1) / a.iters
    summ = timer.summary()
    own = sum(n * t for k, (n, t, u, kind) in summ.items()) / a.iters
    print(f"BiMamba d_model={a.d} L={a.L} B={a.B} bf16 fwd+bwd: {ms:.2f} ms/step, "
          f"{a.B * a.L / ms * 1e3:.0f} tokens/s; HIP scan+conv kernels {own:.2f} ms ({own / ms:.0%}); "
          + ", ".join(f"{k} {t:.3f} ms x{n / a.iters:.0f}" for k, (n, t, u, kind) in summ.items()),
          flush=True)


if __name__ == "__main__":
    main()
