#!/usr/bin/env python
"""HyenaOperator fwd+bwd at BASELINE config D scale (HyenaDNA-small layer: d_model 256, order 2,
filter_order 64, emb_dim 5, bidirectional, L = 65536), fp32, GPU. Reports tokens/s of one
operator layer and the share of its time spent in the HIP long-conv kernels (OpTimer)."""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dna_amd.functional import OpTimer  # noqa: E402
from dna_amd.hyena import HyenaOperator  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=4)
    ap.add_argument("--L", type=int, default=65536)
    ap.add_argument("--d", type=int, default=256)
    ap.add_argument("--iters", type=int, default=5)
    a = ap.parse_args()
    torch.manual_seed(0)
    op = HyenaOperator(d_model=a.d, l_max=a.L, order=2, filter_order=64, emb_dim=5, w=10,
                       bidirectional=True, lr_pos_emb=0.0).cuda()
    x = torch.randn(a.B, a.L, a.d, device="cuda", requires_grad=True)
    dy = torch.randn(a.B, a.L, a.d, device="cuda")

    def step():
        y = op(x)
        y.backward(dy)

    step()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
    timer = OpTimer()
    timer.__enter__()
    e0.record()
    for _ in range(a.iters):
        step()
    e1.record()
    e1.synchronize()
    timer.__exit__()
    ms = e0.elapsed_time(e1) / a.iters
    summ = timer.summary()
    conv_ms = sum(n * t for k, (n, t, u, kind) in summ.items() if k.startswith("fftconv")) / a.iters
    print(f"HyenaOperator d={a.d} L={a.L} B={a.B} fp32 fwd+bwd: {ms:.2f} ms/step, "
          f"{a.B * a.L / ms * 1e3:.0f} tokens/s; long-conv kernels {conv_ms:.2f} ms "
          f"({conv_ms / ms:.0%}); " + ", ".join(f"{k} {t:.3f} ms x{n / a.iters:.0f}" for k, (n, t, u, kind) in summ.items()),
          flush=True)


if __name__ == "__main__":
    main()
