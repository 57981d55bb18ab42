#!/usr/bin/env python
"""Time HyenaDNA's implicit filter (HyenaFilter.filter_t: the positional MLP + modulation, the
config-D shape: emb_dim 5, filter_order 64, d_model 256, L 65,536) forward + backward under bf16
autocast, per call, with HIP events -- the share of the config-D step outside the long convolution.

    python scripts/filter_bench.py [--L 65536] [--iters 20]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dna_amd.hyena import HyenaFilter  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--L", type=int, default=65536)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    torch.manual_seed(0)
    f = HyenaFilter(256, emb_dim=5, order=64, seq_len=a.L, w=10, lr_pos_emb=0.0, modulate=True,
                    bidirectional=True).cuda()

    def run():
        with torch.autocast("cuda", dtype=torch.bfloat16):
            k = f.filter_t(a.L, 1)
        k.backward(torch.ones_like(k))

    for _ in range(3):
        run()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
    e0.record()
    for _ in range(a.iters):
        run()
    e1.record()
    e1.synchronize()
    print(f'{{"filter_fwd_bwd_us": {e0.elapsed_time(e1) * 1e3 / a.iters:.1f}, "L": {a.L}}}')


if __name__ == "__main__":
    main()
