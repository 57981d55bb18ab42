#!/usr/bin/env python
"""Caduceus MLM training step at BASELINE config E scale on 1 GPU: bi-directional Mamba,
d_model 256, n_layer 8 (rcps=False, RMSNorm, tied in/out projections), seq_len 131072, char
vocabulary (12 -> 16), bf16 autocast, 15 % masked positions, fused AdamW. Synthetic uniform ACGT
tokens, random init. Reports sequences/s, tokens/s and the share of the HIP scan / conv kernels.
(The config's 8-GPU DDP run is data parallel over independent sequences.)"""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dna_amd.caduceus import CaduceusForMaskedLM  # noqa: E402
from dna_amd.functional import OpTimer  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=1)
    ap.add_argument("--L", type=int, default=131072)
    ap.add_argument("--layers", type=int, default=8)
    ap.add_argument("--steps", type=int, default=3)
    a = ap.parse_args()
    torch.manual_seed(0)
    m = CaduceusForMaskedLM(d_model=256, n_layer=a.layers, vocab_size=12,
                            ssm_cfg={"d_state": 16}).cuda()
    opt = torch.optim.AdamW(m.parameters(), lr=8e-3, weight_decay=0.1, fused=True)
    g = torch.Generator(device="cuda").manual_seed(1)
    ids = torch.randint(7, 11, (a.B, a.L), device="cuda", generator=g)
    masked = torch.rand(a.B, a.L, device="cuda", generator=g) < 0.15
    inp = torch.where(masked, torch.full_like(ids, 3), ids)
    labels = torch.where(masked, ids, torch.full_like(ids, -100))

    def step():
        opt.zero_grad(set_to_none=True)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            loss, _ = m(inp, labels=labels)
        loss.backward()
        opt.step()
        return loss

    for _ in range(2):
        step()
    torch.cuda.synchronize()
    timer = OpTimer()
    timer.__enter__()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        loss = step()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / a.steps
    timer.__exit__()
    summ = timer.summary()
    own = sum(n * t for k, (n, t, u, kind) in summ.items()) / a.steps
    print(f"Caduceus (d256 x{a.layers}, bi-Mamba) L={a.L} B={a.B} bf16 train step: {dt * 1e3:.1f} ms, "
          f"{a.B / dt:.2f} seq/s, {a.B * a.L / dt:.0f} tokens/s, loss {loss.item():.3f}; HIP scan/conv "
          f"kernels {own:.1f} ms ({own / (dt * 1e3):.0%}): "
          + ", ".join(f"{k} {t:.3f} ms x{n / a.steps:.0f}" for k, (n, t, u, kind) in summ.items()),
          flush=True)


if __name__ == "__main__":
    main()
