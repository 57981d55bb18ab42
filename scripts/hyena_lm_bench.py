#!/usr/bin/env python
"""HyenaDNA LM training step at BASELINE config D scale: HyenaDNA-small (d_model 256, 8 layers,
d_inner 1024, order 2, filter_order 64, emb_dim 5, bidirectional -- SURVEY §8f row 1) at
seq_len 65536, char vocabulary (12 -> 16), bf16 autocast, on 1 GPU. One step = fwd + CE over the
15 %-masked positions + bwd + fused AdamW. Synthetic uniform ACGT tokens, random init.
Reports sequences/s and tokens/s and the share of the HIP long-conv / operator kernels."""
import argparse
import os
import sys
import time

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dna_amd.functional import OpTimer  # noqa: E402
from dna_amd.hyena_lm import BertLMHeadModel  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=2)
    ap.add_argument("--L", type=int, default=65536)
    ap.add_argument("--layers", type=int, default=8)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--trainer", default="module", choices=["module", "torch"],
                    help="module: dna_amd.trainer.ModuleTrainer (flat buffers, clip 1.0 + fused "
                         "AdamW, direct gradients); torch: torch AdamW(fused), no clip (rounds 3-5)")
    a = ap.parse_args()
    torch.manual_seed(0)
    layer = {"_name_": "hyena", "emb_dim": 5, "filter_order": 64, "short_filter_order": 3,
             "l_max": a.L, "modulate": True, "w": 10, "lr_pos_emb": 0.0, "bidirectional": True}
    m = BertLMHeadModel(d_model=256, n_layer=a.layers, d_inner=1024, vocab_size=12,
                        pad_vocab_size_multiple=8, embed_dropout=0.1, residual_in_fp32=True,
                        layer=layer).cuda()
    g = torch.Generator(device="cuda").manual_seed(1)
    ids = torch.randint(7, 11, (a.B, a.L), device="cuda", generator=g)   # A C G T char ids
    masked = torch.rand(a.B, a.L, device="cuda", generator=g) < 0.15
    inp = torch.where(masked, torch.full_like(ids, 3), ids)              # [MASK] = 3
    if a.trainer == "module":
        from dna_amd.trainer import ModuleTrainer
        labels = torch.where(masked, ids, torch.full_like(ids, -100)).view(-1)

        def loss_fn(model, batch):
            # CE mean over the masked positions without a host sync (no boolean indexing):
            # per-token losses with ignore_index, summed, over their count
            (out, _) = model(batch)
            logits = out.logits[0]
            ce = F.cross_entropy(logits.reshape(-1, logits.shape[-1]).float(), labels,
                                 ignore_index=-100, reduction="none")
            return ce.sum() / (labels != -100).sum()

        tr = ModuleTrainer(m, "cuda", loss_fn, lr=6e-4, weight_decay=0.1, max_grad_norm=1.0)

        def step():
            return tr.step((inp, masked))
    else:
        opt = torch.optim.AdamW(m.parameters(), lr=6e-4, weight_decay=0.1, fused=True)

        def step():
            opt.zero_grad(set_to_none=True)
            with torch.autocast("cuda", dtype=torch.bfloat16):
                (out, _) = m((inp, masked))
                logits = out.logits[0]
            loss = F.cross_entropy(logits[masked].float(), ids[masked])
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
    print(f"HyenaDNA-small (d256 x{a.layers}) L={a.L} B={a.B} bf16 train step: {dt * 1e3:.1f} ms, "
          f"{a.B / dt:.2f} seq/s, {a.B * a.L / dt:.0f} tokens/s, loss {loss.item():.3f}; HIP Hyena "
          f"kernels {own:.1f} ms ({own / (dt * 1e3):.0%}): "
          + ", ".join(f"{k} {t:.3f} ms x{n / a.steps:.0f}" for k, (n, t, u, kind) in summ.items()),
          flush=True)
    # one JSON line in bench.py's format: HBM roofline of the dominant HIP kernel family
    # (algorithmic bytes per launch from the op's own accounting / HIP-event average duration)
    kernels = {}
    for k, (n, t, u, kind) in summ.items():
        rate = u / (t * 1e-3)
        kernels[k] = {"launches_per_step": n / a.steps, "avg_ms": round(t, 4),
                      "share_of_step": round(n * t / a.steps / (dt * 1e3), 4)}
        if kind == "flop":
            kernels[k].update(bound="mfma", achieved_tflops=round(rate / 1e12, 1), frac=round(rate / 2.5e15, 4))
        else:
            kernels[k].update(bound="hbm", achieved_gbs=round(rate / 1e9, 1), frac=round(rate / 8e12, 4))
    # FFT long conv: roofline = max(algorithmic bytes / HBM peak, FFT flops / fp32 VALU peak)
    # (5 N log2 N per N-point complex transform; forward: the filter's D/2 channel pairs + a
    # forward and an inverse transform per row pair; backward: dy forward + du inverse per pair,
    # one inverse per channel for dk)
    D, N = 256, 2 * a.L
    lg, P = N.bit_length() - 1, (a.B + 1) // 2 * D
    tr = {"fftconv_fwd": (D // 2 + 2 * P), "fftconv_bwd": (2 * P + D)}
    for k, ntr in tr.items():
        if k in summ:
            n, t, u, kind = summ[k]
            flop = ntr * 5 * N * lg
            bound_ms = max(u / 8e12, flop / 157.3e12) * 1e3
            kernels[k].update(flop_per_launch=flop, roofline_bound_ms=round(bound_ms, 4),
                              roofline_frac=round(bound_ms / t, 4))
    dom = max(summ, key=lambda k: summ[k][0] * summ[k][1]) if summ else None
    roof = None
    if dom:
        n, t, u, kind = summ[dom]
        roof = {"kernel": dom, "bound": kernels[dom]["bound"], "avg_ms": round(t, 4),
                "algorithmic_per_launch": u, "frac": kernels[dom]["frac"],
                "achieved": kernels[dom].get("achieved_gbs", kernels[dom].get("achieved_tflops")),
                "peak": 8000.0 if kind != "flop" else 2500.0,
                "unit": "GB/s" if kind != "flop" else "TFLOP/s"}
        if "roofline_frac" in kernels[dom]:
            roof.update(fft_roofline_bound_ms=kernels[dom]["roofline_bound_ms"],
                        fft_roofline_frac=kernels[dom]["roofline_frac"])
    import json
    print(json.dumps({"metric": "HyenaDNA-small MLM train step (BASELINE config D)", "value": round(a.B / dt, 3),
                      "unit": "sequences/s", "tokens_per_s": round(a.B * a.L / dt), "ms_per_step": round(dt * 1e3, 2),
                      "steps": a.steps, "dtype": "bf16", "data": "synthetic uniform ACGT, random init",
                      "config": {"workload": f"HyenaDNA-small d256 x{a.layers} L={a.L}", "batch": a.B,
                                 "seq_len": a.L, "trainer": a.trainer}, "roofline": roof, "kernels": kernels}), flush=True)


if __name__ == "__main__":
    main()
