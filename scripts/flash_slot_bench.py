#!/usr/bin/env python
"""The generic flash_attn_qkvpacked_func slot (csrc/flash_slot.hip) at the DNABERT-2 shape
(S = 512, 12 heads x 64, bf16 qkv) with the [b, H, S, S] fp32 bias the reference's
BertEncoder.forward builds (ALiBi + key-pad mask, bert_layers.py:421-448), called as
bert_layers.py:188 does; HIP events, interleaved. Prints one JSON line per variant with the
forward and forward+backward times, TFLOP/s (4 b H S^2 D forward, 10 b H S^2 D backward) and the
bias bytes per launch (the HBM floor of the bias stream). Variants: LDS-staged bias tiles (default)
vs per-score global reads (DNA_FLASH_BIAS_DIRECT=1), no bias, and the PyTorch path it replaces
(bert_layers.py:167-178, materialised scores)."""
import argparse
import json
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timeit(fn, iters):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--b", type=int, default=32)
    ap.add_argument("--S", type=int, default=512)
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args()
    from dna_amd.config import alibi_slopes
    from dna_amd.ops import flash_attn_qkvpacked_func
    b, S, H, D = a.b, a.S, 12, 64
    g = torch.Generator().manual_seed(0)
    valid = torch.ones(b, S, dtype=torch.bool)
    valid[1::2, S - 37:] = False
    # the reference's bias: (1 - keymask) * -10000 + ALiBi, [b, H, S, S] fp32
    pos = torch.arange(S)
    rel = (pos[None, :] - pos[:, None]).abs().float()
    alibi = -torch.tensor(alibi_slopes(H)).view(H, 1, 1) * rel
    bias = ((~valid).float() * -10000.0).view(b, 1, 1, S) + alibi.view(1, H, S, S)
    bias = bias.to("cuda")
    qkv = (torch.randn(b, S, 3, H, D, generator=g) * 0.7).to("cuda", torch.bfloat16)
    dout = torch.randn(b, S, H, D, generator=g).to("cuda", torch.bfloat16)
    x = qkv.clone().requires_grad_(True)
    fl_f = 4.0 * b * H * S * S * D
    fl_b = 10.0 * b * H * S * S * D

    def torch_path(t, bias_):
        q, k, v = t.unbind(2)
        q, k, v = (u.permute(0, 2, 1, 3) for u in (q, k, v))
        s = q @ k.transpose(-1, -2) / math.sqrt(D) + bias_
        return (torch.softmax(s.float(), -1).to(t.dtype) @ v).permute(0, 2, 1, 3)

    variants = {"staged_bias": ("0", bias), "direct_bias": ("1", bias), "no_bias": ("0", None),
                "torch_path": (None, bias)}
    res = {k: {"fwd": [], "fwd_bwd": []} for k in variants}
    for _ in range(3):
        for name, (env, bb) in variants.items():
            if env is not None:
                os.environ["DNA_FLASH_BIAS_DIRECT"] = env
                fwd = lambda: flash_attn_qkvpacked_func(qkv, bb)  # noqa
                fb = lambda: flash_attn_qkvpacked_func(x, bb).backward(dout)  # noqa
            else:
                fwd = lambda: torch_path(qkv, bb)  # noqa
                fb = lambda: torch_path(x, bb).backward(dout)  # noqa
            with torch.no_grad():
                res[name]["fwd"].append(timeit(fwd, a.iters))
            res[name]["fwd_bwd"].append(timeit(fb, a.iters))
    os.environ.pop("DNA_FLASH_BIAS_DIRECT", None)
    bias_bytes = bias.numel() * bias.element_size()
    for name, r in res.items():
        tf, tfb = min(r["fwd"]), min(r["fwd_bwd"])
        tb = tfb - tf
        print(json.dumps({"variant": name, "b": b, "S": S, "H": H, "D": D, "fwd_ms": round(tf, 4),
                          "bwd_ms": round(tb, 4), "fwd_tflops": round(fl_f / tf / 1e9, 1),
                          "bwd_tflops": round(fl_b / tb / 1e9, 1),
                          "fwd_frac_bf16_peak": round(fl_f / tf / 1e9 / 2500.0, 4),
                          "bias_bytes": bias_bytes if variants[name][1] is not None else 0,
                          "bias_gbs_fwd": round(bias_bytes / tf / 1e6, 1) if variants[name][1] is not None else 0}),
              flush=True)


if __name__ == "__main__":
    main()
