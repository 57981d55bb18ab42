#!/usr/bin/env python
"""Which torch ops (outside the HIP library) a training step of config D (HyenaDNA) or E
(Caduceus) launches, and from where: one profiled step under torch.profiler (CPU activity, Python
stacks), aten ops counted per step and grouped by the innermost dna_amd frames. Used to find the
small copy / cast / fill / reduce kernels around the hand-written ones.

    python scripts/op_census.py --model hyena|caduceus [--L 65536] [--top 40]
"""
import argparse
import collections
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

WATCH = ("aten::copy_", "aten::to", "aten::_to_copy", "aten::fill_", "aten::zero_", "aten::sum",
         "aten::add", "aten::add_", "aten::mul", "aten::neg", "aten::exp", "aten::cos", "aten::sin",
         "aten::clone", "aten::contiguous", "aten::zeros", "aten::empty_like", "aten::cat",
         "aten::gelu", "aten::gelu_backward", "aten::sub", "aten::div", "aten::index", "aten::where")


def build(model, L):
    if model == "bert":  # bench.py's DNABERT-2 step (MLMTrainer), at a small per-GPU batch
        import bench
        from dna_amd.bert_layers import BertForMaskedLM
        from dna_amd.trainer import MLMTrainer
        dev = torch.device("cuda", 0)
        m = BertForMaskedLM(bench.MODEL_CFG, precision="bf16")
        tr = MLMTrainer(m, dev, lr=5e-4, weight_decay=1e-5, max_grad_norm=1.0)
        batches = bench.make_batches(1, 64, 0, dev)
        return lambda: tr.step(batches[0])
    if model == "hyena":
        from dna_amd.hyena_lm import BertLMHeadModel
        layer = {"_name_": "hyena", "emb_dim": 5, "filter_order": 64, "short_filter_order": 3,
                 "l_max": L, "modulate": True, "w": 10, "lr_pos_emb": 0.0, "bidirectional": True}
        m = BertLMHeadModel(d_model=256, n_layer=8, d_inner=1024, vocab_size=12,
                            pad_vocab_size_multiple=8, embed_dropout=0.1, residual_in_fp32=True,
                            layer=layer).cuda()
        opt = torch.optim.AdamW(m.parameters(), lr=6e-4, weight_decay=0.1, fused=True)
        g = torch.Generator(device="cuda").manual_seed(1)
        ids = torch.randint(7, 11, (2, L), device="cuda", generator=g)
        masked = torch.rand(2, L, device="cuda", generator=g) < 0.15
        inp = torch.where(masked, torch.full_like(ids, 3), ids)

        def step():
            opt.zero_grad(set_to_none=True)
            with torch.autocast("cuda", dtype=torch.bfloat16):
                (out, _) = m((inp, masked))
                logits = out.logits[0]
            loss = F.cross_entropy(logits[masked].float(), ids[masked])
            loss.backward()
            opt.step()
        return step
    from dna_amd.caduceus import CaduceusForMaskedLM
    from dna_amd.trainer import ModuleTrainer
    m = CaduceusForMaskedLM(d_model=256, n_layer=8, vocab_size=12, ssm_cfg={"d_state": 16})
    tr = ModuleTrainer(m, torch.device("cuda", 0), lambda model, b: model(b[0], labels=b[1])[0],
                       lr=8e-3, weight_decay=0.1, max_grad_norm=1.0)
    g = torch.Generator(device="cuda").manual_seed(1)
    ids = torch.randint(7, 11, (1, L), device="cuda", generator=g)
    masked = torch.rand(1, L, device="cuda", generator=g) < 0.15
    inp = torch.where(masked, torch.full_like(ids, 3), ids)
    labels = torch.where(masked, ids, torch.full_like(ids, -100))
    return lambda: tr.step((inp, labels))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="hyena", choices=["hyena", "caduceus", "bert"])
    ap.add_argument("--L", type=int, default=0)
    ap.add_argument("--top", type=int, default=40)
    a = ap.parse_args()
    L = a.L or (65536 if a.model == "hyena" else 131072)
    os.environ.setdefault("DNA_STRICT_NATIVE", "1")
    torch.manual_seed(0)
    step = build(a.model, L)
    for _ in range(2):
        step()
    torch.cuda.synchronize()
    import traceback

    from torch.utils._python_dispatch import TorchDispatchMode

    per = collections.Counter()
    sites = collections.Counter()

    class Census(TorchDispatchMode):
        def __torch_dispatch__(self, func, types, args=(), kwargs=None):
            name = str(func.overloadpacket.__name__)
            if any(name == w.split("::")[1] for w in WATCH) or name in ("_to_copy", "fill_", "zero_", "copy_"):
                per[name] += 1
                frames = [f"{os.path.basename(fr.filename)}:{fr.lineno}"
                          for fr in traceback.extract_stack()[:-1]
                          if "dna_amd" in fr.filename or "scripts" in fr.filename]
                shp = "x".join(str(v) for v in args[0].shape) if args and hasattr(args[0], "shape") else ""
                dt = str(args[0].dtype).replace("torch.", "") if args and hasattr(args[0], "dtype") else ""
                sites[(name, (" <- ".join(reversed(frames[-3:])) or "(autograd)") + f" [{shp} {dt}]")] += 1
            return func(*args, **(kwargs or {}))

    with Census():
        step()
        torch.cuda.synchronize()
    print("aten ops per step:", dict(per.most_common()))
    for (name, where), n in sites.most_common(a.top):
        print(f"{n:5d}  {name:14s} {where or '(autograd engine / no dna_amd frame)'}")

if __name__ == "__main__":
    main()
