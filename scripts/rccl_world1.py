#!/usr/bin/env python
"""The RCCL leg of the data-parallel step on ONE GPU (tests/test_gpu_rccl.py runs it).

A one-GPU box cannot run a multi-rank RCCL job, but a world-1 "nccl" process group executes the
same code: `init_process_group("nccl", device_id=...)` (dna_amd.launch), GradBucketReducer's
per-bucket async all_reduce on RCCL's stream, finish()'s waits and the bf16 wire format's
cast-back -- everything configs C / E do per step except the xGMI transfer itself. With one rank
the SUM is the identity, so the reduced gradients must equal the reducer-off gradients bit for bit
(fp32 wire) or their bf16 rounding exactly (bf16 wire).

Prints one JSON line per model (DNABERT-2 117M at a small batch through MLMTrainer; Caduceus
through ModuleTrainer). Run as a fresh process: RANK=0 WORLD_SIZE=1 DNA_DDP_FORCE=1.
"""
import json
import os
import sys

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _grads(tr, run_backward, enabled, wire):
    """One backward with the reducer on/off and the given wire format; returns the flat fp32
    gradient after finish() and how many buckets the backward itself launched."""
    tr.reducer.enabled = enabled
    tr.reducer.wire_dtype = wire
    tr.opt.zero_grad()
    tr.reducer.prepare(sync=True)
    run_backward()
    tr.reducer.finish()
    torch.cuda.synchronize()
    return tr.flat.grad.detach().clone(), tr.reducer.fired_in_backward


def _compare(tr, run_backward, reset):
    reset()
    g_learn, _ = _grads(tr, run_backward, True, "fp32")      # first backward: counts learned
    reset()
    g_on, fired = _grads(tr, run_backward, True, "fp32")     # buckets fire inside the backward
    reset()
    g_off, _ = _grads(tr, run_backward, False, "fp32")
    reset()
    g_bf16, fired_bf16 = _grads(tr, run_backward, True, "bf16")
    ref_bf16 = g_off.to(torch.bfloat16).float()
    scale = float(g_off.abs().max())
    return {
        "n_buckets": len(tr.reducer.buckets),
        "fired_in_backward": fired, "fired_in_backward_bf16": fired_bf16,
        "fp32_wire_max_abs_diff": float((g_on - g_off).abs().max()),
        "fp32_wire_bit_equal": bool(torch.equal(g_on, g_off)),
        "first_step_max_abs_diff": float((g_learn - g_off).abs().max()),
        "bf16_wire_vs_rounded_max_abs_diff": float((g_bf16 - ref_bf16).abs().max()),
        "bf16_wire_vs_fp32_max_rel": float((g_bf16 - g_off).abs().max()) / max(scale, 1e-30),
        "grad_abs_max": scale,
    }


def dnabert2(device):
    import bench
    from dna_amd.bert_layers import BertForMaskedLM
    from dna_amd.trainer import MLMTrainer
    torch.manual_seed(2222)
    model = BertForMaskedLM(bench.MODEL_CFG, precision="bf16")
    tr = MLMTrainer(model, device, lr=5e-4, weight_decay=1e-5, max_grad_norm=1.0)
    assert tr.reducer.enabled and tr.world == 1, "DNA_DDP_FORCE=1 must enable the reducer"
    (b,) = bench.make_batches(1, 8, 0, device)
    rng = model.dropout_rng
    st = (rng.seed, rng.offset)

    def reset():
        rng.seed, rng.offset = st

    def run_backward():
        loss, _ = model.mlm_loss(b.masked_ids, b.mask, b.index, b.n_mask, b.n_unk_masked)
        loss.backward()

    res = _compare(tr, run_backward, reset)
    # and the trainer's own step (reducer -> grad_scale -> fused clip + AdamW) twice
    losses = [float(tr.step(b)) for _ in range(2)]
    res.update(model="dnabert2-117m", batch=8, step_losses=losses,
               backend=dist.get_backend())
    return res


def caduceus(device):
    from dna_amd.caduceus import CaduceusForMaskedLM
    from dna_amd.trainer import ModuleTrainer
    torch.manual_seed(0)
    L = 2048
    m = CaduceusForMaskedLM(d_model=128, n_layer=2, vocab_size=12, ssm_cfg={"d_state": 16})
    g = torch.Generator().manual_seed(1)
    ids = torch.randint(7, 11, (2, L), generator=g)
    mask = torch.rand(2, L, generator=g) < 0.15
    inp = torch.where(mask, torch.full_like(ids, 3), ids).to(device)
    labels = torch.where(mask, ids, torch.full_like(ids, -100)).to(device)

    def loss_fn(model, batch):
        return model(batch[0], labels=batch[1])[0]

    tr = ModuleTrainer(m, device, loss_fn, lr=1e-3, bucket_mb=0.25, autocast=torch.bfloat16)
    assert tr.reducer.enabled and tr.world == 1

    def run_backward():
        with torch.autocast("cuda", dtype=torch.bfloat16):
            loss = loss_fn(tr.model, (inp, labels))
        loss.backward()

    res = _compare(tr, run_backward, lambda: None)
    losses = [float(tr.step((inp, labels))) for _ in range(2)]
    res.update(model="caduceus", L=L, step_losses=losses, backend=dist.get_backend())
    return res


def main():
    os.environ.setdefault("DNA_DDP_FORCE", "1")
    from dna_amd.launch import init_rank_process_group
    device = init_rank_process_group(int(os.environ.get("LOCAL_RANK", "0")))
    try:
        which = sys.argv[1:] or ["dnabert2", "caduceus"]
        for w in which:
            print(json.dumps({"dnabert2": dnabert2, "caduceus": caduceus}[w](device)), flush=True)
    finally:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
