#!/usr/bin/env python
"""Error of the bf16 gradient wire against the fp32 wire on DNABERT-2-117M's real gradients,
with N ranks that each hold a different batch.

Start N rank processes with `python scripts/wire_error.py --ranks N` (gloo: every rank on the
visible GPU; the RCCL path differs only in where the sums are formed). Each rank computes its own
gradient of the 117M model (bf16 step, dropout on, its own synthetic batch) and the step's
GradBucketReducer all-reduces it three ways:
  * fp32 wire (the default; what configs C / E run),
  * bf16 wire as the reducer ships it (GradBucketReducer(wire_dtype="bf16"): each rank's bucket
    cast to bf16, SUM over the ranks, cast back),
  * an emulation of RCCL's ring over a bf16 wire, which rounds every partial sum to bf16 on its
    way round the ring: sum_{r<N} bf16(g_r) accumulated in bf16, rank 0 first -- the worst
    rounding any hop order gives for N ranks.
The exact reference is the float64 sum of the fp32 gradients. Rank 0 prints one JSON line:
max |err| / max |g| and ||err|| / ||g|| over the whole flat gradient, and the worst
per-parameter ||err|| / ||g||, for each of the three.
Reference: Lightning DDP (/root/reference/train.py:630-639), all-reduce of fp32 gradients.
"""
import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _metrics(flat, approx, exact):
    err = (approx.double() - exact)
    gmax, gnorm = float(exact.abs().max()), float(exact.norm())
    worst, worst_name = 0.0, None
    for name, (o, n) in flat:
        e = float(err[o:o + n].norm())
        g = float(exact[o:o + n].norm())
        if g > 0 and e / g > worst:
            worst, worst_name = e / g, name
    return {"max_abs_rel": float(err.abs().max()) / gmax, "norm_rel": float(err.norm()) / gnorm,
            "worst_param_norm_rel": worst, "worst_param": worst_name}


def _note(rank, t0, what):
    if rank == 0:  # progress on stderr (a silent multi-minute run looks hung)
        print(f"[wire_error {time.perf_counter() - t0:7.1f}s] {what}", file=sys.stderr, flush=True)


def run(args):
    t0 = time.perf_counter()
    import bench
    from dna_amd.bert_layers import BertForMaskedLM
    from dna_amd.launch import init_rank_process_group
    from dna_amd.trainer import MLMTrainer
    device = init_rank_process_group(int(os.environ.get("LOCAL_RANK", "0")))
    rank, world = dist.get_rank(), dist.get_world_size()
    _note(rank, t0, f"process group up ({dist.get_backend()}, {world} ranks)")
    torch.manual_seed(2222)
    model = BertForMaskedLM(bench.MODEL_CFG, precision="bf16")
    tr = MLMTrainer(model, device, lr=5e-4, weight_decay=1e-5, max_grad_norm=1.0)
    (b,) = bench.make_batches(1, args.batch, rank, device)  # a different batch on every rank
    rng = model.dropout_rng
    st = (rng.seed, rng.offset)

    def grads(enabled, wire):
        rng.seed, rng.offset = st
        tr.reducer.enabled, tr.reducer.wire_dtype = enabled, wire
        tr.opt.zero_grad()
        tr.reducer.prepare(sync=True)
        loss, _ = model.mlm_loss(b.masked_ids, b.mask, b.index, b.n_mask, b.n_unk_masked)
        loss.backward()
        tr.reducer.finish()
        torch.cuda.synchronize()
        return tr.flat.grad.detach().clone()

    _note(rank, t0, "model and batch ready")
    grads(True, "fp32")                      # first backward: the reducer learns its counts
    local = grads(False, "fp32")             # this rank's own gradient
    g32 = grads(True, "fp32")
    _note(rank, t0, "fp32 wire done")
    g16 = grads(True, "bf16")
    _note(rank, t0, "bf16 wire done")
    # the checks' own exchanges on host tensors (gloo moves CUDA tensors through the host anyway)
    local_h = local.cpu()
    exact = local_h.double()
    dist.all_reduce(exact, op=dist.ReduceOp.SUM)
    parts = [torch.empty_like(local_h) for _ in range(world)]
    dist.all_gather(parts, local_h.to(torch.bfloat16).float())  # bf16 values, fp32 carrier
    ring = parts[0].to(torch.bfloat16)
    for p in parts[1:]:
        ring = (ring.float() + p).to(torch.bfloat16)  # every hop rounds to bf16
    del parts
    g32, g16 = g32.cpu(), g16.cpu()
    _note(rank, t0, "exact sum and ring emulation done")
    if rank == 0:
        names = {id(p): n for n, p in model.named_parameters()}
        flat = [(names.get(id(p), "?"), (o, n)) for p, (o, n, _) in zip(tr.flat.params, tr.flat.slices)]
        out = {"ranks": world, "backend": dist.get_backend(), "batch_per_rank": args.batch,
               "n_params": int(local.numel()), "n_buckets": len(tr.reducer.buckets),
               "fp32_wire": _metrics(flat, g32, exact),
               "bf16_wire": _metrics(flat, g16, exact),
               "bf16_ring_emulated": _metrics(flat, ring, exact),
               "bf16_unit_roundoff": 2.0 ** -8}
        print(json.dumps(out), flush=True)
    dist.barrier()
    dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ranks", type=int, default=4)
    ap.add_argument("--batch", type=int, default=8)
    args = ap.parse_args()
    if "WORLD_SIZE" not in os.environ:
        from dna_amd.launch import launch_ranks
        os.environ.setdefault("DNA_DIST_BACKEND", "gloo")
        sys.exit(launch_ranks(args.ranks, __file__, sys.argv[1:]))
    run(args)


if __name__ == "__main__":
    main()
