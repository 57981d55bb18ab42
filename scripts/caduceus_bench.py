#!/usr/bin/env python
"""BASELINE config E: Caduceus bi-directional Mamba MLM pretraining at seq_len 131,072
(configs[4], "DDP on 8xMI355X"), d_model 256 x 8 BiMamba layers (rcps=False, RMSNorm, tied
in/out projections), char vocabulary (12 -> 16), bf16 autocast, 15 % masked positions. One step =
forward + masked CE + backward + gradient all-reduce (dna_amd.trainer.ModuleTrainer: flat
buckets over RCCL, overlapped with the backward) + global clip + fused AdamW. Synthetic uniform
ACGT tokens, random init. Data parallel over independent sequences (weak scaling):

    python scripts/caduceus_bench.py [--B 1] [--steps 5] [--warmup 2] [--json out.json]
    python -m torch.distributed.run --nproc-per-node N scripts/caduceus_bench.py ...

Prints one JSON line (rank 0): sequences/s over all ranks, the HIP kernel families with their
HBM rate (algorithmic bytes / HIP-event time on the launch stream) and, for the selective scan,
its VALU rate under the work model of DESIGN.md §5.2; `roofline` = the dominant HIP family.
"""
import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dna_amd.caduceus import CaduceusForMaskedLM  # noqa: E402
from dna_amd.functional import OpTimer  # noqa: E402
from dna_amd.tokenizer import CharacterTokenizer  # noqa: E402
from dna_amd.trainer import ModuleTrainer  # noqa: E402

PEAK_HBM_GBS = 8000.0
PEAK_FP32_TFLOPS = 157.3  # MI355X fp32 vector (MI355X_MICROARCH.md)
# selective scan VALU work model per (batch, channel, position, state), in fp32 FMA-issue
# equivalents x 2 flop (v_exp_f32 costs two FMA issue slots): forward 3 FMA + 1 exp = 10,
# backward (state recompute + reverse recurrence + the dA/dB/dC/ddelta/du terms) 10 FMA + 1 exp = 24
SCAN_FLOP_EQ = {"selective_scan_fwd": 10, "selective_scan_bwd": 24}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=1, help="sequences per GPU")
    ap.add_argument("--L", type=int, default=131072)
    ap.add_argument("--layers", type=int, default=8)
    ap.add_argument("--d-model", type=int, default=256)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--wire", default="fp32", choices=["fp32", "bf16"])
    ap.add_argument("--rcps", action="store_true",
                    help="RC-equivariant variant (RCPS layers, 2*d_model hidden channels)")
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    backend = os.environ.get("DNA_DIST_BACKEND", "nccl")
    if backend != "nccl":
        local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    torch.manual_seed(0)
    n_state = 16
    cm = CharacterTokenizer("ACGTN", a.L + 2).complement_map() if a.rcps else None
    m = CaduceusForMaskedLM(d_model=a.d_model, n_layer=a.layers, vocab_size=12,
                            ssm_cfg={"d_state": n_state}, rcps=a.rcps, complement_map=cm)
    loss_fn = lambda model, batch: model(batch[0], labels=batch[1])[0]
    tr = ModuleTrainer(m, torch.device("cuda", local), loss_fn, lr=8e-3, weight_decay=0.1,
                       max_grad_norm=1.0, wire_dtype=a.wire)
    g = torch.Generator(device="cuda").manual_seed(1 + rank)
    ids = torch.randint(7, 11, (a.B, a.L), device="cuda", generator=g)
    masked = torch.rand(a.B, a.L, device="cuda", generator=g) < 0.15
    batch = (torch.where(masked, torch.full_like(ids, 3), ids),
             torch.where(masked, ids, torch.full_like(ids, -100)))

    for _ in range(a.warmup):
        tr.step(batch)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    timer = OpTimer()
    timer.__enter__()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        loss = tr.step(batch)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    timer.__exit__()
    el_t = torch.tensor([el], dtype=torch.float64, device="cuda")
    if world > 1:
        dist.all_reduce(el_t, op=dist.ReduceOp.MAX)
    el = float(el_t.item())
    summ = timer.summary()
    d_inner = 2 * a.d_model
    kernels, total = {}, {}
    for k, (n, ms, units, kind) in summ.items():
        rate = units / (ms * 1e-3)
        kernels[k] = {"launches_per_step": n / a.steps, "avg_ms": round(ms, 4),
                      "share_of_step": round(n * ms / (el * 1e3), 4), "bound": "hbm",
                      "bytes_per_launch": units, "achieved_gbs": round(rate / 1e9, 1),
                      "frac": round(rate / 1e9 / PEAK_HBM_GBS, 4)}
        if k in SCAN_FLOP_EQ:  # one launch = one direction of one layer: [B, d_inner, L, N]
            fl = SCAN_FLOP_EQ[k] * a.B * d_inner * a.L * n_state
            tf = fl / (ms * 1e-3) / 1e12
            kernels[k].update(valu_flop_eq_per_launch=fl, achieved_valu_tflops=round(tf, 2),
                              valu_frac=round(tf / PEAK_FP32_TFLOPS, 4))
            if tf / PEAK_FP32_TFLOPS > rate / 1e9 / PEAK_HBM_GBS:
                kernels[k]["bound"] = "valu"
        total[k] = n * ms
    dom = max(total, key=total.get)
    kd = kernels[dom]
    if kd["bound"] == "valu":
        roof = {"bound": "valu", "achieved": kd["achieved_valu_tflops"], "peak": PEAK_FP32_TFLOPS,
                "unit": "TFLOP/s", "frac": kd["valu_frac"], "kernel": dom,
                "algorithmic_per_launch": kd["valu_flop_eq_per_launch"],
                "hbm": {"achieved_gbs": kd["achieved_gbs"], "frac": kd["frac"]}}
    else:
        roof = {"bound": "hbm", "achieved": kd["achieved_gbs"], "peak": PEAK_HBM_GBS, "unit": "GB/s",
                "frac": kd["frac"], "kernel": dom, "algorithmic_per_launch": kd["bytes_per_launch"]}
    seqs = a.B * a.steps * world
    line = {"metric": "Caduceus MLM sequences/sec, seq_len=131072 (BASELINE configs[4])",
            "value": round(seqs / el, 3), "unit": "sequences/s", "n_gpus": world, "steps": a.steps,
            "warmup": a.warmup, "ms_per_step": round(el / a.steps * 1e3, 2),
            "tokens_per_s": round(seqs * a.L / el), "higher_is_better": True, "scaling": "weak",
            "dtype": "bf16", "data": "synthetic uniform ACGT tokens, 15% masked, random init",
            "config": {"workload": "Caduceus bi-Mamba MLM (BASELINE configs[4])",
                       "d_model": a.d_model, "n_layer": a.layers, "d_state": n_state,
                       "seq_len": a.L, "per_gpu_batch": a.B, "parallelism": f"dp{world}",
                       "grad_wire": a.wire, "rcps": a.rcps},
            "final_loss": round(float(loss.item()), 4),
            "hip_kernel_share": round(sum(total.values()) / (el * 1e3), 4),
            "roofline": roof, "kernels": kernels}
    if rank == 0:
        print(json.dumps(line), flush=True)
        if a.json:
            with open(a.json, "w") as f:
                json.dump(line, f, indent=1)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
