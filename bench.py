#!/usr/bin/env python
"""MLM pretraining throughput of DNABERT-2-117M at seq_len 512 on MI355X (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B]
    N > 1: either under a launcher (python -m torch.distributed.run --nproc-per-node N ...
    bench.py --gpus N ...) or plain `bench.py --gpus N`, which starts the N rank processes itself
    (rank r on cuda:r, RCCL; DNA_DIST_BACKEND=gloo rehearses it with every rank on one GPU).

One step = forward (HIP kernels) + fused masked-CE + backward + RCCL gradient all-reduce + global
clip + AdamW on a per-GPU batch of B synthetic hg38 windows (uniform ACGT, 4096 bp -> exactly 512
BPE tokens each, BERT 15 % masking), random-init weights of the 117,074,176-parameter
architecture, bf16 compute, dropout 0.1. Batches are tokenised/masked on the host before timing
and sit in HBM; K steps are timed between barrier + synchronize, max over ranks.
Prints ONE JSON line (rank 0) with the roofline of the dominant kernel (HIP events on the launch
stream over the timed region) and the CPU baseline (oracle restatement on this host's cores).
"""
import argparse
import json
import math
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "MLM sequences/sec, DNABERT-2-117M seq_len=512, at 1/2/4/8 MI355X"
MODEL_CFG = dict(vocab_size=4096, hidden_size=768, num_hidden_layers=12, num_attention_heads=12,
                 intermediate_size=3072, hidden_dropout_prob=0.1, attention_probs_dropout_prob=0.0,
                 layer_norm_eps=1e-12, max_position_embeddings=512, type_vocab_size=2,
                 pad_token_id=0, alibi_starting_size=512, hidden_act="gelu",
                 initializer_range=0.02, hyena_framework=True)
SEQ, WINDOW_BP = 512, 4096
PEAK_BF16_TFLOPS = 2500.0   # MI355X dense bf16 MFMA (MI355X_MICROARCH.md)
PEAK_HBM_GBS = 8000.0
TRAIN_FLOP_PER_SEQ = 3.586e11  # 3 x fwd FLOPs at S=512 incl. last-layer subset


def load_traffic(batch):
    """HBM bytes per launch of each timed op family from the newest profiles/r*/traffic.json
    measured at this per-GPU batch (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes over this
    bench, FETCH_SIZE doubled per the gfx950 correction; scripts/traffic_from_pmc.py). {} when
    there is none for this batch."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*", "traffic.json")))
    d = None
    for fn in reversed(files):
        with open(fn) as f:
            cand = json.load(f)
        if cand.get("batch") == batch:
            d = cand
            break
    if d is None:
        return {}
    rel = os.path.relpath(fn, ROOT)
    return {k: dict(v, source=rel) for k, v in d.get("families", {}).items()}


def make_batches(n_batches, batch, rank, device):
    from dna_amd.hg38 import bert_mask_fast
    from dna_amd.synthetic import random_windows
    from dna_amd.tokenizer import DNABertTokenizer
    from dna_amd.trainer import DeviceBatch
    tok = DNABertTokenizer()
    out = []
    for i in range(n_batches):
        wins = random_windows(batch, WINDOW_BP, seed=10_000 * rank + i)
        ids = torch.from_numpy(tok.encode_windows(wins, SEQ + 2, nthreads=min(16, os.cpu_count() or 1)))
        assert ids.shape == (batch, SEQ)
        assert int((ids == tok.pad_token_id).sum()) == 0, "4096-bp windows must fill 512 tokens"
        ms, mk, lb = [], [], []
        for j in range(batch):
            s, m, l = bert_mask_fast(ids[j], tok.mask_token_id, tok.pad_token_id, tok.vocab_size,
                                     tok.all_special_ids, seed=2222, sample_id=(rank << 40) | (i * batch + j))
            ms.append(s); mk.append(m); lb.append(l)
        out.append(DeviceBatch.from_host(torch.stack(ms), torch.stack(mk), torch.stack(lb), ids,
                                         device))
    return out


def measure_data_pipeline(batch, device):
    """train.py's data path: registry dataset bert_hg38 over a synthetic FASTA/BED -> torch
    DataLoader (batched __getitems__: FASTA -> native multithreaded BPE -> native masking; 8
    worker processes sharing this rank's host threads) -> DeviceBatch.from_host (row bookkeeping
    + pinned H2D copy), steady state over 60 batches."""
    import shutil
    from dna_amd.hg38 import host_threads
    from scripts.data_pipeline_bench import measure, synthetic_root
    # enough 4096-bp windows for warm-up + 60 timed batches of this size in one epoch
    root = synthetic_root(n_chroms=8, chrom_len=16_777_216 * max(1, -(-batch // 256)))
    workers = 8
    try:
        rate = measure(root, workers, batch, 60, device=device)
    finally:
        shutil.rmtree(root, ignore_errors=True)
    return {"seq_per_s": round(rate, 1), "threads": host_threads(), "workers": workers,
            "what": "train.py data path: BertHG38 DataLoader (FASTA -> native BPE -> masking, "
                    "8 workers) + DeviceBatch.from_host (pinned H2D) over 4096-bp synthetic hg38 "
                    "windows, steady state over 60 batches; not part of value"}


def cpu_baseline(seconds_budget=10.0, threads=None, cfg=None, seq=None, batch=2, max_seq=100000,
                 label="DNABERT-2-117M S=512"):
    """Oracle restatement (PyTorch CPU fp32, oracle/bert_ref.py, pinned to the reference) timing
    the same step (fwd + bert_cross_entropy + bwd + clip + AdamW, dropout 0.1) on a bounded sample."""
    from oracle import bert_ref
    from dna_amd.hg38 import host_threads
    threads = threads or min(host_threads(), 16)
    prev_threads = torch.get_num_threads()
    torch.set_num_threads(threads)
    torch.manual_seed(0)
    cfg = dict(cfg or MODEL_CFG)
    seq = seq or SEQ
    sd = {}
    for n, shape in bert_ref.state_dict_shapes(cfg):
        t = torch.randn(shape) * 0.02 if len(shape) > 1 else torch.zeros(shape)
        if "LayerNorm" in n or "layernorm" in n:
            t = torch.ones(shape) if n.endswith("weight") else torch.zeros(shape)
        sd[n] = t.requires_grad_(True)
    opt = torch.optim.AdamW(list(sd.values()), lr=5e-4, weight_decay=1e-5)
    drop = lambda t, site: torch.nn.functional.dropout(t, 0.1, True)

    def step(b):
        rng = np.random.default_rng(b)
        ids = torch.as_tensor(rng.integers(5, 4096, size=(b, seq)))
        u = torch.as_tensor(rng.random((b, seq)))
        mask = u < 0.15
        labels = torch.where(mask, ids, torch.full_like(ids, -100))
        masked = torch.where(mask, torch.full_like(ids, 4), ids)
        opt.zero_grad()
        _, _, dense = bert_ref.dnabert2_forward(sd, cfg, masked, labels, dropout=drop)
        loss = bert_ref.bert_cross_entropy(dense, mask, ids)
        loss.backward()
        torch.nn.utils.clip_grad_norm_(list(sd.values()), 1.0)
        opt.step()

    step(1)  # warmup
    b, n_seq, t_used = batch, 0, 0.0
    while (t_used < seconds_budget and n_seq < max_seq) or n_seq == 0:
        t0 = time.perf_counter()
        step(b)
        t_used += time.perf_counter() - t0
        n_seq += b
    torch.set_num_threads(prev_threads)
    return {"value": round(n_seq / t_used, 4), "unit": "sequences/s", "cores": threads,
            "kind": "port",
            "sample": f"{n_seq} sequences (batches of {b}) of {label} fp32 train steps "
                      f"(fwd+loss+bwd+clip+AdamW) with the oracle restatement on {threads} threads, "
                      f"{t_used:.1f} s timed"}


# BASELINE configs[0] / SURVEY §8(d) config A: 2 layers, d_model 128, 2 heads, S = 128, batch 8
CONFIG_A = dict(vocab_size=4096, hidden_size=128, num_hidden_layers=2, num_attention_heads=2,
                intermediate_size=512)


def dist_skeleton(args, world, rank, out=None):
    """--dist-dry-run: the multi-rank measurement protocol without the model (CPU, gloo): the
    same barrier / timed region / max-over-ranks / one-JSON-line path, with a gradient-sized
    all-reduce as the step. Used by the CPU test of the launcher; never a bench number."""
    dist.init_process_group("gloo")
    g = torch.ones(1 << 16)
    for _ in range(args.warmup):
        dist.all_reduce(g)
    dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        dist.all_reduce(g)
    dist.barrier()
    el = torch.tensor([time.perf_counter() - t0], dtype=torch.float64)
    dist.all_reduce(el, op=dist.ReduceOp.MAX)
    if rank == 0:
        print(json.dumps({"metric": METRIC, "value": None, "unit": "sequences/s", "n_gpus": world,
                          "steps": args.steps, "warmup": args.warmup, "dry_run": True,
                          "ms_per_step": round(float(el) / max(1, args.steps) * 1e3, 3),
                          "config": {"parallelism": f"dp{world}", "global_batch": args.batch * world}}),
              file=out or sys.stdout, flush=True)
    dist.barrier()
    dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)   # 100 timed, 20 warm-up
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--batch", type=int, default=int(os.environ.get("DNA_BENCH_BATCH", 512)))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-kernel-timing", action="store_true")
    ap.add_argument("--no-b64", action="store_true", help="skip the extra per-GPU b=64 measurement")
    ap.add_argument("--no-data-pipeline", action="store_true", help="skip the host data-path timing")
    ap.add_argument("--grad-wire", choices=("fp32", "bf16"), default="fp32",
                    help="gradient all-reduce wire format (GradBucketReducer wire_dtype)")
    ap.add_argument("--dist-dry-run", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--dump-params", default=None, help=argparse.SUPPRESS)  # debug: per-rank digest
    args = ap.parse_args()
    # the timed step must stay on the hand-written kernels: any torch/hipBLASLt GEMM fallback in
    # dna_amd.functional raises (DNA_STRICT_NATIVE=0 turns the check off for experiments)
    os.environ.setdefault("DNA_STRICT_NATIVE", "1")

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # no launcher: become one (N rank processes), before any GPU call in this process
        from dna_amd.launch import launch_ranks
        sys.exit(launch_ranks(args.gpus, __file__, sys.argv[1:]))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus and rank == 0:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}; measuring {world} ranks",
              file=sys.stderr)
    # the result is ONE JSON line on stdout: everything else the process writes to fd 1 -- RCCL's
    # init banner ("RCCL version ...", NCCL WARN lines), gloo's "[Gloo] Rank ..." lines -- goes
    # to stderr
    result_out = os.fdopen(os.dup(1), "w")
    sys.stdout.flush()
    os.dup2(2, 1)
    if args.dist_dry_run:
        return dist_skeleton(args, world, rank, result_out)

    data_pipeline = None
    if rank == 0 and world == 1 and not args.no_data_pipeline:
        # train.py's own data path, timed before this process touches the GPU (its DataLoader
        # workers fork from a clean process; the H2D leg then brings HIP up) -- not part of value
        data_pipeline = measure_data_pipeline(args.batch, torch.device("cuda", local))
    # DNA_DIST_BACKEND=gloo (rehearsal only): every rank on the visible GPUs round-robin, gradient
    # all-reduce over gloo -- exercises the multi-rank bench path on a one-GPU box
    from dna_amd.launch import init_rank_process_group, rank_device_index, wants_process_group
    use_pg = wants_process_group(world)  # DNA_DDP_FORCE=1: the RCCL leg at world 1 too
    if use_pg:
        device = init_rank_process_group(local)
    else:
        device = torch.device("cuda", rank_device_index(local))
    torch.cuda.set_device(device)

    from dna_amd.bert_layers import BertForMaskedLM
    from dna_amd.ddp import all_reduce_
    from dna_amd.functional import OpTimer
    from dna_amd.trainer import MLMTrainer

    torch.manual_seed(2222)
    model = BertForMaskedLM(MODEL_CFG, precision="bf16")
    trainer = MLMTrainer(model, device, lr=5e-4, weight_decay=1e-5, max_grad_norm=1.0,
                         wire_dtype=args.grad_wire)
    t_data = time.perf_counter()
    batches = make_batches(4, args.batch, rank, device)
    t_data = time.perf_counter() - t_data
    if data_pipeline is not None:
        data_pipeline["bench_batch_prep_seq_per_s"] = round(4 * args.batch / t_data, 1)

    if rank == 0:  # progress on stderr (the stdout line is the result)
        print(f"bench.py: {world} rank(s), model and batches ready", file=sys.stderr, flush=True)
    for i in range(args.warmup):
        trainer.step(batches[i % len(batches)])
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    timer = OpTimer() if not args.no_kernel_timing else None
    t0 = time.perf_counter()
    if timer:
        timer.__enter__()
    for i in range(args.steps):
        loss = trainer.step(batches[i % len(batches)])
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t1 = time.perf_counter()
    if timer:
        timer.__exit__()
    elapsed = torch.tensor([t1 - t0], dtype=torch.float64, device=device)
    if world > 1:
        all_reduce_(elapsed, op=dist.ReduceOp.MAX)
    elapsed = float(elapsed.item())
    final_loss = float(loss.item())

    seqs = args.batch * args.steps * world
    value = seqs / elapsed
    ms_per_step = elapsed / args.steps * 1e3

    # besides the best per-GPU batch, always report b=64
    b64 = None
    if args.batch != 64 and not args.no_b64:
        bb = make_batches(2, 64, rank, device)
        for i in range(3):
            trainer.step(bb[i % 2])
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        n64 = max(5, args.steps // 3)
        for i in range(n64):
            trainer.step(bb[i % 2])
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        e64 = torch.tensor([time.perf_counter() - t2], dtype=torch.float64, device=device)
        if world > 1:
            all_reduce_(e64, op=dist.ReduceOp.MAX)
        e64 = float(e64.item())
        b64 = {"value": round(64 * n64 * world / e64, 2), "ms_per_step": round(e64 / n64 * 1e3, 3),
               "steps": n64, "warmup": 3, "per_gpu_batch": 64}

    roofline, kernels = None, {}
    if timer:
        summ = timer.summary()
        total_ms = {k: v[0] * v[1] for k, v in summ.items()}
        traffic = load_traffic(args.batch)
        for k, (n, ms, units, kind) in summ.items():
            rate = units / (ms * 1e-3)
            kernels[k] = {"launches_per_step": n / args.steps, "avg_ms": round(ms, 4),
                          "share_of_step": round(total_ms[k] / (elapsed * 1e3), 4)}
            if kind == "flop":
                kernels[k].update(bound="mfma", achieved_tflops=round(rate / 1e12, 1),
                                  frac=round(rate / 1e12 / PEAK_BF16_TFLOPS, 4))
            else:
                kernels[k].update(bound="hbm", achieved_gbs=round(rate / 1e9, 1),
                                  frac=round(rate / 1e9 / PEAK_HBM_GBS, 4))
            if k in traffic:
                kernels[k]["traffic"] = traffic[k]["bytes_per_launch"]
        dom = max(total_ms, key=total_ms.get)
        n, ms, units, kind = summ[dom]
        rate = units / (ms * 1e-3)
        if kind == "flop":
            roofline = {"bound": "mfma", "achieved": round(rate / 1e12, 1), "peak": PEAK_BF16_TFLOPS,
                        "unit": "TFLOP/s", "frac": round(rate / 1e12 / PEAK_BF16_TFLOPS, 4)}
        else:
            roofline = {"bound": "hbm", "achieved": round(rate / 1e9, 1), "peak": PEAK_HBM_GBS,
                        "unit": "GB/s", "frac": round(rate / 1e9 / PEAK_HBM_GBS, 4)}
        roofline["traffic"] = traffic.get(dom, {}).get("bytes_per_launch")
        roofline["kernel"] = dom
        roofline["algorithmic_per_launch"] = units
        if dom in traffic:
            roofline["traffic_source"] = traffic[dom]["source"]

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline()
        one = cpu_baseline(seconds_budget=10.0, threads=1)  # the reference forces OMP_NUM_THREADS=1
        cpu["single_thread"] = {"value": one["value"], "cores": 1, "sample": one["sample"]}
        ca = {}
        for th in (None, 1):
            r = cpu_baseline(seconds_budget=10.0, threads=th, cfg=CONFIG_A, seq=128, batch=8,
                             label="config A (2 layers, d=128, S=128)")
            ca["single_thread" if th == 1 else "all_threads"] = {k: r[k] for k in ("value", "cores", "sample")}
        cpu["config_a"] = ca

    if args.dump_params:  # debug dump: every rank's flat parameters after the timed steps
        from dna_amd.launch import flat_digest
        os.makedirs(args.dump_params, exist_ok=True)
        with open(os.path.join(args.dump_params, f"rank{rank}.json"), "w") as f:
            json.dump(dict(flat_digest(trainer.flat.flat), rank=rank, world=world,
                           loss=final_loss, global_step=trainer.global_step), f)

    if rank == 0:
        line = {
            "metric": METRIC, "value": round(value, 2), "unit": "sequences/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms_per_step, 3),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "bf16",
            "data": "synthetic hg38 windows (uniform ACGT 4096 bp -> 512 BPE tokens, 15% BERT "
                    "masking), random-init weights",
            "config": {"workload": "DNABERT-2-117M MLM pretrain seq_len=512 bf16 (BASELINE configs[1])",
                       "model": "DNABERT-2-117M", "global_batch": args.batch * world,
                       "seq_len": SEQ, "parallelism": f"dp{world}", "grad_wire": args.grad_wire,
                       "grad_allreduce": trainer.reducer.enabled},
            "native_only": os.environ.get("DNA_STRICT_NATIVE") == "1",
            "model_tflops_per_gpu": round(value / world * TRAIN_FLOP_PER_SEQ / 1e12, 1),
            "model_mfu": round(value / world * TRAIN_FLOP_PER_SEQ / 1e12 / PEAK_BF16_TFLOPS, 4),
            "final_loss": round(final_loss, 4),
            "roofline": roofline, "kernels": kernels, "cpu_baseline": cpu,
            "data_pipeline": data_pipeline, "b64": b64,
        }
        print(json.dumps(line), file=result_out, flush=True)
    if use_pg:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
