#!/usr/bin/env python
"""`python train.py experiment=dnabert2/dnabert2_hg38_pretrain key=value ...` on MI355X.

Mirrors the reference entry point (train.py:699-711: Hydra main over configs/config.yaml, then
train() :668-694 -> Lightning fit) for the DNABERT-2 MLM path, without Hydra or Lightning:
  * config: dna_amd.compose (defaults lists, @package, overrides, eval/div_up resolvers);
    `--config-dir` may point at the reference's own configs/ tree, which composes unchanged;
  * registries: model "dnabert2" -> dna_amd.bert_layers.BertForMaskedLM (src/utils/registry.py:39),
    dataset "bert_hg38" -> dna_amd.hg38.BertHG38, "dnabert2_pretrain" (text corpus) ->
    dna_amd.corpus.DNABERT2Pretrain, task "hg38" + loss "bert_cross_entropy";
  * loop: MLMTrainer steps (fused loss, bucketed RCCL all-reduce, clip + AdamW, LR schedule per
    optimizer step, `accumulate_grad_batches`), DistributedSampler sharding across ranks
    (one process per GPU, torch.distributed.run), metrics train/loss, trainer/loss,
    train/perplexity, train/num_tokens, timer/step;
  * checkpoints in Lightning's layout ({"state_dict": {"model.<key>": ...}, ...}) so
    `train.pretrained_model_path` / `trainer.resume_from_checkpoint` interoperate; a missing
    resume path (the reference configs carry cluster paths) is a warning, not a crash.
The product path is GPU-only: `trainer.accelerator=cpu` is rejected (no CPU fallback).
"""
import argparse
import json
import math
import os
import sys
import time
import warnings

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from dna_amd.compose import compose  # noqa: E402

MODEL_REGISTRY = {"dnabert2": "dna_amd.bert_layers.BertForMaskedLM"}


def _import(path):
    mod, name = path.rsplit(".", 1)
    return getattr(__import__(mod, fromlist=[name]), name)


def _precision(p):
    p = str(p)
    if p in ("bf16", "bf16-mixed", "bfloat16"):
        return "bf16"
    if p in ("32", "32-true", "fp32", "float32"):
        return "fp32"
    raise ValueError(f"trainer.precision={p!r}: bf16 or 32")


def build_dataset(cfg):
    import dna_amd.corpus  # noqa: F401  (registers "dnabert2_pretrain")
    from dna_amd.hg38 import SequenceDataset
    kw = {k: v for k, v in cfg.dataset.to_container().items()
          if k != "_name_" and not k.startswith("__")}  # process_config drops "__" keys
    ds = SequenceDataset.registry[cfg.dataset._name_](**kw)
    return ds


def load_lightning_state(model, path, strict):
    ck = torch.load(path, map_location="cpu", weights_only=True)
    sd = ck.get("state_dict", ck)
    sd = {k[len("model."):] if k.startswith("model.") else k: v for k, v in sd.items()}
    missing, unexpected = model.load_state_dict(sd, strict=strict)
    return missing, unexpected


def save_checkpoint(path, trainer, epoch, batches_done=0, metrics=None):
    """Lightning-1.8 checkpoint layout: state_dict with the "model." prefix, torch AdamW
    optimizer state, timm scheduler state, epoch / global_step; plus this engine's dropout-stream
    position and the count of batches already consumed in `epoch` (mid-epoch resume). Written to
    a temporary file and renamed, so a crash never leaves a truncated last.ckpt."""
    m = trainer.model
    sd = {"model." + k: v.detach().cpu() for k, v in m.state_dict().items()}
    ck = {"state_dict": sd, "epoch": int(epoch), "global_step": int(trainer.global_step),
          "pytorch-lightning_version": "1.8.0",
          "optimizer_states": [trainer.opt.state_dict()],
          "lr_schedulers": [trainer.sched.state_dict()] if trainer.sched else [],
          "dna_amd": {"dropout_rng": trainer.rng_state(), "batches_done": int(batches_done),
                      "metrics": metrics or {}}}
    tmp = path + ".tmp"
    torch.save(ck, tmp)
    os.replace(tmp, path)


def train(cfg, dry_run=False, out=sys.stdout):
    from dna_amd.bert_layers import BertForMaskedLM  # noqa: F401
    from dna_amd.ddp import reduce_metrics
    from dna_amd.trainer import DeviceBatch, MLMTrainer

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    seed = cfg.train.get("seed")
    if seed is not None:
        torch.manual_seed(int(seed) + rank)

    tr = cfg.trainer
    if str(tr.get("accelerator", "gpu")) not in ("gpu", "cuda", "auto"):
        raise RuntimeError(f"trainer.accelerator={tr.accelerator!r}: dna_amd runs the hot path "
                           "on MI355X GPUs only (no CPU fallback)")
    model_cls = _import(MODEL_REGISTRY[cfg.model._name_])
    model = model_cls(config=cfg.model.config.to_container(),
                      precision=_precision(tr.get("precision", "bf16")))
    pre = cfg.train.get("pretrained_model_path")
    if pre:
        if os.path.exists(pre):
            load_lightning_state(model, pre, bool(cfg.train.get("pretrained_model_strict_load", True)))
        else:
            warnings.warn(f"train.pretrained_model_path {pre} not found; starting from init")
    ds = build_dataset(cfg)
    ds.setup()
    task = _import("dna_amd.tasks.registry")[cfg.task._name_]
    task = task(loss=cfg.task.loss, torchmetrics=cfg.task.get("torchmetrics"))
    sched = None
    if "scheduler" in cfg and cfg.scheduler is not None:
        sc = {k: v for k, v in cfg.scheduler.to_container().items() if k != "_name_"}
        if cfg.scheduler._name_ != "linear_warmup":
            raise NotImplementedError(f"scheduler {cfg.scheduler._name_!r} (linear_warmup only)")
        sched = sc
    opt = cfg.optimizer
    if dry_run:
        print(json.dumps({"dry_run": True, "model_params": sum(p.numel() for p in model.parameters()),
                          "train_windows": len(ds.dataset_train), "task": task.loss_name,
                          "scheduler": sched, "optimizer": opt.to_container()}), file=out)
        return None

    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    device = torch.device("cuda", local)
    torch.cuda.set_device(device)
    trainer = MLMTrainer(model, device, lr=float(opt.lr),
                         weight_decay=float(opt.get("weight_decay", 0.0)),
                         betas=tuple(opt.get("betas", (0.9, 0.999))),
                         max_grad_norm=float(tr.get("gradient_clip_val", 0.0) or 0.0),
                         scheduler=sched, seed=seed)
    resume = tr.get("resume_from_checkpoint") or cfg.train.get("ckpt")
    start_epoch, skip_batches, restored = 0, 0, {}
    if resume:
        if os.path.exists(resume):
            ck = torch.load(resume, map_location="cpu", weights_only=True)
            load_lightning_state(model, resume, True)
            trainer.flat.refresh_shadow()
            if ck.get("optimizer_states"):
                trainer.opt.load_state_dict(ck["optimizer_states"][0])
            if ck.get("lr_schedulers") and trainer.sched:
                trainer.sched.load_state_dict(ck["lr_schedulers"][0])
            trainer.global_step = int(ck.get("global_step", 0))
            start_epoch = int(ck.get("epoch", 0))
            extra = ck.get("dna_amd") or {}
            if extra.get("dropout_rng"):
                trainer.load_rng_state(extra["dropout_rng"])
                # distinct per rank, as MLMTrainer derives it
                trainer.model.dropout_rng.seed = (trainer.model.dropout_rng.seed + rank) & (2 ** 63 - 1)
            skip_batches = int(extra.get("batches_done", 0))
            restored = extra.get("metrics") or {}
        else:
            warnings.warn(f"resume checkpoint {resume} not found; training from scratch")

    # the permutation is randperm(seed + epoch) on every world size (DistributedSampler
    # semantics), so a mid-epoch resume replays exactly the interrupted epoch's
    # order, and the masks are keyed on (train.seed, epoch, window) (EpochSampler)
    sampler = torch.utils.data.distributed.DistributedSampler(
        ds.dataset_train, num_replicas=world, rank=rank,
        shuffle=True if world > 1 else bool(getattr(ds, "shuffle", True)), seed=int(seed or 0))
    if seed is not None and hasattr(ds.dataset_train, "mask_seed"):
        ds.dataset_train.mask_seed = (int(seed) * 0x9E3779B1 + 2222) & (2 ** 63 - 1)
    loader = ds.train_dataloader(sampler=sampler)
    accum = int(tr.get("accumulate_grad_batches", 1) or 1)
    max_steps = cfg.train.get("max_steps") or tr.get("max_steps")
    max_epochs = int(tr.get("max_epochs", 1) or 1)
    log_every = int(tr.get("log_every_n_steps", 10) or 10)
    limit = tr.get("limit_train_batches", 1.0)
    pad_id = getattr(ds.tokenizer, "pad_token_id", 3)
    ck_cfg = cfg.get("callbacks", {}) or {}
    mc = ck_cfg.get("model_checkpoint") if ck_cfg else None
    ck_path = None
    if rank == 0 and mc is not None:
        d = mc.get("dirpath", "checkpoints/")
        os.makedirs(d, exist_ok=True)
        ck_path = os.path.join(d, "last.ckpt")
    ck_every = int((mc.get("every_n_train_steps") if mc is not None else 0) or 1000)
    # task torchmetrics (torchmetrics.py:24-115): Perplexity reset each epoch, NumTokens never.
    # Both are updated per micro-batch with that micro-batch's loss and target.numel(), and
    # SUM-reduced over ranks when logged (dist_reduce_fx="sum", sync_dist=True).
    from dna_amd.tasks import NumTokens, Perplexity
    ppl, ntok = Perplexity(), NumTokens()
    ntok.count = torch.tensor(int(restored.get("num_tokens_local", 0)), dtype=torch.int64)
    t_last = time.perf_counter()
    done = False
    epoch = start_epoch

    def optimizer_step(micro):
        # Lightning 1.8 divides every micro-batch loss by accumulate_grad_batches, also in the
        # epoch's last, shorter window
        loss = trainer.step([m for m, _ in micro], accum=accum)
        for (_, numel), ml in zip(micro, trainer.micro_losses):
            ppl.update_count(ml, numel)  # numel = target.numel() of that micro-batch
            ntok.count = ntok.count + numel
        return loss

    def log_line(loss):
        nonlocal t_last
        step = trainer.global_step
        lv, sums = reduce_metrics(loss, 0, extra=[ppl.total_log_probs, ppl.count, ntok.count])
        now = time.perf_counter()
        if rank == 0:
            print(json.dumps({"step": step, "epoch": epoch, "train/loss": round(lv, 5),
                              "trainer/loss": round(lv, 5),
                              "train/perplexity": round(math.exp(sums[0] / max(sums[1], 1)), 4),
                              "train/num_tokens": int(sums[2]),
                              "trainer/lr": trainer.opt.param_groups[0]["lr"],
                              "timer/step": round((now - t_last) / (log_every if step > 1 else 1), 5)}),
                  file=out, flush=True)
        t_last = now

    def checkpoint(ep, batches_done):
        if ck_path is not None:
            save_checkpoint(ck_path, trainer, ep, batches_done,
                            {"num_tokens_local": int(ntok.count)})

    for epoch in range(start_epoch, max_epochs):
        if hasattr(loader.sampler, "set_epoch"):
            loader.sampler.set_epoch(epoch)  # EpochSampler: forwarded to the DistributedSampler
        else:
            sampler.set_epoch(epoch)
        ppl.reset()
        n_batches = len(loader)
        if isinstance(limit, float) and limit <= 1.0:
            n_batches = max(1, int(n_batches * limit))
        elif limit:
            n_batches = min(n_batches, int(limit))
        micro = []
        bi = -1
        for bi, ((masked, mask, labels), target) in enumerate(loader):
            if bi >= n_batches:
                bi -= 1
                break
            if bi < skip_batches:  # mid-epoch resume: these batches were consumed before
                continue
            micro.append((DeviceBatch.from_host(masked, mask, labels, target, device, pad_id),
                          target.numel()))
            if len(micro) < accum:
                continue
            loss = optimizer_step(micro)
            micro = []
            step = trainer.global_step
            if step % log_every == 0 or step == 1:
                log_line(loss)  # every rank joins the metric all-reduce
            if step % ck_every == 0:
                checkpoint(epoch, bi + 1)
            if max_steps and step >= int(max_steps):
                done = True
                break
        if micro and not done:  # Lightning steps on the epoch's last, partial accumulation
            loss = optimizer_step(micro)
            log_line(loss)
        skip_batches = 0
        # epoch finished (or max_steps reached inside it): resume starts at the next batch
        checkpoint(epoch + 1, 0) if not done else checkpoint(epoch, bi + 1)
        if done:
            break
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    return trainer


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--config-dir", default=os.environ.get("DNA_CONFIG_DIR",
                                                           os.path.join(ROOT, "configs")))
    ap.add_argument("--config-name", default="config")
    ap.add_argument("--dry-run", action="store_true", help="compose + build, no training")
    ap.add_argument("--print-config", action="store_true")
    ap.add_argument("overrides", nargs="*")
    a = ap.parse_args(argv)
    cfg = compose(a.config_dir, a.config_name, a.overrides)
    if a.print_config:
        print(json.dumps(cfg.to_container(skip_errors=True), indent=1, default=str))
    return train(cfg, dry_run=a.dry_run)


if __name__ == "__main__":
    main()
