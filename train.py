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
  * one process per device: `trainer.devices=N` (N > 1) without a launcher starts N rank
    processes of this script (dna_amd.launch, as Lightning's DDP does for the reference,
    train.py:630-639); under a launcher WORLD_SIZE must equal devices x num_nodes;
  * evaluation (train.py:339-406,442-460,547-596): after every training epoch (and when
    train.max_steps ends the run) the val and test loaders run forward-only on the same kernels
    (dropout off, compact masked rows, no dense logits), each rank on its DistributedSampler
    shard, logging {val,test}/{loss,perplexity,num_tokens} through one packed all-reduce;
    `train.validate_at_start` and `train.test` (final/val, final/test) as the reference;
  * ModelCheckpoint (configs/callbacks/checkpoint.yaml): the top-1 checkpoint by
    callbacks.model_checkpoint.monitor (${train.monitor}, e.g. test/loss, mode min) saved as
    <dirpath>/<filename>.ckpt (filename defaults to the monitor name, so test/loss.ckpt), plus
    last.ckpt; the best score survives a resume;
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


def _progress(n):
    """A Lightning 1.8 `Progress` state dict whose trackers all stand at n (ready == started ==
    processed == completed: the counted units finished); `total` = `current` here, since the
    run's earlier epochs are not kept per batch."""
    t = {"ready": int(n), "started": int(n), "processed": int(n), "completed": int(n)}
    return {"total": dict(t), "current": dict(t)}


def save_checkpoint(path, trainer, epoch, batches_done=0, metrics=None, best=None):
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
                      "metrics": metrics or {}},
          # the two Lightning loop counters the reference's fault-tolerant data modules read on
          # resume (genomics.py:1249-1253), as whole Lightning 1.8 Progress / BatchProgress
          # states (total + current trackers), so Loop._load_from_state_dict can restore them
          "loops": {"fit_loop": {"epoch_progress": _progress(epoch),
                                 "epoch_loop.batch_progress": dict(_progress(batches_done),
                                                                   is_last_batch=False)}}}
    if best is not None:  # ModelCheckpoint state, keyed and typed as Lightning 1.8 keeps it
        ck["callbacks"] = {best.state_key: best.state_dict()}
    os.makedirs(os.path.dirname(path) or ".", exist_ok=True)
    tmp = path + ".tmp"
    torch.save(ck, tmp)
    os.replace(tmp, path)


def n_devices(tr):
    """Processes the run wants: trainer.devices (an int, or a list of device ids as in the
    reference, train.py:631-633) x trainer.num_nodes (one node only here)."""
    d = tr.get("devices", 1)
    if isinstance(d, (list, tuple)) or hasattr(d, "to_container"):
        d = len(list(d))
    elif d in (None, "auto", -1, "-1"):
        d = max(1, torch.cuda.device_count())  # counts devices without initialising HIP
    nodes = int(tr.get("num_nodes", 1) or 1)
    if nodes != 1:
        raise NotImplementedError(f"trainer.num_nodes={nodes}: one node (up to 8 MI355X) only")
    return int(d)


class BestCheckpoint:
    """ModelCheckpoint(monitor, mode, save_top_k=1, filename) of configs/callbacks/checkpoint.yaml:
    keeps the best-so-far file <dirpath>/<filename>.ckpt (Lightning's format_checkpoint_name with
    auto_insert_metric_name=False: the filename is the monitor name, "/" making a sub-directory),
    overwritten in place whenever the monitored value improves."""

    def __init__(self, dirpath, monitor, mode="min", filename=None, save_top_k=1,
                 every_n_train_steps=None, every_n_epochs=None):
        if mode not in ("min", "max"):
            raise ValueError(f"model_checkpoint.mode={mode!r}: min or max")
        self.monitor, self.mode = monitor, mode
        self.enabled = bool(monitor) and int(save_top_k) != 0
        if self.enabled and int(save_top_k) != 1:
            raise NotImplementedError(f"model_checkpoint.save_top_k={save_top_k} (1 or 0)")
        self.path = os.path.join(dirpath, (filename or monitor or "best") + ".ckpt")
        self.dirpath = dirpath
        # Lightning 1.8 ModelCheckpoint.__init_triggers: every_n_epochs defaults to 1 only when
        # no trigger at all is given, otherwise a missing one counts as 0
        if every_n_train_steps is None and every_n_epochs is None:
            self.every_n_epochs, self.every_n_train_steps = 1, 0
        else:
            self.every_n_epochs = int(every_n_epochs or 0)
            self.every_n_train_steps = int(every_n_train_steps or 0)
        self.score = None

    @property
    def state_key(self):
        """Lightning 1.8's ModelCheckpoint.state_key: class name + repr of the identifying
        arguments, so Lightning's resume_from_checkpoint finds this entry."""
        return "ModelCheckpoint" + repr({"monitor": self.monitor, "mode": self.mode,
                                         "every_n_train_steps": self.every_n_train_steps,
                                         "every_n_epochs": self.every_n_epochs,
                                         "train_time_interval": None})

    def state_dict(self):
        score = None if self.score is None else torch.tensor(float(self.score))
        return {"monitor": self.monitor, "best_model_score": score,
                "best_model_path": self.path, "current_score": score, "dirpath": self.dirpath,
                "best_k_models": {self.path: score} if score is not None else {},
                "kth_best_model_path": self.path if score is not None else "",
                "kth_value": score, "last_model_path": ""}

    def load_from_checkpoint(self, ck):
        """Best score from a checkpoint's callbacks: Lightning's state-key entry (tensor score),
        or the plain "ModelCheckpoint" entry of round-4 checkpoints (float score)."""
        cbs = ck.get("callbacks") or {}
        st = cbs.get(self.state_key)
        if st is None:
            st = next((v for k, v in cbs.items() if k.startswith("ModelCheckpoint")
                       and isinstance(v, dict) and v.get("monitor") == self.monitor), None)
        if st is None or st.get("monitor", self.monitor) != self.monitor:
            return
        sc = st.get("best_model_score")
        self.score = None if sc is None else float(sc)

    def improves(self, value):
        if self.score is None:
            return True
        return value < self.score if self.mode == "min" else value > self.score


def eval_loaders(cfg, ds, world, rank, final=False):
    """The reference's _eval_dataloaders (train.py:559-582): val then test loaders, named
    "val" / "test" ("final/val" / "final/test" for trainer.test), one dropped by
    train.remove_test_loader_in_eval / remove_val_loader_in_eval. Each rank reads its
    DistributedSampler shard (Lightning replaces the eval samplers under DDP, shuffle off)."""
    from torch.utils.data.distributed import DistributedSampler
    out = []
    for name, dset, make in (("val", ds.dataset_val, ds.val_dataloader),
                             ("test", ds.dataset_test, ds.test_dataloader)):
        if name == "test" and cfg.train.get("remove_test_loader_in_eval", False):
            continue
        if name == "val" and cfg.train.get("remove_val_loader_in_eval", False):
            continue
        if len(dset) == 0:
            warnings.warn(f"{name} split is empty; skipped in evaluation")
            continue
        sampler = DistributedSampler(dset, num_replicas=world, rank=rank, shuffle=False)
        out.append((("final/" if final else "") + name, make(sampler=sampler)))
    return out


def params_log(model, pcfg):
    """ParamsLog.on_fit_start (src/callbacks/params.py:26-37, on the hot-path callback list
    configs/callbacks/base.yaml): params/total, params/trainable, params/fixed, each switched by
    the callback's total / trainable / fixed flags."""
    pcfg = pcfg.to_container() if hasattr(pcfg, "to_container") else dict(pcfg or {})
    ps = list(model.parameters())
    logs = {}
    if pcfg.get("total", True):
        logs["params/total"] = sum(p.numel() for p in ps)
    if pcfg.get("trainable", True):
        logs["params/trainable"] = sum(p.numel() for p in ps if p.requires_grad)
    if pcfg.get("fixed", True):
        logs["params/fixed"] = sum(p.numel() for p in ps if not p.requires_grad)
    return logs


def eval_batches(n, limit):
    """Batches Lightning runs of an n-batch loader under limit_{val,test}_batches: a float is a
    fraction (at least one batch when it is > 0), an int a count; 0 / 0.0 disables the loop."""
    if limit is None:
        return n
    if isinstance(limit, float) and limit <= 1.0:
        if limit <= 0.0:
            return 0
        return max(1, int(n * limit)) if n else 0
    return min(n, max(0, int(limit)))


def evaluate(trainer, loaders, device, pad_id, limit=1.0, tokens=None):
    """validation_step / test_step through _shared_step (train.py:339-380, 442-460) for the MLM
    task: forward-only on the training kernels in eval mode (dropout off), the task loss
    bert_cross_entropy on the compact masked rows (no dense [b, S, V] logits), per loader
      <name>/loss        batch-size-weighted mean over all batches of all ranks (Lightning's
                         on_epoch mean with sync_dist)
      <name>/perplexity  exp(sum loss*numel / sum numel) over the epoch (Perplexity, reset per
                         evaluation, torchmetrics.py:24-73)
      <name>/num_tokens  running target-token count (NumTokens, never reset: `tokens` carries it)
    All sums of all loaders travel in ONE all-reduce. Returns {metric: float}."""
    from dna_amd.ddp import reduce_metrics
    from dna_amd.trainer import DeviceBatch
    model = trainer.model
    was_training = model.training
    model.eval()
    tokens = tokens if tokens is not None else {}
    sums, names = [], []
    try:
        with torch.no_grad():
            for name, loader in loaders:
                n = eval_batches(len(loader), limit)
                loss_w = torch.zeros((), dtype=torch.float64, device=device)
                nll = torch.zeros((), dtype=torch.float64, device=device)
                bs_sum, numel_sum = 0, 0
                for bi, ((masked, mask, labels), target) in enumerate(loader):
                    if bi >= n:
                        break
                    db = DeviceBatch.from_host(masked, mask, labels, target, device, pad_id)
                    loss, _ = model.mlm_loss(db.masked_ids, db.mask, db.index, db.n_mask,
                                             db.n_unk_masked)
                    bs, numel = int(target.shape[0]), int(target.numel())
                    loss_w += loss.double() * bs
                    nll += loss.double() * numel
                    bs_sum += bs
                    numel_sum += numel
                tokens[name] = tokens.get(name, 0) + numel_sum
                sums += [loss_w, bs_sum, nll, numel_sum, tokens[name]]
                names.append(name)
    finally:
        model.train(was_training)
    if not names:
        return {}
    _, g = reduce_metrics(torch.zeros(()), 0, extra=sums)
    res = {}
    for i, name in enumerate(names):
        lw, bs, nl, ne, tk = g[5 * i: 5 * i + 5]
        if bs == 0:
            # no rank ran a batch of this loader (a zero limit, or drop_last shards smaller than
            # the eval batch): nothing is logged -- a made-up 0.0 loss would become the best score
            continue
        res[f"{name}/loss"] = lw / bs
        res[f"{name}/perplexity"] = math.exp(nl / max(ne, 1))
        res[f"{name}/num_tokens"] = int(round(tk))
    return res


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

    want = n_devices(tr)
    if want != world:
        raise ValueError(f"trainer.devices={want} but WORLD_SIZE={world}: start the run with "
                         f"`python train.py ...` (it launches one process per device) or a "
                         f"launcher with --nproc-per-node {want}")
    from dna_amd.launch import init_rank_process_group, rank_device_index, wants_process_group
    use_pg = wants_process_group(world)  # DNA_DDP_FORCE=1: the RCCL leg at world 1 too
    if use_pg:
        device = init_rank_process_group(local)
    else:
        device = torch.device("cuda", rank_device_index(local))
    torch.cuda.set_device(device)
    if rank == 0:
        print(json.dumps({"event": "start", "world": world, "parallelism": f"dp{world}",
                          "backend": dist.get_backend() if use_pg else None,
                          "global_batch": int(cfg.dataset.get("batch_size", 0) or 0) * world}),
              file=out, flush=True)
    ck_cfg = cfg.get("callbacks", {}) or {}
    timer_cfg = (ck_cfg.get("timer") if ck_cfg else None) or {}  # configs/callbacks/base.yaml
    if rank == 0 and ck_cfg and ck_cfg.get("params") is not None:
        print(json.dumps(dict({"event": "params"}, **params_log(model, ck_cfg.params))),
              file=out, flush=True)
    wire = str(tr.get("grad_wire", "fp32") or "fp32")
    trainer = MLMTrainer(model, device, lr=float(opt.lr),
                         weight_decay=float(opt.get("weight_decay", 0.0)),
                         betas=tuple(opt.get("betas", (0.9, 0.999))),
                         max_grad_norm=float(tr.get("gradient_clip_val", 0.0) or 0.0),
                         scheduler=sched, seed=seed, wire_dtype=wire)
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
            if "batches_done" not in extra and "loops" in ck and \
                    getattr(ds, "fault_tolerant", False) and hasattr(ds, "load_state_dict"):
                # a reference / Lightning checkpoint: the data module reads the fit loop's
                # counters (genomics.py:1249-1253) and the sampler fast-forwards from them
                ds.load_state_dict(ck)
                start_epoch = int(ds.fast_forward_epochs)
                skip_batches = int(ds.fast_forward_batches)
        else:
            warnings.warn(f"resume checkpoint {resume} not found; training from scratch")

    # the permutation is randperm(seed + epoch) on every world size (DistributedSampler
    # semantics), so a mid-epoch resume replays exactly the interrupted epoch's
    # order, and the masks are keyed on (train.seed, epoch, window) (EpochSampler)
    fault_tolerant = bool(getattr(ds, "fault_tolerant", False))
    sampler_cls = torch.utils.data.distributed.DistributedSampler
    if fault_tolerant:
        # the reference's FaultTolerantDistributedSampler (fault_tolerant_sampler.py:64-122,
        # genomics.py:1208-1217): a resume skips the consumed indices in the sampler, so the
        # loader never reads / tokenises them
        from dna_amd.hg38 import FaultTolerantDistributedSampler as sampler_cls
    sampler = sampler_cls(
        ds.dataset_train, num_replicas=world, rank=rank,
        shuffle=True if world > 1 else bool(getattr(ds, "shuffle", True)), seed=int(seed or 0))
    if fault_tolerant and skip_batches == 0 and getattr(ds, "fast_forward_epochs", None) is not None \
            and getattr(ds, "fast_forward_batches", None) is not None:
        # dataset.fast_forward_{epochs,batches} given in the config (genomics.py:1212-1217)
        start_epoch, skip_batches = int(ds.fast_forward_epochs), int(ds.fast_forward_batches)
    if seed is not None and hasattr(ds.dataset_train, "mask_seed"):
        ds.dataset_train.mask_seed = (int(seed) * 0x9E3779B1 + 2222) & (2 ** 63 - 1)
    loader = ds.train_dataloader(sampler=sampler)
    accum = int(tr.get("accumulate_grad_batches", 1) or 1)
    max_steps = cfg.train.get("max_steps") or tr.get("max_steps")
    max_epochs = int(tr.get("max_epochs", 1) or 1)
    log_every = int(tr.get("log_every_n_steps", 10) or 10)
    limit = tr.get("limit_train_batches", 1.0)
    pad_id = getattr(ds.tokenizer, "pad_token_id", 3)
    mc = ck_cfg.get("model_checkpoint") if ck_cfg else None
    ck_path, best = None, None
    if mc is not None:
        d = mc.get("dirpath", "checkpoints/")
        if rank == 0:
            os.makedirs(d, exist_ok=True)
        if mc.get("save_last", True):
            ck_path = os.path.join(d, "last.ckpt")
        # configs/callbacks/checkpoint.yaml: monitor ${train.monitor}, mode ${train.mode},
        # save_top_k 1, filename ${train.monitor}
        monitor = mc.get("monitor", cfg.train.get("monitor"))
        best = BestCheckpoint(d, monitor, mode=mc.get("mode", cfg.train.get("mode", "min")),
                              filename=mc.get("filename", monitor),
                              save_top_k=mc.get("save_top_k", 1),
                              every_n_train_steps=mc.get("every_n_train_steps"),
                              every_n_epochs=mc.get("every_n_epochs"))
        if resume and os.path.exists(resume):
            best.load_from_checkpoint(ck)
    ck_every = int((mc.get("every_n_train_steps") if mc is not None else 0) or 1000)
    limit_val = tr.get("limit_val_batches", 1.0)
    limit_test = tr.get("limit_test_batches", 1.0)
    eval_tokens = {}  # NumTokens per eval loader: never reset (torchmetrics.py:75-115)
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
                              "trainer/loss": round(lv, 5), "trainer/epoch": epoch,
                              "train/perplexity": round(math.exp(sums[0] / max(sums[1], 1)), 4),
                              "train/num_tokens": int(sums[2]),
                              "trainer/lr": trainer.opt.param_groups[0]["lr"],
                              "timer/step": round((now - t_last) / (log_every if step > 1 else 1), 5)}),
                  file=out, flush=True)
        t_last = now

    eval_cache = {}

    def run_eval(final=False):
        if final not in eval_cache:  # built once: persistent workers live across epochs
            eval_cache[final] = eval_loaders(cfg, ds, world, rank, final=final)
        loaders = eval_cache[final]
        lim = limit_test if final else limit_val
        if lim is not None and not isinstance(lim, bool) and float(lim) == 0.0:
            return {}  # limit_{val,test}_batches=0: the evaluation loop is disabled
        t_val = time.perf_counter()
        res = evaluate(trainer, loaders, device, pad_id,
                       limit=limit_test if final else limit_val, tokens=eval_tokens)
        if res and not final and timer_cfg.get("val", True):
            # Timer.on_validation_epoch_end (src/callbacks/timer.py:91-96)
            res = dict(res, **{"timer/validation": round(time.perf_counter() - t_val, 5)})
        if rank == 0 and res:
            print(json.dumps(dict({"step": trainer.global_step, "epoch": epoch},
                                  **{k: (round(v, 6) if isinstance(v, float) else v)
                                     for k, v in res.items()})), file=out, flush=True)
        return res

    def checkpoint(ep, batches_done, metrics=None):
        """last.ckpt, and the monitored top-1 file when `metrics` (an evaluation) improve it.
        Rank 0 writes; every rank keeps the same best score (the metrics are all-reduced)."""
        state = {"num_tokens_local": int(ntok.count)}
        if best is not None and best.enabled and metrics:
            if best.monitor not in metrics:
                warnings.warn(f"model_checkpoint.monitor={best.monitor!r} was not logged "
                              f"(have {sorted(metrics)}); no best checkpoint")
            elif best.improves(metrics[best.monitor]):
                best.score = float(metrics[best.monitor])
                if rank == 0:
                    save_checkpoint(best.path, trainer, ep, batches_done, state, best)
                    print(json.dumps({"step": trainer.global_step, "checkpoint": best.path,
                                      best.monitor: best.score}), file=out, flush=True)
        if ck_path is not None and rank == 0:
            save_checkpoint(ck_path, trainer, ep, batches_done, state, best)

    if cfg.train.get("validate_at_start", False):  # trainer.validate(model), train.py:684-687
        run_eval()

    for epoch in range(start_epoch, max_epochs):
        t_epoch = time.perf_counter()  # Timer.on_train_epoch_start (src/callbacks/timer.py:38-41)
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
        first = 0
        if fault_tolerant and skip_batches:
            # mid-epoch resume in the sampler: this rank's first skip_batches * batch_size
            # indices of the epoch's permutation are not yielded again
            sampler.load_state_dict({"epoch": epoch, "counter": skip_batches * int(ds.batch_size)})
            first, skip_batches = skip_batches, 0
        bi = first - 1
        for bi, ((masked, mask, labels), target) in enumerate(loader, start=first):
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
        # end of the epoch (or of the run at max_steps): the validation epoch (val + test
        # loaders), then ModelCheckpoint on its metrics; a resume starts at the next batch
        metrics = run_eval()
        if rank == 0 and timer_cfg.get("epoch", True):
            # Timer.on_train_epoch_end (src/callbacks/timer.py:80-86); Lightning 1.8 calls it
            # after the epoch-end validation loop, so the epoch time includes it
            print(json.dumps({"step": trainer.global_step, "epoch": epoch,
                              "timer/epoch": round(time.perf_counter() - t_epoch, 5)}),
                  file=out, flush=True)
        checkpoint(epoch + 1, 0, metrics) if not done else checkpoint(epoch, bi + 1, metrics)
        if done:
            break
    if cfg.train.get("test", False):  # trainer.test(model) after fit, train.py:693-694
        run_eval(final=True)
    dump = os.environ.get("DNA_DUMP_PARAMS")
    if dump:  # debug: every rank's parameter digest (multi-rank tests compare them)
        from dna_amd.launch import flat_digest
        os.makedirs(dump, exist_ok=True)
        with open(os.path.join(dump, f"rank{rank}.json"), "w") as f:
            json.dump(dict(flat_digest(trainer.flat.flat), rank=rank, world=world,
                           global_step=trainer.global_step), f)
    if use_pg:
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
    want = n_devices(cfg.trainer)
    if want > 1 and "WORLD_SIZE" not in os.environ and not a.dry_run:
        # Lightning's DDP launch (train.py:630-639): one process per device, started before
        # this process touches the GPU; rank 0 prints the log stream
        from dna_amd.launch import launch_ranks
        sys.exit(launch_ranks(want, __file__, sys.argv[1:] if argv is None else list(argv)))
    return train(cfg, dry_run=a.dry_run)


if __name__ == "__main__":
    main()
