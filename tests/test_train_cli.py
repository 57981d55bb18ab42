"""train.py / config composition: our configs and (when present in this container) the reference's
own configs/ tree compose and build the run unchanged; GPU test runs real steps of config A."""
import io
import json
import math
import os
import subprocess
import sys

import pytest

from tests.conftest import ROOT

REF_CONFIGS = "/root/reference/configs"
CFG_A = ["trainer.devices=1", "model.config.num_hidden_layers=2", "model.config.hidden_size=128",
         "model.config.num_attention_heads=2", "model.config.intermediate_size=512",
         "dataset.max_length=1024", "dataset.pad_max_length=130", "dataset.batch_size=8",
         "dataset.num_workers=0", "wandb=null", "trainer.resume_from_checkpoint=null"]


@pytest.fixture(scope="module")
def data_root(tmp_path_factory):
    from dna_amd.synthetic import write_hg38
    root = tmp_path_factory.mktemp("data")
    write_hg38(str(root), n_chroms=2, chrom_len=200_000, max_length=1024)
    return str(root)


def _dry(config_dir, overrides, data_root, monkeypatch):
    import train
    from dna_amd.compose import compose
    monkeypatch.setenv("DATA_PATH", data_root)
    cfg = compose(config_dir, "config", ["experiment=dnabert2/dnabert2_hg38_pretrain"] + overrides)
    buf = io.StringIO()
    train.train(cfg, dry_run=True, out=buf)
    return cfg, json.loads(buf.getvalue())


def test_own_configs_compose_and_build(data_root, monkeypatch):
    cfg, res = _dry(os.path.join(ROOT, "configs"), CFG_A, data_root, monkeypatch)
    assert res["task"] == "bert_cross_entropy"
    assert cfg.trainer.accumulate_grad_batches == 4 and cfg.trainer.gradient_clip_val == 1.0
    assert cfg.optimizer.lr == 5e-4 and cfg.optimizer.weight_decay == 1e-5
    assert cfg.train.global_batch_size == 8
    assert res["scheduler"]["warmup_t"] == 120000 and res["scheduler"]["t_initial"] == 2000000
    assert res["train_windows"] > 0


@pytest.mark.skipif(not os.path.isdir(REF_CONFIGS), reason="reference configs not mounted")
def test_reference_configs_compose_unchanged(data_root, monkeypatch):
    """The reference's configs/experiment/dnabert2/dnabert2_hg38_pretrain.yaml (+ its defaults
    tree) composes through dna_amd.compose and builds the same run (config A overrides)."""
    cfg, res = _dry(REF_CONFIGS, CFG_A, data_root, monkeypatch)
    assert cfg.hydra_choices["scheduler"] == ["linear_warmup"]  # `override /scheduler`
    assert cfg.dataset.batch_size_eval == 16                      # ${eval:${.batch_size} * 2}
    assert cfg.train.global_batch_size == 8                       # ${eval:devices*batch}
    assert cfg.scheduler.t_initial == 2_000_000 and cfg.scheduler.warmup_t == 120_000
    assert cfg.optimizer.lr == 5e-4 and cfg.task.loss == "bert_cross_entropy"
    assert sorted(cfg.callbacks.keys()) == ["learning_rate_monitor", "model_checkpoint", "params",
                                            "timer"]
    assert res["model_params"] > 0


def test_cpu_accelerator_is_rejected(data_root, monkeypatch):
    import train
    from dna_amd.compose import compose
    monkeypatch.setenv("DATA_PATH", data_root)
    cfg = compose(os.path.join(ROOT, "configs"), "config", CFG_A + ["trainer.accelerator=cpu"])
    with pytest.raises(RuntimeError, match="GPU"):
        train.train(cfg, dry_run=True, out=io.StringIO())


def test_compose_overrides_and_resolvers(tmp_path):
    from dna_amd.compose import ConfigError, compose
    (tmp_path / "grp").mkdir()
    (tmp_path / "config.yaml").write_text(
        "defaults:\n  - _self_\n  - grp: a\nx: 1\nlr: 5e-4\nnested: {y: '${x}', z: '${.y}', "
        "w: '${div_up:10, 3}', e: '${eval:${x} + 41}', s: 'v${x}'}\nmiss: ???\n")
    (tmp_path / "grp" / "a.yaml").write_text("k: 1\n")
    (tmp_path / "grp" / "b.yaml").write_text("# @package _global_\nx: 7\n")
    c = compose(str(tmp_path), "config", [])
    assert c.grp.k == 1 and c.nested.y == 1 and c.nested.z == 1 and c.nested.w == 4
    assert c.nested.e == 42 and c.nested.s == "v1" and c.lr == 5e-4
    with pytest.raises(ConfigError):
        _ = c.miss
    c = compose(str(tmp_path), "config", ["grp=b", "+new.key=3", "~lr"])
    assert c.x == 7 and c.nested.e == 48 and c.new.key == 3 and "lr" not in c
    assert "grp" not in c


@pytest.mark.gpu
def test_train_config_a_runs_on_gpu(data_root, monkeypatch, tmp_path):
    import train
    from dna_amd.compose import compose
    monkeypatch.setenv("DATA_PATH", data_root)
    monkeypatch.chdir(tmp_path)
    cfg = compose(os.path.join(ROOT, "configs"), "config",
                  ["experiment=dnabert2/dnabert2_hg38_pretrain"] + CFG_A +
                  ["trainer.accumulate_grad_batches=2", "train.max_steps=6",
                   "trainer.log_every_n_steps=2"])
    buf = io.StringIO()
    tr = train.train(cfg, out=buf)
    logs = [json.loads(l) for l in buf.getvalue().splitlines()]
    assert logs[0]["event"] == "start" and logs[0]["world"] == 1
    train_logs = [l for l in logs if "train/loss" in l]
    assert tr.global_step == 6 and train_logs[-1]["step"] == 6
    assert all(l["train/loss"] == l["train/loss"] for l in train_logs)  # finite
    assert os.path.exists(tmp_path / "checkpoints" / "last.ckpt")
    # the validation epoch at the end of the run: val + test loaders, then ModelCheckpoint
    # (monitor test/loss, mode min) writes checkpoints/test/loss.ckpt
    ev = [l for l in logs if "val/loss" in l]
    assert len(ev) == 1 and ev[0]["step"] == 6
    # Timer callback (configs/callbacks/base.yaml: step, epoch, val) and trainer/epoch
    assert all(l["trainer/epoch"] == l["epoch"] for l in train_logs)
    assert ev[0]["timer/validation"] > 0
    te = [l for l in logs if "timer/epoch" in l]
    assert len(te) == 1 and te[0]["timer/epoch"] >= ev[0]["timer/validation"]
    for k in ("val/loss", "val/perplexity", "test/loss", "test/perplexity"):
        assert math.isfinite(ev[0][k]), k
    assert abs(ev[0]["val/perplexity"] - math.exp(ev[0]["val/loss"])) < 1e-3 * ev[0]["val/perplexity"]
    assert ev[0]["val/num_tokens"] > 0
    best = tmp_path / "checkpoints" / "test" / "loss.ckpt"
    assert os.path.exists(best)
    import torch
    ck = torch.load(best, map_location="cpu", weights_only=True)
    (key, st), = ck["callbacks"].items()  # Lightning 1.8's ModelCheckpoint state_key, tensor score
    assert key.startswith("ModelCheckpoint{'monitor': 'test/loss'")
    assert float(st["best_model_score"]) == pytest.approx(ev[0]["test/loss"])
    # resume from the Lightning-layout checkpoint
    cfg2 = compose(os.path.join(ROOT, "configs"), "config",
                   ["experiment=dnabert2/dnabert2_hg38_pretrain"] + CFG_A[:-1] +
                   [f"trainer.resume_from_checkpoint={tmp_path}/checkpoints/last.ckpt",
                    "train.max_steps=8", "trainer.accumulate_grad_batches=2"])
    tr2 = train.train(cfg2, out=io.StringIO())
    assert tr2.global_step == 8


@pytest.mark.parametrize("cdir", [os.path.join(ROOT, "configs"), REF_CONFIGS])
def test_text_corpus_experiment_builds(cdir, tmp_path, monkeypatch):
    """experiment=dnabert2/dnabert2_pretrain (text corpus) composes from our
    configs and, when mounted here, the reference's, and builds the dnabert2_pretrain data module."""
    if not os.path.isdir(cdir):
        pytest.skip("reference configs not mounted")
    import numpy as np
    import train
    from dna_amd.compose import compose
    z = np.load(os.path.join(ROOT, "tests", "golden", "corpus_golden.npz"))
    d = tmp_path / "dnabert2"
    d.mkdir()
    for split in ("train", "dev"):
        (d / f"{split}.txt").write_text("\n".join(str(s) for s in z["lines"]) + "\n")
    cfg = compose(cdir, "config", ["experiment=dnabert2/dnabert2_pretrain", "trainer.devices=1",
                                   "dataset.num_workers=0", "wandb=null",
                                   "trainer.resume_from_checkpoint=null", f"dataset.text_file={d}"])
    buf = io.StringIO()
    train.train(cfg, dry_run=True, out=buf)
    res = json.loads(buf.getvalue())
    assert res["train_windows"] == len(z["lines"]) and cfg.dataset.max_length == 128
    assert list(cfg.optimizer.betas) == [0.9, 0.98] and cfg.scheduler.warmup_t == 60000


def test_devices_world_size_mismatch_raises(data_root, monkeypatch):
    """trainer.devices must equal the launcher's WORLD_SIZE (the reference's Lightning would
    start `devices` processes; a silent one-GPU run is an error here)."""
    import train
    from dna_amd.compose import compose
    monkeypatch.setenv("DATA_PATH", data_root)
    monkeypatch.setenv("WORLD_SIZE", "2")
    cfg = compose(os.path.join(ROOT, "configs"), "config", CFG_A)
    with pytest.raises(ValueError, match="WORLD_SIZE"):
        train.train(cfg, out=io.StringIO())
    monkeypatch.delenv("WORLD_SIZE")
    assert train.n_devices(compose(os.path.join(ROOT, "configs"), "config",
                                   CFG_A + ["trainer.devices=[0,3]"]).trainer) == 2


def _two_rank_env(data_root, dump):
    env = dict(os.environ, DATA_PATH=data_root, DNA_DIST_BACKEND="gloo", DNA_DUMP_PARAMS=dump,
               PYTHONUNBUFFERED="1")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT"):
        env.pop(k, None)
    return env


def _digests(dump, n):
    ds = [json.load(open(os.path.join(dump, f"rank{r}.json"))) for r in range(n)]
    assert all(d["world"] == n for d in ds)
    return ds


@pytest.mark.gpu
def test_train_devices_2_starts_two_ranks(data_root, tmp_path):
    """`python train.py ... trainer.devices=2` without a launcher starts two rank processes (the
    reference's Lightning DDP launch, train.py:630-639) that train the config-A model together:
    one log stream (rank 0) with world=2, identical parameters on both ranks afterwards, the
    evaluation epoch and the monitored checkpoint. gloo backend: both ranks share the one GPU
    of the test box (the RCCL run is the driver's 8-GPU bench)."""
    dump = str(tmp_path / "dump")
    cmd = [sys.executable, os.path.join(ROOT, "train.py"), "experiment=dnabert2/dnabert2_hg38_pretrain"] + \
        [o for o in CFG_A if not o.startswith("trainer.devices")] + \
        ["trainer.devices=2", "train.max_steps=3", "trainer.accumulate_grad_batches=1",
         "trainer.log_every_n_steps=1"]
    r = subprocess.run(cmd, cwd=str(tmp_path), env=_two_rank_env(data_root, dump),
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    logs = [json.loads(l) for l in r.stdout.splitlines() if l.startswith("{")]
    assert logs[0]["event"] == "start" and logs[0]["world"] == 2 and logs[0]["parallelism"] == "dp2"
    steps = [l["step"] for l in logs if "train/loss" in l]
    assert steps == [1, 2, 3]  # one stream: rank 0 prints, every step once
    assert all(math.isfinite(l["train/loss"]) for l in logs if "train/loss" in l)
    assert any("test/loss" in l for l in logs)
    d0, d1 = _digests(dump, 2)
    assert d0["global_step"] == d1["global_step"] == 3
    assert d0["sha256"] == d1["sha256"], (d0, d1)
    assert os.path.exists(tmp_path / "checkpoints" / "test" / "loss.ckpt")


@pytest.mark.gpu
@pytest.mark.parametrize("ranks", [2, 8])
def test_bench_multi_rank_real_model(tmp_path, ranks):
    """bench.py's own world > 1 path with the real DNABERT-2 step (not the --dist-dry-run
    skeleton): process group init, the model step with GradBucketReducer, max-over-ranks timing,
    one JSON line from rank 0 -- gloo ranks on the test box's GPU. ranks=8 rehearses the
    driver's SCALE command (`bench.py --gpus 8`: the launcher, 8 children, the port, the
    rank -> device binding) with every rank bound to the one visible GPU."""
    dump = str(tmp_path / "dump")
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(ranks), "--steps", "2",
           "--warmup", "1", "--batch", "8", "--no-cpu-baseline", "--no-b64", "--no-data-pipeline",
           "--dump-params", dump]
    env = _two_rank_env("", dump)
    env.pop("DNA_DUMP_PARAMS")
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    log = os.path.join(ROOT, "gpurun_out", f"bench_{ranks}rank.log")  # visible while it runs
    with open(log, "w") as err:
        r = subprocess.run(cmd, cwd=ROOT, env=env, stdout=subprocess.PIPE, stderr=err, text=True,
                           timeout=400)
    assert r.returncode == 0, open(log).read()[-3000:]
    assert len(r.stdout.strip().splitlines()) == 1, r.stdout  # ONE line: RCCL / gloo talk -> stderr
    lines = [json.loads(l) for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1
    line = lines[0]
    assert line["n_gpus"] == ranks and line["config"]["parallelism"] == f"dp{ranks}"
    assert line["config"]["global_batch"] == 8 * ranks and line["value"] > 0
    assert math.isfinite(line["final_loss"])
    ds = _digests(dump, ranks)
    assert len({d["sha256"] for d in ds}) == 1, ds
    assert all(d["global_step"] == ds[0]["global_step"] for d in ds)


@pytest.mark.gpu
@pytest.mark.parametrize("fault_tolerant", [False, True])
def test_mid_epoch_resume_replays_the_uninterrupted_run(data_root, monkeypatch, tmp_path,
                                                        fault_tolerant):
    """Stop after 2 optimizer steps, resume from last.ckpt, run 2 more: steps 3-4 log the same
    losses as an uninterrupted 4-step run. fault_tolerant=True (the reference's
    FaultTolerantDistributedSampler, fault_tolerant_sampler.py:64-122) resumes inside the sampler
    -- the consumed windows are never read again -- and the checkpoint carries the Lightning loop
    counters its data modules read (genomics.py:1249-1253)."""
    import torch
    import train
    from dna_amd.compose import compose
    monkeypatch.setenv("DATA_PATH", data_root)
    ft = [f"+dataset.fault_tolerant={str(fault_tolerant).lower()}"]
    base = ["experiment=dnabert2/dnabert2_hg38_pretrain"] + CFG_A[:-1] + ft + \
        ["trainer.accumulate_grad_batches=1", "trainer.log_every_n_steps=1",
         "trainer.limit_val_batches=0", "trainer.limit_test_batches=0"]

    def run(d, steps, resume=None):
        monkeypatch.chdir(d)
        extra = [f"trainer.resume_from_checkpoint={resume}" if resume else
                 "trainer.resume_from_checkpoint=null", f"train.max_steps={steps}"]
        buf = io.StringIO()
        train.train(compose(os.path.join(ROOT, "configs"), "config", base + extra), out=buf)
        logs = [json.loads(l) for l in buf.getvalue().splitlines()]
        assert not any("val/loss" in l for l in logs)  # limit_val_batches=0: no evaluation
        return {l["step"]: l["train/loss"] for l in logs if "train/loss" in l}

    (tmp_path / "a").mkdir()
    (tmp_path / "b").mkdir()
    full = run(tmp_path / "a", 4)
    first = run(tmp_path / "b", 2)
    ck = torch.load(tmp_path / "b" / "checkpoints" / "last.ckpt", map_location="cpu",
                    weights_only=True)
    assert ck["loops"]["fit_loop"]["epoch_loop.batch_progress"]["current"]["completed"] == 2
    ck_path = tmp_path / "b" / "checkpoints" / "last.ckpt"
    if fault_tolerant:
        # a reference / Lightning checkpoint has the loop counters but not this engine's
        # batches_done: the data module's load_state_dict fast-forwards from the counters
        lt = dict(ck, dna_amd={k: v for k, v in ck["dna_amd"].items() if k != "batches_done"})
        (tmp_path / "c").mkdir()
        torch.save(lt, tmp_path / "c" / "loops_only.ckpt")
    rest = run(tmp_path / "b", 4, resume=str(ck_path))
    assert first == {1: full[1], 2: full[2]}
    assert rest == {3: full[3], 4: full[4]}, (rest, full)
    if fault_tolerant:
        rest2 = run(tmp_path / "c", 4, resume=str(tmp_path / "c" / "loops_only.ckpt"))
        assert rest2 == {3: full[3], 4: full[4]}, (rest2, full)
