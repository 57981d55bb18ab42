"""train.py / config composition: our configs and (when present in this container) the reference's
own configs/ tree compose and build the run unchanged; GPU test runs real steps of config A."""
import io
import json
import os

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
    assert tr.global_step == 6 and logs[-1]["step"] == 6
    assert all(l["train/loss"] == l["train/loss"] for l in logs)  # finite
    assert os.path.exists(tmp_path / "checkpoints" / "last.ckpt")
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
