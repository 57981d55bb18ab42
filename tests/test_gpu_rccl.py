"""The RCCL leg of configs C / E on the one GPU a test box has.

A world-1 process group on the "nccl" backend (RCCL) runs everything the 8-GPU data-parallel step
runs except the xGMI transfer: `init_process_group("nccl", device_id=...)`, the construction
broadcast, GradBucketReducer's per-bucket async all_reduce on RCCL's stream (fired from inside the
backward), finish()'s waits, the bf16 wire's cast-back, and the packed metric all-reduce. With one
rank the SUM is the identity: reduced gradients == reducer-off gradients bit for bit (fp32 wire;
DNABERT-2's kernels are deterministic) or == their bf16 rounding (bf16 wire). Caduceus' scan
backward sums dB / dC with float atomics, so its two backward passes agree to rounding only.
Reference: Lightning DDP, /root/reference/train.py:630-639 (strategy: ddp)."""
import json
import math
import os
import subprocess
import sys

import pytest

from tests.conftest import ROOT

pytestmark = pytest.mark.gpu


def _env(**kw):
    from dna_amd.launch import free_port
    env = dict(os.environ, RANK="0", LOCAL_RANK="0", WORLD_SIZE="1", LOCAL_WORLD_SIZE="1",
               MASTER_ADDR="127.0.0.1", MASTER_PORT=str(free_port()), DNA_DDP_FORCE="1",
               PYTHONUNBUFFERED="1")
    env.pop("DNA_DIST_BACKEND", None)  # nccl (RCCL)
    env.update(kw)
    return env


def _run(cmd, env, cwd=ROOT, timeout=600):
    r = subprocess.run(cmd, cwd=cwd, env=env, capture_output=True, text=True, timeout=timeout)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-4000:])
    return [json.loads(l) for l in r.stdout.splitlines() if l.startswith("{")]


@pytest.fixture(scope="module")
def world1():
    res = _run([sys.executable, os.path.join(ROOT, "scripts", "rccl_world1.py")], _env())
    return {r["model"].split("-")[0]: r for r in res}


def test_dnabert2_buckets_over_rccl_equal_reducer_off(world1):
    r = world1["dnabert2"]
    assert r["backend"] == "nccl"
    assert r["n_buckets"] >= 10                      # 468 MB in 25-MB buckets
    assert r["fired_in_backward"] == r["n_buckets"]  # every bucket launched inside the backward
    assert r["fp32_wire_bit_equal"], r
    assert r["first_step_max_abs_diff"] == 0.0       # the unoverlapped first step, too
    assert r["bf16_wire_vs_rounded_max_abs_diff"] == 0.0, r
    assert r["bf16_wire_vs_fp32_max_rel"] < 2 ** -7
    assert all(math.isfinite(x) for x in r["step_losses"])


def test_caduceus_buckets_over_rccl_equal_reducer_off(world1):
    r = world1["caduceus"]
    assert r["backend"] == "nccl" and r["n_buckets"] >= 2
    assert r["fired_in_backward"] >= 1
    # dB / dC float atomics in the scan backward: two bf16-autocast backward passes agree to
    # rounding (measured 1.1e-5 of the largest gradient)
    assert r["fp32_wire_max_abs_diff"] <= 1e-4 * r["grad_abs_max"], r
    assert r["bf16_wire_vs_fp32_max_rel"] < 2 ** -7, r
    assert all(math.isfinite(x) for x in r["step_losses"])


def test_bench_world1_rccl_bf16_wire():
    """bench.py's data-parallel path at world 1 over RCCL, bf16 wire, strict native mode."""
    lines = _run([sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "3", "--warmup", "1",
                  "--batch", "16", "--grad-wire", "bf16", "--no-cpu-baseline", "--no-b64",
                  "--no-data-pipeline"], _env())
    assert len(lines) == 1
    line = lines[0]
    assert line["config"]["grad_allreduce"] is True and line["config"]["grad_wire"] == "bf16"
    # RCCL writes its init banner to stdout; bench.py routes it to stderr so the driver reads
    # exactly one line (round 6: the banner broke a JSON parse of the RCCL arm)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "2", "--warmup",
                        "1", "--batch", "16", "--no-cpu-baseline", "--no-b64",
                        "--no-data-pipeline", "--no-kernel-timing"],
                       cwd=ROOT, env=_env(NCCL_DEBUG="WARN"), capture_output=True, text=True,
                       timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    assert len(r.stdout.strip().splitlines()) == 1, r.stdout[:2000]
    json.loads(r.stdout)
    assert line["native_only"] is True and line["value"] > 0
    assert math.isfinite(line["final_loss"])


def test_train_world1_rccl_bf16_wire(tmp_path):
    """train.py with trainer.grad_wire=bf16 over a world-1 RCCL group: steps, the packed metric
    all-reduce, the evaluation epoch (its CPU placeholder loss goes to the device for RCCL) and
    the ParamsLog line."""
    from dna_amd.synthetic import write_hg38
    data = tmp_path / "data"
    write_hg38(str(data), n_chroms=2, chrom_len=200_000, max_length=1024)
    cmd = [sys.executable, os.path.join(ROOT, "train.py"), "experiment=dnabert2/dnabert2_hg38_pretrain",
           "trainer.devices=1", "model.config.num_hidden_layers=2", "model.config.hidden_size=128",
           "model.config.num_attention_heads=2", "model.config.intermediate_size=512",
           "dataset.max_length=1024", "dataset.pad_max_length=130", "dataset.batch_size=8",
           "dataset.num_workers=0", "wandb=null", "trainer.resume_from_checkpoint=null",
           "train.max_steps=3", "trainer.accumulate_grad_batches=1", "trainer.log_every_n_steps=1",
           "+trainer.grad_wire=bf16"]
    logs = _run(cmd, _env(DATA_PATH=str(data)), cwd=str(tmp_path))
    assert logs[0]["event"] == "start" and logs[0]["backend"] == "nccl"
    params = [l for l in logs if l.get("event") == "params"]
    assert params and params[0]["params/total"] == params[0]["params/trainable"] > 0
    assert [l["step"] for l in logs if "train/loss" in l] == [1, 2, 3]
    assert any("test/loss" in l and math.isfinite(l["test/loss"]) for l in logs)
