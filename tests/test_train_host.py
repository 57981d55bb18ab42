"""Host-side pieces of train.py / the data modules / the reducer (CPU):

* evaluation limits: limit_{val,test}_batches = 0 / 0.0 disable the loop, and a loader no rank ran
  a batch of is not logged (no fake 0.0 loss that would become the best checkpoint score);
* ParamsLog (src/callbacks/params.py:26-37);
* ModelCheckpoint state under Lightning 1.8's state_key with a tensor score, and round-4 files;
* the fault-tolerant sampler (fault_tolerant_sampler.py:64-122) and the data modules' argument
  checks (genomics.py:1117-1126);
* DNA_STRICT_NATIVE and GradBucketReducer(force=True) without a process group."""
import os

import pytest
import torch

import train


class _Model(torch.nn.Module):
    def __init__(self):
        super().__init__()
        self.a = torch.nn.Linear(4, 3)
        self.b = torch.nn.Parameter(torch.zeros(5), requires_grad=False)

    def mlm_loss(self, *a, **k):
        raise AssertionError("no batch should run")


class _Trainer:
    model = _Model()


def test_eval_batches_limits():
    assert train.eval_batches(10, 1.0) == 10
    assert train.eval_batches(10, 0.25) == 2
    assert train.eval_batches(10, 0.01) == 1      # a positive fraction runs at least one batch
    assert train.eval_batches(10, 0.0) == 0       # 0.0 disables (Lightning)
    assert train.eval_batches(10, 0) == 0
    assert train.eval_batches(10, 3) == 3 and train.eval_batches(2, 3) == 2
    assert train.eval_batches(0, 1.0) == 0
    assert train.eval_batches(7, None) == 7


def test_evaluate_skips_empty_loaders_and_zero_limit():
    tr = _Trainer()
    assert train.evaluate(tr, [("val", []), ("test", [])], "cpu", 3) == {}
    batch = ((torch.zeros(1, 4, dtype=torch.long),) * 3, torch.zeros(1, 4, dtype=torch.long))
    assert train.evaluate(tr, [("val", [batch])], "cpu", 3, limit=0) == {}
    assert train.evaluate(tr, [("val", [batch])], "cpu", 3, limit=0.0) == {}


def test_best_checkpoint_ignores_missing_monitor():
    best = train.BestCheckpoint("ck", "test/loss")
    assert best.improves(5.0)
    best.score = 1.0
    assert not best.improves(2.0) and best.improves(0.5)


def test_params_log():
    m = _Model()
    logs = train.params_log(m, {"total": True, "trainable": True, "fixed": True})
    assert logs == {"params/total": 4 * 3 + 3 + 5, "params/trainable": 15, "params/fixed": 5}
    assert train.params_log(m, {"total": False, "trainable": True, "fixed": False}) == \
        {"params/trainable": 15}


def test_model_checkpoint_state_key_and_resume(tmp_path):
    # Lightning 1.8 __init_triggers: every_n_epochs = 1 only when no trigger is given at all
    best = train.BestCheckpoint(str(tmp_path), "test/loss", mode="min")
    assert best.state_key == ("ModelCheckpoint{'monitor': 'test/loss', 'mode': 'min', "
                              "'every_n_train_steps': 0, 'every_n_epochs': 1, "
                              "'train_time_interval': None}")
    assert "'every_n_train_steps': 1000, 'every_n_epochs': 0," in train.BestCheckpoint(
        str(tmp_path), "test/loss", every_n_train_steps=1000).state_key
    assert "'every_n_train_steps': 0, 'every_n_epochs': 2," in train.BestCheckpoint(
        str(tmp_path), "test/loss", every_n_epochs=2).state_key
    assert "'every_n_train_steps': 0, 'every_n_epochs': 0," in train.BestCheckpoint(
        str(tmp_path), "test/loss", every_n_train_steps=0).state_key
    best.score = 1.25
    st = best.state_dict()
    assert isinstance(st["best_model_score"], torch.Tensor) and float(st["best_model_score"]) == 1.25
    path = tmp_path / "x.ckpt"
    torch.save({"callbacks": {best.state_key: st}}, path)
    b2 = train.BestCheckpoint(str(tmp_path), "test/loss")
    b2.load_from_checkpoint(torch.load(path, weights_only=True))
    assert b2.score == 1.25
    # a round-4 checkpoint (plain key, float score) still resumes
    b3 = train.BestCheckpoint(str(tmp_path), "test/loss")
    b3.load_from_checkpoint({"callbacks": {"ModelCheckpoint": {"monitor": "test/loss",
                                                               "best_model_score": 0.5}}})
    assert b3.score == 0.5
    b4 = train.BestCheckpoint(str(tmp_path), "val/loss")  # another monitor: not restored
    b4.load_from_checkpoint(torch.load(path, weights_only=True))
    assert b4.score is None


def test_checkpoint_loops_are_whole_lightning_progress_states():
    """The fit-loop counters are complete Lightning 1.8 Progress / BatchProgress states: every
    tracker of `total` and `current` (Progress.load_state_dict indexes both) and is_last_batch
    (BatchProgress) -- ADVICE r5; the reference's data module reads current.completed."""
    ep = train._progress(3)
    bp = dict(train._progress(11), is_last_batch=False)
    for st in (ep, bp):
        for part in ("total", "current"):
            assert set(st[part]) == {"ready", "started", "processed", "completed"}
    from dna_amd.hg38 import BertHG38
    d = BertHG38(fault_tolerant=True, ddp=True, shuffle=True)
    d.load_state_dict({"loops": {"fit_loop": {"epoch_progress": ep,
                                              "epoch_loop.batch_progress": bp}}})
    assert (d.fast_forward_epochs, d.fast_forward_batches) == (3, 11)


def _shard(n, world, rank, epoch, seed=0):
    s = torch.utils.data.distributed.DistributedSampler(range(n), num_replicas=world, rank=rank,
                                                        shuffle=True, seed=seed)
    s.set_epoch(epoch)
    return list(s)


@pytest.mark.parametrize("world,rank", [(1, 0), (3, 1)])
def test_fault_tolerant_sampler_resumes_mid_epoch(world, rank):
    from dna_amd.hg38 import FaultTolerantDistributedSampler
    n = 50
    s = FaultTolerantDistributedSampler(range(n), num_replicas=world, rank=rank, shuffle=True,
                                        seed=7)
    s.set_epoch(2)
    full = _shard(n, world, rank, 2, seed=7)
    assert list(s) == full and s.counter == 0       # a whole pass resets the counter
    it = iter(s)
    head = [next(it) for _ in range(6)]
    st = s.state_dict()
    assert st == {"epoch": 2, "counter": 6}
    s2 = FaultTolerantDistributedSampler(range(n), num_replicas=world, rank=rank, shuffle=True,
                                         seed=7)
    s2.load_state_dict(st)
    assert head + list(s2) == full                  # the rest of the epoch, once
    assert list(s2) == full                         # then whole epochs again


def test_fault_tolerant_argument_checks(tmp_path):
    from dna_amd.hg38 import BertHG38
    with pytest.raises(ValueError, match="shuffle"):
        BertHG38(fault_tolerant=True, shuffle=False)
    with pytest.raises(ValueError, match="ddp"):
        BertHG38(ddp=True, fault_tolerant=False, shuffle=True)
    with pytest.raises(ValueError, match="fast_forward"):
        BertHG38(fault_tolerant=True, shuffle=True, fast_forward_epochs=1)
    d = BertHG38(fault_tolerant=True, ddp=True, shuffle=True)
    d.load_state_dict({"loops": {"fit_loop": {"epoch_progress": {"current": {"completed": 3}},
                                              "epoch_loop.batch_progress": {"current": {"completed": 11}}}}})
    assert (d.fast_forward_epochs, d.fast_forward_batches) == (3, 11)


def test_strict_native_raises(monkeypatch):
    from dna_amd import functional as DF
    monkeypatch.setenv("DNA_STRICT_NATIVE", "1")
    with pytest.raises(DF.LibraryFallbackError):
        DF.library_fallback("linear forward", (3, 4), (5, 4))
    monkeypatch.setenv("DNA_STRICT_NATIVE", "0")
    DF.library_fallback("linear forward", (3, 4), (5, 4))
    assert ("linear forward", (3, 4), (5, 4)) in DF._FALLBACK_SEEN


def test_forced_reducer_needs_a_process_group(monkeypatch):
    from dna_amd.ddp import GradBucketReducer
    from dna_amd.flat import FlatParams
    m = torch.nn.Linear(4, 4)
    flat = FlatParams(m, "cpu", shadow_dtype=None)
    assert not GradBucketReducer(flat).enabled
    with pytest.raises(RuntimeError, match="process group"):
        GradBucketReducer(flat, force=True)
    monkeypatch.setenv("DNA_DDP_FORCE", "1")
    with pytest.raises(RuntimeError, match="process group"):
        GradBucketReducer(flat)
