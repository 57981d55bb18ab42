"""CPU tests of the training-loop bookkeeping around the hot path:

* task torchmetrics Perplexity / NumTokens (reference src/tasks/torchmetrics.py:24-115) -- the
  reference's own docstring example (5.2545) and its token-weighted accumulation, summed over
  ranks like dist_reduce_fx="sum" (gloo, 2 ranks);
* checkpoint interop: FusedAdamW state in torch AdamW's layout (what a Lightning checkpoint of
  the reference holds, train.py:462-473: one group over list(self.parameters())) loads into the
  flat moment buffers and back; the timm scheduler state key `_last_epoch`.
torchmetrics / Lightning are not installed here, so the expected values are the formulas the
reference file states, and torch.optim.AdamW itself produces the foreign optimizer state.
"""
import math
import os

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp
import torch.nn.functional as F

from tests.test_host_cpu import _free_port


def test_perplexity_reference_docstring_example():
    """torchmetrics.py:33-39: preds rand(2,8,5) / target randint(5,(2,8)) seeded 22, the last
    two targets of row 0 ignored (-100) -> tensor(5.2545)."""
    from dna_amd.tasks import Perplexity
    preds = torch.rand(2, 8, 5, generator=torch.manual_seed(22))
    target = torch.randint(5, (2, 8), generator=torch.manual_seed(22))
    target[0, 6:] = -100
    loss = F.cross_entropy(preds.view(-1, 5), target.view(-1), ignore_index=-100)
    m = Perplexity()
    m.update(preds, target, loss)
    assert round(float(m.compute()), 4) == 5.2545


def test_perplexity_is_token_weighted_and_num_tokens_never_resets():
    from dna_amd.tasks import NumTokens, Perplexity
    m, n = Perplexity(), NumTokens()
    batches = [(1.5, (4, 16)), (2.25, (8, 16)), (0.75, (2, 16))]
    for loss, shape in batches:
        t = torch.zeros(shape, dtype=torch.long)
        m.update(None, t, torch.tensor(loss))
        n.update(None, t)
    want = math.exp(sum(l * a * b for l, (a, b) in batches) / sum(a * b for _, (a, b) in batches))
    assert math.isclose(float(m.compute()), want, rel_tol=1e-12)
    assert m.total_log_probs.dtype == torch.float64
    m.reset()
    n.reset()  # NumTokens.reset keeps the count (torchmetrics.py:104-107)
    assert float(m.count) == 0 and int(n.compute()) == sum(a * b for _, (a, b) in batches)


def _ppl_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from dna_amd.ddp import reduce_metrics
        from dna_amd.tasks import Perplexity
        m = Perplexity()
        # rank r sees micro-batches of different sizes and losses
        for j in range(3):
            m.update_count(torch.tensor(1.0 + 0.5 * rank + 0.1 * j), (rank + 1) * (j + 2) * 128)
        lv, sums = reduce_metrics(torch.tensor(1.0 + rank), 0,
                                  extra=[m.total_log_probs, m.count, 1000 * (rank + 1)])
        q.put((rank, (lv, sums)))
    finally:
        dist.destroy_process_group()


def test_perplexity_sum_reduced_over_ranks_gloo():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_ppl_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    out = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert out[0] == out[1]
    lv, (tlp, cnt, ntok) = out[0]
    num = sum((1.0 + 0.5 * r + 0.1 * j) * (r + 1) * (j + 2) * 128 for r in range(2) for j in range(3))
    den = sum((r + 1) * (j + 2) * 128 for r in range(2) for j in range(3))
    assert lv == 1.5 and cnt == den and ntok == 3000
    # losses are float32 tensors (as the step returns them); sums in float64
    assert math.isclose(math.exp(tlp / cnt), math.exp(num / den), rel_tol=1e-6)


def _tiny_model():
    torch.manual_seed(0)
    emb = torch.nn.Embedding(11, 8)
    m = torch.nn.ModuleDict({"emb": emb, "l1": torch.nn.Linear(8, 16), "l2": torch.nn.Linear(16, 8)})
    return m


def _torch_adamw_state(m, steps=3):
    opt = torch.optim.AdamW(m.parameters(), lr=5e-4, betas=(0.9, 0.98), eps=1e-8,
                            weight_decay=1e-5)
    for s in range(steps):
        opt.zero_grad()
        x = m["emb"](torch.arange(11) % (s + 3))
        m["l2"](torch.relu(m["l1"](x))).pow(2).sum().backward()
        opt.step()
    return opt.state_dict()


def test_fused_adamw_loads_torch_adamw_layout_and_round_trips():
    """A reference (Lightning / torch AdamW) optimizer state maps into the flat moment buffers
    through the parameter slices; the state written back is the same torch layout and loads into
    torch.optim.AdamW unchanged."""
    from dna_amd.flat import FlatParams
    from dna_amd.optim import FusedAdamW
    ref = _tiny_model()
    sd = _torch_adamw_state(ref)
    m = _tiny_model()
    flat = FlatParams(m, "cpu", shadow_dtype=None)
    opt = FusedAdamW(flat, lr=1.0)
    opt.load_state_dict(sd)
    assert opt.step_count == 3
    g = opt.param_groups[0]
    assert g["lr"] == 5e-4 and g["betas"] == (0.9, 0.98) and g["weight_decay"] == 1e-5
    for i, p in enumerate(m.parameters()):
        o, n, shape = flat.slice_of(p)
        assert torch.equal(opt.exp_avg[o:o + n].view(shape), sd["state"][i]["exp_avg"])
        assert torch.equal(opt.exp_avg_sq[o:o + n].view(shape), sd["state"][i]["exp_avg_sq"])
    out = opt.state_dict()
    assert sorted(out) == ["param_groups", "state"] and out["param_groups"][0]["params"] == list(range(5))
    back = torch.optim.AdamW(_tiny_model().parameters(), lr=1.0)
    back.load_state_dict(out)  # torch accepts it
    for i in range(5):
        assert torch.equal(back.state_dict()["state"][i]["exp_avg"], sd["state"][i]["exp_avg"])
        assert float(back.state_dict()["state"][i]["step"]) == 3.0
    # flat form still accepted (round-1 checkpoints)
    opt2 = FusedAdamW(flat, lr=1.0)
    opt2.load_state_dict(opt.state_dict(torch_layout=False))
    assert torch.equal(opt2.exp_avg, opt.exp_avg) and opt2.step_count == 3
    bad = dict(sd, param_groups=[dict(sd["param_groups"][0], params=[0, 1])])
    with pytest.raises(ValueError, match="parameters"):
        opt2.load_state_dict(bad)


def test_scheduler_state_uses_timm_key():
    from dna_amd.optim import LinearLRSchedulerWarmup

    class O:
        param_groups = [{"lr": 5e-4, "initial_lr": 5e-4}]

    s = LinearLRSchedulerWarmup(O(), t_initial=2000, warmup_t=120)
    for _ in range(7):
        s.step()
    st = s.state_dict()
    assert st["_last_epoch"] == 7
    o2 = O()
    o2.param_groups = [{"lr": 5e-4, "initial_lr": 5e-4}]
    s2 = LinearLRSchedulerWarmup(o2, t_initial=2000, warmup_t=120)
    s2.load_state_dict({"_last_epoch": 7, "base_values": [5e-4]})  # reference timm layout
    assert o2.param_groups[0]["lr"] == s.optimizer.param_groups[0]["lr"]
    s2.load_state_dict({"last_epoch": 9})  # round-1 layout
    assert s2._last_epoch == 9
