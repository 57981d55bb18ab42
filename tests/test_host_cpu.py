"""CPU tests of the host-side training machinery: flat parameter store, LR schedule, the model
mirror's interface, and the data-parallel gradient reducer over gloo with 2 ranks."""
import math
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import optim_ref


def test_flat_params_views_and_order():
    from dna_amd.flat import ALIGN, FlatParams
    m = torch.nn.Sequential(torch.nn.Linear(7, 5), torch.nn.Linear(5, 3))
    ref = [p.detach().clone() for p in m.parameters()]
    flat = FlatParams(m, "cpu")
    for p, r in zip(m.parameters(), ref):
        assert torch.equal(p.detach(), r)
        assert p.data.data_ptr() >= flat.flat.data_ptr()
        assert p.grad is not None and p.grad.data_ptr() >= flat.grad.data_ptr()
    offs = [o for o, _, _ in flat.slices]
    assert all(o % ALIGN == 0 for o in offs) and offs == sorted(offs)
    # reverse registration order: the last parameter sits at offset 0
    assert flat.slice_of(list(m.parameters())[-1])[0] == 0
    x = torch.randn(4, 7)
    m(x).sum().backward()
    assert flat.grad.abs().sum() > 0
    assert torch.equal(flat.lp(m[0].weight).float(), m[0].weight.detach().to(torch.bfloat16).float())


def test_model_mirror_interface():
    from dna_amd.bert_layers import BertForMaskedLM, MLMIndex
    cfg = dict(vocab_size=4096, hidden_size=128, num_hidden_layers=2, num_attention_heads=2,
               intermediate_size=512, hyena_framework=True)
    m = BertForMaskedLM(cfg)
    assert m.cls.predictions.decoder.weight is m.bert.embeddings.word_embeddings.weight
    # like the reference (checked by importing it): HF post_init zeroes the padding_idx row in the
    # Embedding init, then the tied decoder's Linear init redraws the whole table, row 0 included
    assert m.bert.embeddings.word_embeddings.weight[0].abs().max() > 0
    n = sum(p.numel() for p in m.parameters())
    assert n == 4096 * 128 + 2 * 128 + 2 * 128 + 2 * (3 * 128 * 128 + 3 * 128 + 128 * 128 + 128 +
                                                    2 * 128 + 1024 * 128 + 512 * 128 + 128 +
                                                    2 * 128) + 128 * 128 + 128 + 2 * 128 + 4096
    ids = torch.tensor([[5, 6, 7, 3], [8, 9, 10, 11]])
    labels = torch.tensor([[-100, 6, -100, -100], [8, -100, -100, 11]])
    idx = MLMIndex.build(ids, labels)
    # subset rows: masked | first column, never pads; head rows: masked rows within the subset
    assert idx.subset_idx.tolist() == [0, 1, 4, 7]
    assert idx.head_idx.tolist() == [1, 2, 3]
    assert idx.target.tolist() == [6, 8, 11] and idx.flat_masked.tolist() == [1, 4, 7]
    with pytest.raises(RuntimeError, match="GPU"):
        m.mlm_logits(ids, idx)  # product path has no CPU fallback


def test_lr_scheduler_matches_restatement():
    from dna_amd.optim import LinearLRSchedulerWarmup

    class O:
        param_groups = [{"lr": 5e-4, "initial_lr": 5e-4}]

    o = O()
    s = LinearLRSchedulerWarmup(o, t_initial=2000, warmup_t=120, warmup_lr_init=0.0, lr_min=0.0)
    for t in range(1, 2500, 37):
        s.step(epoch=t)
        assert math.isclose(o.param_groups[0]["lr"],
                            optim_ref.linear_warmup_lr(t, 5e-4, 120, 2000), rel_tol=1e-12)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _ddp_worker(rank, world, port, q, wire="fp32"):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from dna_amd.ddp import GradBucketReducer
        from dna_amd.flat import FlatParams
        torch.manual_seed(0)
        emb = torch.nn.Embedding(50, 16)
        m = torch.nn.ModuleDict({"emb": emb, "l1": torch.nn.Linear(16, 32),
                                 "l2": torch.nn.Linear(32, 50)})
        m["l2"].weight = emb.weight.__class__(torch.randn(50, 32))  # distinct weight
        head = torch.nn.Linear(16, 50, bias=False)
        head.weight = emb.weight  # tied: two gradient contributions per step
        m["head"] = head
        flat = FlatParams(m, "cpu", shadow_dtype=None)
        red = GradBucketReducer(flat, bucket_mb=0.002, wire_dtype=wire)  # tiny buckets
        assert len(red.buckets) > 3
        results = []
        for step in range(3):
            g = torch.Generator().manual_seed(100 * step + rank)
            ids = torch.randint(0, 50, (8,), generator=g)
            flat.zero_grad()
            red.prepare()
            h = m["emb"](ids)
            out = m["l2"](torch.relu(m["l1"](h))) + m["head"](h)
            loss = torch.nn.functional.cross_entropy(out, ids)
            loss.backward()
            red.finish()
            results.append(flat.grad.clone() * red.grad_scale)
        q.put((rank, [r.tolist() for r in results]))
    finally:
        dist.destroy_process_group()


def _single_grads():
    """Average of per-rank gradients computed without any collective."""
    torch.manual_seed(0)
    emb = torch.nn.Embedding(50, 16)
    l1, l2 = torch.nn.Linear(16, 32), torch.nn.Linear(32, 50)
    l2.weight = emb.weight.__class__(torch.randn(50, 32))
    from dna_amd.flat import FlatParams
    m = torch.nn.ModuleDict({"emb": emb, "l1": l1, "l2": l2})
    head = torch.nn.Linear(16, 50, bias=False)
    head.weight = emb.weight
    m["head"] = head
    flat = FlatParams(m, "cpu", shadow_dtype=None)
    out = []
    for step in range(3):
        acc = torch.zeros_like(flat.grad)
        for rank in range(2):
            g = torch.Generator().manual_seed(100 * step + rank)
            ids = torch.randint(0, 50, (8,), generator=g)
            flat.zero_grad()
            h = m["emb"](ids)
            o = m["l2"](torch.relu(m["l1"](h))) + m["head"](h)
            torch.nn.functional.cross_entropy(o, ids).backward()
            acc += flat.grad
        out.append(acc / 2)
    return out


@pytest.mark.parametrize("wire", ["fp32", "bf16"])
def test_grad_bucket_reducer_gloo_two_ranks(wire):
    """fp32 wire: exact average; bf16 wire (SURVEY §8(e) 234 MB format): within bf16 rounding of
    the summands (one cast per rank, the sum itself rounded once more)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_ddp_worker, args=(r, 2, port, q, wire)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    ref = _single_grads()
    for step in range(3):
        a, b = torch.tensor(res[0][step]), torch.tensor(res[1][step])
        assert torch.equal(a, b)  # every rank holds the same averaged gradient
        if wire == "fp32":
            assert torch.allclose(a, ref[step], atol=1e-6), (a - ref[step]).abs().max()
        else:
            rel = float((a - ref[step]).norm() / ref[step].norm())
            assert rel < 1e-2, rel
            assert not torch.equal(a, ref[step])  # the bf16 wire really was used


def _metrics_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from dna_amd.ddp import reduce_metrics
        loss = torch.tensor(1.0 + rank)      # per-rank masked-token means
        q.put((rank, reduce_metrics(loss, 100 * (rank + 1))))
    finally:
        dist.destroy_process_group()


def test_reduce_metrics_two_ranks_gloo():
    """One packed all-reduce: rank-mean loss (DDP loss semantics) and the global token count,
    identical on every rank."""
    from dna_amd.ddp import reduce_metrics
    assert reduce_metrics(torch.tensor(2.5), 7) == (2.5, 7)  # no process group: local values
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_metrics_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    out = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    assert out[0] == out[1] == (1.5, 300)
