"""The real training step (MLMTrainer: HIP forward/backward, fused loss, gradient buckets, fused
clip + AdamW) under the reference's Lightning semantics (GPU only):

* accumulate_grad_batches=k (dnabert2_hg38_pretrain.yaml:49; Lightning divides each micro-batch
  loss by k, DDP no_sync until the last) == one k-times-larger batch when every micro-batch has
  the same masked-token count;
* DDP (strategy: ddp, train.py:630-639) with two ranks -- gloo, both on cuda:0 -- == one process
  on the concatenated batch (mean of per-rank means = global mean at equal mask counts), with
  every gradient bucket launched from inside the backward (direct-gradient `_dna_notify` path of
  the fused weight gradients in bf16, AccumulateGrad hooks in fp32, the tied embedding's two
  contributions) and the 1/world average folded into AdamW (grad_scale);
* a torch.optim.AdamW state (a reference Lightning checkpoint's optimizer_states) continues
  exactly in FusedAdamW.
"""
import copy
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

CFG_A = dict(vocab_size=4096, hidden_size=128, num_hidden_layers=2, num_attention_heads=2,
             intermediate_size=512, hidden_dropout_prob=0.0, attention_probs_dropout_prob=0.0,
             layer_norm_eps=1e-12, max_position_embeddings=512, type_vocab_size=2,
             pad_token_id=0, alibi_starting_size=512, hidden_act="gelu",
             initializer_range=0.02, hyena_framework=True)
S = 128
K_MASK = 19  # masked positions per row: equal mask counts in every micro-batch / rank


def _batch(seed, b):
    """Host batch in the dataset's form ((masked, mask, labels), target): ids >= 5 (no pad /
    [UNK] / special ids), exactly K_MASK masked positions per row replaced by [MASK] = 4."""
    g = torch.Generator().manual_seed(seed)
    target = torch.randint(5, 4096, (b, S), generator=g)
    mask = torch.zeros(b, S, dtype=torch.bool)
    for r in range(b):
        mask[r, torch.randperm(S, generator=g)[:K_MASK]] = True
    masked = torch.where(mask, torch.full_like(target, 4), target)
    labels = torch.where(mask, target, torch.full_like(target, -100))
    return masked, mask, labels, target


def _cat(*bs):
    return tuple(torch.cat(t) for t in zip(*bs))


def _trainer(precision, seed=0, **kw):
    from dna_amd.bert_layers import BertForMaskedLM
    from dna_amd.trainer import MLMTrainer
    torch.manual_seed(seed)
    m = BertForMaskedLM(CFG_A, precision=precision)
    return MLMTrainer(m, torch.device("cuda", 0), lr=1e-3, weight_decay=1e-5,
                      max_grad_norm=1.0, **kw)


def _dev(hb):
    from dna_amd.trainer import DeviceBatch
    masked, mask, labels, target = hb
    return DeviceBatch.from_host(masked, mask, labels, target, torch.device("cuda", 0))


@pytest.mark.parametrize("precision", ["fp32", "bf16"])
def test_accumulation_equals_one_large_batch(precision):
    k, b = 3, 4
    micro = [_batch(100 + i, b) for i in range(k)]
    runs = []
    for accumulate in (True, False):
        tr = _trainer(precision)
        for step in range(2):
            mbs = [_batch(1000 * step + 100 + i, b) for i in range(k)] if step else micro
            if accumulate:
                loss = tr.step([_dev(x) for x in mbs])
            else:
                loss = tr.step(_dev(_cat(*mbs)))
            grad = tr.flat.grad.clone()
            if step == 0:
                first = (float(loss), grad)
        torch.cuda.synchronize()
        runs.append((first, tr.flat.flat.clone()))
    (l_acc, g_acc), p_acc = runs[0]
    (l_big, g_big), p_big = runs[1]
    scale = g_big.abs().max().item()
    if precision == "fp32":
        assert abs(l_acc - l_big) < 1e-5 * abs(l_big)
        assert (g_acc - g_big).abs().max().item() < 1e-5 * scale
        assert (p_acc - p_big).abs().max().item() < 2e-5
    else:  # bf16 activations: the k micro-batches and the big batch round the same values
        assert abs(l_acc - l_big) < 2e-3 * abs(l_big)
        assert float((g_acc - g_big).norm() / g_big.norm()) < 2e-2
        assert (p_acc - p_big).abs().max().item() < 2 * 2 * 1e-3  # <= 2 AdamW steps of lr


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _ddp_worker(rank, world, port, precision, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        tr = _trainer(precision, seed=rank, bucket_mb=0.25)  # different init: broadcast must fix it
        n_buckets = len(tr.reducer.buckets)
        grads, fired, scales = [], [], []
        for step in range(3):
            tr.step(_dev(_batch(10 * step + rank, 4)))
            torch.cuda.synchronize()
            grads.append((tr.flat.grad * tr.reducer.grad_scale).cpu().numpy())
            fired.append(tr.reducer.fired_in_backward)
            scales.append(tr.reducer.grad_scale)
        # numpy, not tensors: torch's queue would share tensor storage through a file
        # descriptor that dies with this process
        q.put((rank, dict(grads=grads, fired=fired, n_buckets=n_buckets, scales=scales,
                          flat=tr.flat.flat.cpu().numpy())))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("precision", ["fp32", "bf16"])
def test_ddp_two_ranks_equals_single_process(precision):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_ddp_worker, args=(r, 2, port, precision, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=300) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    tr = _trainer(precision, seed=0)
    ref_grads = []
    for step in range(3):
        tr.step(_dev(_cat(_batch(10 * step, 4), _batch(10 * step + 1, 4))))
        torch.cuda.synchronize()
        ref_grads.append(tr.flat.grad.cpu())
    ref_flat = tr.flat.flat.cpu()
    r0, r1 = res[0], res[1]
    for r in (r0, r1):
        r["flat"] = torch.from_numpy(r["flat"])
        r["grads"] = [torch.from_numpy(g) for g in r["grads"]]
    assert r0["scales"] == [0.5] * 3 and r0["n_buckets"] > 4
    # step 0 learns the per-parameter contribution counts; afterwards every bucket is launched
    # from the backward's hooks / the fused wgrad notify, none left for finish()
    assert r0["fired"][1:] == [r0["n_buckets"]] * 2 and r1["fired"][1:] == [r1["n_buckets"]] * 2
    assert torch.equal(r0["flat"], r1["flat"])  # replicas stay identical
    for step in range(3):
        assert torch.equal(r0["grads"][step], r1["grads"][step])
        g, ref = r0["grads"][step], ref_grads[step]
        if precision == "fp32":
            assert (g - ref).abs().max().item() < 1e-5 * ref.abs().max().item(), step
        else:
            assert float((g - ref).norm() / ref.norm()) < 2e-2, step
    tol = 2e-5 if precision == "fp32" else 3 * 2 * 1e-3
    assert (r0["flat"] - ref_flat).abs().max().item() < tol


def test_fused_adamw_continues_torch_adamw_state():
    """Optimizer state of a reference checkpoint (torch AdamW after 2 steps) loaded into the flat
    buffers: one more step with the same gradient gives torch AdamW's parameters (fp32)."""
    from dna_amd.bert_layers import BertForMaskedLM
    from dna_amd.flat import FlatParams
    from dna_amd.optim import FusedAdamW
    torch.manual_seed(0)
    ref = BertForMaskedLM(CFG_A, precision="fp32")
    init = {k: v.clone() for k, v in ref.state_dict().items()}
    opt = torch.optim.AdamW(ref.parameters(), lr=5e-4, betas=(0.9, 0.98), eps=1e-8,
                            weight_decay=1e-5)
    g = torch.Generator().manual_seed(1)
    fake = [[torch.randn(p.shape, generator=g) * 1e-2 for p in ref.parameters()] for _ in range(3)]
    for s in range(2):
        for p, gr in zip(ref.parameters(), fake[s]):
            p.grad = gr.clone()
        opt.step()
    mid = {k: v.clone() for k, v in ref.state_dict().items()}
    sd = copy.deepcopy(opt.state_dict())  # state_dict() aliases the live moment tensors
    for p, gr in zip(ref.parameters(), fake[2]):
        p.grad = gr.clone()
    opt.step()
    m = BertForMaskedLM(CFG_A, precision="fp32")
    m.load_state_dict(mid)
    m = m.cuda()
    flat = FlatParams(m, "cuda")
    fo = FusedAdamW(flat, lr=1.0, max_grad_norm=0.0)
    fo.load_state_dict(sd)
    for p, gr in zip(m.parameters(), fake[2]):
        p.grad.copy_(gr)
    fo.step()
    torch.cuda.synchronize()
    for (n, p), pr in zip(m.named_parameters(), ref.parameters()):
        assert torch.allclose(p.detach().cpu(), pr.detach(), atol=1e-6, rtol=1e-5), n
    assert any(not torch.equal(init[k], mid[k]) for k in init)
