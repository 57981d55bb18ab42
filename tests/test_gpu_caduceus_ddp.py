"""Config E's data-parallel leg (BASELINE configs[4]: Caduceus, DDP): the Caduceus MLM step
through dna_amd.trainer.ModuleTrainer -- flat parameters, gradient buckets all-reduced as the
backward produces them, fused clip + AdamW with the 1/world average -- on two gloo ranks (one
GPU) equals one process on the concatenated batch; replicas stay identical; bf16 wire format
within bf16 rounding. GPU."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

CFG = dict(d_model=64, n_layer=2, vocab_size=12, ssm_cfg={"d_state": 16})
L = 1024


def _batch(seed, b):
    """Exactly 150 masked positions per sequence: every rank's masked-token mean then weighs its
    tokens as the concatenated batch's mean does, so DDP's mean of rank means is that mean."""
    g = torch.Generator().manual_seed(seed)
    ids = torch.randint(7, 11, (b, L), generator=g)
    masked = torch.zeros(b, L, dtype=torch.bool)
    for i in range(b):
        masked[i, torch.randperm(L, generator=g)[:150]] = True
    inp = torch.where(masked, torch.full_like(ids, 3), ids)
    labels = torch.where(masked, ids, torch.full_like(ids, -100))
    return inp, labels


def _loss(model, batch):
    inp, labels = batch
    return model(inp, labels=labels)[0]


def _trainer(seed, autocast, wire="fp32", bucket_mb=0.05):
    from dna_amd.caduceus import CaduceusForMaskedLM
    from dna_amd.trainer import ModuleTrainer
    torch.manual_seed(seed)
    m = CaduceusForMaskedLM(**CFG)
    return ModuleTrainer(m, "cuda", _loss, lr=2e-3, weight_decay=0.1, max_grad_norm=1.0,
                         bucket_mb=bucket_mb, wire_dtype=wire, autocast=autocast)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, autocast, wire, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        tr = _trainer(seed=rank, autocast=autocast, wire=wire)  # broadcast fixes the init
        fired = []
        for step in range(2):
            inp, labels = _batch(10 * step + rank, 2)
            tr.step((inp.cuda(), labels.cuda()))
            torch.cuda.synchronize()
            fired.append(tr.reducer.fired_in_backward)
        q.put((rank, dict(flat=tr.flat.flat.cpu().numpy(), fired=fired,
                          n_buckets=len(tr.reducer.buckets), scale=tr.reducer.grad_scale)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("autocast,wire", [(None, "fp32"), (torch.bfloat16, "fp32"),
                                           (None, "bf16")])
def test_caduceus_two_ranks_equals_single_process(autocast, wire):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, autocast, wire, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=300) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    tr = _trainer(seed=0, autocast=autocast)
    p0 = tr.flat.flat.clone()
    for step in range(2):
        a, b = _batch(10 * step, 2), _batch(10 * step + 1, 2)
        tr.step((torch.cat([a[0], b[0]]).cuda(), torch.cat([a[1], b[1]]).cuda()))
    torch.cuda.synchronize()
    ref = tr.flat.flat.cpu()
    r0, r1 = (torch.from_numpy(res[r]["flat"]) for r in (0, 1))
    assert torch.equal(r0, r1)  # replicas identical
    assert res[0]["scale"] == 0.5 and res[0]["n_buckets"] > 3
    # after the first step (which learns the contribution counts) every bucket fires in backward
    assert res[0]["fired"][1] == res[0]["n_buckets"]
    lr = 2e-3
    d_ref, d_dp = ref - p0.cpu(), r0 - p0.cpu()
    assert d_ref.abs().max().item() > 0.5 * lr  # two AdamW steps moved the parameters
    if autocast is None and wire == "fp32":
        assert (r0 - ref).abs().max().item() < 2e-5
    else:
        # bf16 rounding (compute or wire) perturbs the smallest gradient entries; AdamW's first
        # steps are ~ lr * sign(g), so count the entries whose update moved by > lr / 4
        frac = ((r0 - ref).abs() > 0.25 * lr).float().mean().item()
        assert frac < 0.01, frac
        assert float((d_dp - d_ref).norm() / d_ref.norm()) < 0.1


def test_bf16_shadow_follows_load_state_dict():
    """The Mamba projections read the trainer's bf16 parameter copy; weights loaded after the
    trainer exists (load_state_dict) must reach it before the next step."""
    src = _trainer(seed=1, autocast=torch.bfloat16)
    tr = _trainer(seed=0, autocast=torch.bfloat16)
    tr.model.load_state_dict(src.model.state_dict())
    batch = tuple(t.cuda() for t in _batch(3, 2))
    la, lb = tr.step(batch), src.step(batch)
    torch.cuda.synchronize()
    assert float(la) == float(lb)  # the forward saw the loaded weights
    # the scan backward sums dA / dB / dC with atomics (order-dependent last bits), so the two
    # updates agree up to AdamW's lr * sign(g) on near-zero gradient entries
    frac = ((tr.flat.flat - src.flat.flat).abs() > 0.25 * 2e-3).float().mean().item()
    assert frac < 0.01, frac
    assert torch.equal(tr.flat.shadow, tr.flat.flat.bfloat16())
