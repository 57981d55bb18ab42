"""Diagnose side-stream wgrad determinism: flat grads for DNA_WGRAD_STREAM=0/1, twice each."""
import os, sys
ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
import torch
from test_gpu_model import _golden, _batch
from dna_amd.bert_layers import BertForMaskedLM, MLMIndex
from dna_amd.flat import FlatParams

DEV = "cuda:0"
z, cfg = _golden("cfgA")
ids, mask, labels = _batch(z)
idx = MLMIndex.build(ids, labels)
res = {}
for side in ("0", "0", "1", "1"):
    os.environ["DNA_WGRAD_STREAM"] = side
    torch.manual_seed(0)
    m = BertForMaskedLM(cfg, precision="bf16").to(DEV).eval()
    flat = FlatParams(m, DEV)
    flat.enable_direct_grad(True)
    for _ in range(2):
        flat.zero_grad()
        loss, _ = m.mlm_loss(ids, mask, idx)
        loss.backward()
    g = flat.grad.clone()
    torch.cuda.synchronize()
    g2 = flat.grad.clone()
    print("side", side, "post-sync equal", torch.equal(g, g2), flush=True)
    res.setdefault(side, []).append((g2, m))
names = [n for n, _ in res["0"][0][1].named_parameters()]
def cmp(a, b, tag):
    ga, ma = a; gb, mb = b
    print(tag, "equal", torch.equal(ga, gb), "maxdiff", (ga - gb).abs().max().item())
    for (n, pa), (_, pb) in zip(ma.named_parameters(), mb.named_parameters()):
        if pa.grad is None: continue
        d = (pa.grad - pb.grad).abs().max().item()
        if d: print("   ", n, d, pa.grad.abs().max().item())
cmp(res["0"][0], res["0"][1], "0 vs 0")
cmp(res["1"][0], res["1"][1], "1 vs 1")
cmp(res["0"][0], res["1"][0], "0 vs 1")
