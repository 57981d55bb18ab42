#!/usr/bin/env python
"""Diagnostic: config-D (L = 65,536, 2 layers, fp32) logits error vs the float64 oracle with the
implicit-filter MLP on the strided HIP GEMM (default) and on torch's nn.Linear, plus the filter
outputs' own error vs a float64 filter. Prints one JSON line."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
from dna_amd import hyena  # noqa: E402
from oracle import hyena_lm_ref as LM  # noqa: E402
from test_gpu_hyena_lm import _config_d_model  # noqa: E402


def rel(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return float((a - b).abs().max() / (b.abs().max() + 1e-30))


L = 65536
torch.manual_seed(11)
m = _config_d_model(2, L)
with torch.no_grad():
    for n, p in m.named_parameters():
        if not n.endswith("freq"):
            p.add_(torch.randn_like(p) * 0.02)
sd = {k: v.detach().double().clone() for k, v in m.state_dict().items()}
sd["lm_head.weight"] = sd["backbone.embeddings.word_embeddings.weight"]
ids = torch.randint(7, 11, (1, L), generator=torch.Generator().manual_seed(12))
m64 = _config_d_model(2, L).double()
m64.load_state_dict({k: v for k, v in sd.items() if k != "lm_head.weight"}, strict=False)
m = m.to("cuda").eval()
ref = LM.lm_logits(sd, ids, 256, 2, l_max=L, bidirectional=True)
res = {}
orig = hyena._split_k_linear
for name, fn in (("hip_strided", orig), ("torch_linear", lambda x, lin: lin(x))):
    hyena._split_k_linear = fn
    with torch.no_grad():
        (out, _) = m((ids.to("cuda"), torch.ones(1, L, dtype=torch.bool, device="cuda")))
        f = m.backbone.layers[0].mixer.filter_fn.filter(L)
    with torch.no_grad():
        hyena._split_k_linear = lambda x, lin: lin(x)
        f64 = m64.backbone.layers[0].mixer.filter_fn.filter(L)
    res[name] = {"logits_rel": rel(out.logits[0], ref), "filter_rel": rel(f, f64)}
hyena._split_k_linear = orig
print(json.dumps(res))
