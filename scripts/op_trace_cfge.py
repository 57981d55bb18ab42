#!/usr/bin/env python
"""Which torch ops launch the small glue kernels of a config E step (torch.profiler, CUDA
activities): the aten ops with their device-side kernel counts, to find copies / fills / adds
around the HIP kernels. python scripts/op_trace_cfge.py [L]"""
import os
import sys

import torch
from torch.profiler import ProfilerActivity, profile

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dna_amd.caduceus import CaduceusForMaskedLM  # noqa: E402
from dna_amd.trainer import ModuleTrainer  # noqa: E402


def main():
    L = int(sys.argv[1]) if len(sys.argv) > 1 else 131072
    torch.manual_seed(0)
    m = CaduceusForMaskedLM(d_model=256, n_layer=8, vocab_size=12, ssm_cfg={"d_state": 16})
    tr = ModuleTrainer(m, "cuda", lambda mod, b: mod(b[0], labels=b[1])[0], lr=8e-3,
                       weight_decay=0.1, max_grad_norm=1.0)
    g = torch.Generator(device="cuda").manual_seed(1)
    ids = torch.randint(7, 11, (1, L), device="cuda", generator=g)
    masked = torch.rand(1, L, device="cuda", generator=g) < 0.15
    batch = (torch.where(masked, torch.full_like(ids, 3), ids),
             torch.where(masked, ids, torch.full_like(ids, -100)))
    for _ in range(2):
        tr.step(batch)
    torch.cuda.synchronize()
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA]) as prof:
        tr.step(batch)
        torch.cuda.synchronize()
    print(prof.key_averages(group_by_input_shape=True).table(sort_by="cuda_time_total", row_limit=60,
                                                             max_name_column_width=60))


if __name__ == "__main__":
    main()
