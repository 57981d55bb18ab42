#!/usr/bin/env python
"""Micro-benchmark of the weight-gradient GEMM variants at the DNABERT-2 b=256 shapes
(T = 131072 tokens): dW[m, n] (fp32) += dy[T, m]^T x[T, n] with bf16 operands."""
import sys, os
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dna_amd import functional as DF  # noqa: E402
from dna_amd import _native as N  # noqa: E402


def t(fn, it=10):
    fn(); torch.cuda.synchronize()
    a, b = torch.cuda.Event(True), torch.cuda.Event(True)
    a.record()
    for _ in range(it):
        fn()
    b.record(); b.synchronize()
    return a.elapsed_time(b) / it


T = int(sys.argv[1]) if len(sys.argv) > 1 else 131072
for m, n in [(2304, 768), (768, 768), (6144, 768), (768, 3072), (3072, 768), (768, 6144)]:
    dy = torch.randn(T, m, device="cuda", dtype=torch.bfloat16)
    x = torch.randn(T, n, device="cuda", dtype=torch.bfloat16)
    g = torch.zeros(m, n, device="cuda")
    fl = 2.0 * T * m * n
    res = {}
    res["cur"] = t(lambda: DF.wgrad_accumulate(dy, x, g))
    res["mm32"] = t(lambda: torch.mm(dy.t(), x, out_dtype=torch.float32))
    res["mm16"] = t(lambda: torch.mm(dy.t(), x))
    for s in (1, 2, 4, 8, 16):
        def f(s=s):
            parts = torch.bmm(dy.view(s, T // s, m).transpose(1, 2), x.view(s, T // s, n), out_dtype=torch.float32)
            N.call("dna_sum_slices_accum", parts.data_ptr(), s, m * n, g.data_ptr(), N.stream_ptr())
        res[f"s{s}"] = t(f)
    print(f"m={m} n={n} split={DF.wgrad_splits(T, m, n)} " +
          " ".join(f"{k}={v*1e3:.0f}us({fl/v/1e9:.0f}TF)" for k, v in res.items()), flush=True)
