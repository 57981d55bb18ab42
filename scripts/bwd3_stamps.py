#!/usr/bin/env python
"""Phase timing of the fused attention backward (debug build with DNA_BWD3_STAMP=1): runs the
bench shape once and prints per-slice cycle counts of block 0's waves: phase 1, barrier 1,
phase 2 (+ dQ partial write), barrier 2, dQ reduce/store."""
import ctypes
import math
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dna_amd import _native as N  # noqa: E402
from dna_amd.config import alibi_slopes  # noqa: E402

b, S, H, D = 256, 512, 12, 64
T = b * S
qkv = torch.randn(T, 3 * H * D, device="cuda").to(torch.bfloat16)
kv = torch.ones(T, dtype=torch.uint8, device="cuda")
slopes = torch.tensor(alibi_slopes(H), device="cuda")
out = torch.empty(T, H * D, device="cuda", dtype=torch.bfloat16)
lse = torch.empty(b, H, S, device="cuda")
dout = torch.randn(T, H * D, device="cuda").to(torch.bfloat16)
dqkv = torch.empty_like(qkv)
delta = torch.empty(b * H * S, device="cuda")
part = torch.empty(N.lib().dna_attn_dbias_part_rows(b, S), 3 * H * D, device="cuda")
st = torch.cuda.current_stream().cuda_stream
N.call("dna_attn_fwd", qkv.data_ptr(), kv.data_ptr(), slopes.data_ptr(), b, S, H, D, 1,
       1 / math.sqrt(D), out.data_ptr(), lse.data_ptr(), st)
for _ in range(3):
    N.call("dna_attn_bwd_ex", qkv.data_ptr(), out.data_ptr(), dout.data_ptr(), lse.data_ptr(),
           kv.data_ptr(), slopes.data_ptr(), b, S, H, D, 1, 1 / math.sqrt(D), dqkv.data_ptr(),
           delta.data_ptr(), part.data_ptr(), st)
torch.cuda.synchronize()
buf = np.zeros(4 * 16 * 6, dtype=np.uint64)
f = N.lib().dna_attn_debug_stamps
f.argtypes = [ctypes.c_void_p]
assert f(buf.ctypes.data) == 0
ts = buf.reshape(4, 16, 6).astype(np.int64)
print("per slice, cycles (s_memtime ticks): phase1 | barrier1 | phase2 | barrier2 | dQ store | total")
for w in range(4):
    d = np.diff(ts[w], axis=1)
    tot = ts[w, :, 5] - ts[w, :, 0]
    print(f"wave {w}: " + " | ".join(f"{int(np.median(d[:, k])):6d}" for k in range(5)) +
          f" | {int(np.median(tot)):6d}   (slice-to-slice {int(np.median(np.diff(ts[w, :, 0])))})")
