"""Micro-benchmark of dna_embed_grad_segsum (the embedding table gradient: id-sorted segmented sum
of per-token rows) at a config-D shape: B x L tokens over a V-symbol vocabulary, d columns.
Prints one line: avg ms per call (HIP events on torch's current stream, which N.stream_ptr()
launches on) and a checksum of the result, so library builds (DNA_AMD_LIB) can be compared
for speed and for bit-identical output."""
import argparse
import os
import sys
import zlib

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dna_amd import _native as N


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=2)
    ap.add_argument("--L", type=int, default=65536)
    ap.add_argument("--V", type=int, default=16)
    ap.add_argument("--d", type=int, default=256)
    ap.add_argument("--ids", type=int, default=4, help="distinct ids in the text")
    ap.add_argument("--iters", type=int, default=50)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    g = torch.Generator(device="cpu").manual_seed(0)
    # default: a 4-letter DNA text over a 16-symbol vocabulary, 4 frequent ids with ~T/4 rows each
    ids = ((torch.randint(0, a.ids, (a.B * a.L,), generator=g) + 7) % a.V).to(dev)
    drows = torch.randn(a.B * a.L, a.d, generator=g).to(dev)
    T = ids.numel()
    sorted_ids, perm = torch.sort(ids, stable=True)
    dE = torch.zeros(a.V, a.d, device=dev)
    nsw = N.lib().dna_embed_grad_segsum_workspace(T, a.d)
    sw = torch.empty(max(nsw // 4, 4), device=dev)

    def call():
        dE.zero_()
        N.call("dna_embed_grad_segsum", drows.data_ptr(), sorted_ids.data_ptr(), perm.data_ptr(),
               T, a.d, a.V, -1, dE.data_ptr(), sw.data_ptr(), nsw, N.stream_ptr())

    for _ in range(3):
        call()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(a.iters):
        call()
    e1.record()
    torch.cuda.synchronize()
    ref = torch.zeros_like(dE).index_add_(0, ids, drows)
    err = (dE - ref).abs().max().item()
    print(f"{e0.elapsed_time(e1) / a.iters:.4f} ms/call  sum {dE.double().sum().item():.10e}  "
          f"bits {zlib.crc32(dE.cpu().numpy().tobytes()):08x}  max|err| vs index_add {err:.2e}",
          flush=True)


if __name__ == "__main__":
    main()
