#!/usr/bin/env python
"""Time hipBLASLt (torch.mm) on every GEMM shape of the DNABERT-2 training step (GPU)."""
import sys

import torch

T = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
SHAPES = {"Wqkv": (768, 2304), "Wo": (768, 768), "Wg": (768, 6144), "Wwo": (3072, 768)}


def bench(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(True), torch.cuda.Event(True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters


def main():
    dev = "cuda"
    for name, (K, N) in SHAPES.items():
        x = torch.randn(T, K, device=dev).to(torch.bfloat16)
        w = (torch.randn(N, K, device=dev) * 0.02).to(torch.bfloat16)
        dy = torch.randn(T, N, device=dev).to(torch.bfloat16)
        fl = 2.0 * T * K * N
        res = {
            "fwd x@W^T": bench(lambda: torch.mm(x, w.t())),
            "dgrad dy@W": bench(lambda: torch.mm(dy, w)),
            "wgrad dy^T@x bf16": bench(lambda: torch.mm(dy.t(), x)),
            "wgrad dy^T@x fp32out": bench(lambda: torch.mm(dy.t(), x, out_dtype=torch.float32)),
            "wgrad x^T@dy bf16": bench(lambda: torch.mm(x.t(), dy)),
        }
        for k, ms in res.items():
            print(f"{name:5s} T={T} K={K} N={N} {k:22s} {ms * 1e3:8.1f} us {fl / ms / 1e9:7.1f} TF/s",
                  flush=True)


if __name__ == "__main__" and (len(sys.argv) < 3 or sys.argv[2] != "splitk"):
    main()


def probe_splitk():
    dev = "cuda"
    for name, (K, N) in SHAPES.items():
        x = torch.randn(T, K, device=dev).to(torch.bfloat16)
        dy = torch.randn(T, N, device=dev).to(torch.bfloat16)
        fl = 2.0 * T * K * N
        for s in (4, 8, 16, 32):
            a = dy.view(s, T // s, N).transpose(1, 2)
            b = x.view(s, T // s, K)
            ms = bench(lambda: torch.bmm(a, b).sum(0, dtype=torch.float32))
            print(f"{name:5s} splitK={s:2d} bmm bf16 + sum      {ms * 1e3:8.1f} us {fl / ms / 1e9:7.1f} TF/s", flush=True)
            try:
                ms = bench(lambda: torch.bmm(a, b, out_dtype=torch.float32).sum(0))
                print(f"{name:5s} splitK={s:2d} bmm fp32out + sum   {ms * 1e3:8.1f} us {fl / ms / 1e9:7.1f} TF/s", flush=True)
            except Exception as e:  # noqa: BLE001
                print("bmm out_dtype unsupported:", str(e)[:80])


if __name__ == "__main__" and len(sys.argv) > 2 and sys.argv[2] == "splitk":
    probe_splitk()
