"""CPU: the selective-scan restatement (oracle/selective_scan_ref.py) agrees with an independent
closed form on a case small enough to unroll by hand (parity unpinned vs mamba_ssm itself)."""
import torch

from oracle.selective_scan_ref import selective_scan_ref


def test_scan_matches_explicit_recurrence():
    g = torch.Generator().manual_seed(0)
    b, d, l, n = 1, 2, 5, 3
    u, delta = torch.randn(b, d, l, generator=g), torch.rand(b, d, l, generator=g)
    A = -torch.rand(d, n, generator=g)
    B, C = torch.randn(b, n, l, generator=g), torch.randn(b, n, l, generator=g)
    D = torch.randn(d, generator=g)
    out = selective_scan_ref(u, delta, A, B, C, D=D).double()
    for dd in range(d):
        x = torch.zeros(n, dtype=torch.float64)
        for t in range(l):
            x = torch.exp(delta[0, dd, t].double() * A[dd].double()) * x + \
                delta[0, dd, t].double() * B[0, :, t].double() * u[0, dd, t].double()
            y = (C[0, :, t].double() * x).sum() + D[dd].double() * u[0, dd, t].double()
            assert abs(float(out[0, dd, t]) - float(y)) < 1e-5
