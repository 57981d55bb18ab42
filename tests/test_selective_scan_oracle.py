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


import numpy as np  # noqa: E402
import pytest  # noqa: E402


@pytest.mark.parametrize("b,d,l,n,use_z,use_D,softplus", [(2, 3, 257, 16, True, True, True),
                                                          (1, 4, 100, 8, False, True, True),
                                                          (1, 2, 64, 4, True, False, False)])
def test_c_oracle_matches_python_restatement(b, d, l, n, use_z, use_D, softplus):
    """oracle/selective_scan_ref.c (analytic float64 backward, the checker at L = 131,072) ==
    the Python float64 restatement, forward and every gradient through torch autograd."""
    from oracle.selective_scan_c import scan_bwd, scan_fwd
    g = torch.Generator().manual_seed(l + n)
    mk = lambda *s: torch.randn(*s, generator=g, dtype=torch.float64)
    u, z = mk(b, d, l), mk(b, d, l)
    delta = mk(b, d, l) * 0.5 - 1.0
    A = -torch.exp(mk(d, n) * 0.5)
    B, C = mk(b, n, l), mk(b, n, l)
    D, bias = mk(d), mk(d) * 0.1
    dout = mk(b, d, l)
    ins = [t.clone().requires_grad_(True) for t in (u, delta, A, B, C, D, z, bias)]
    kw = dict(D=ins[5] if use_D else None, z=ins[6] if use_z else None,
              delta_bias=ins[7] if softplus else None, delta_softplus=softplus)
    ref, last = selective_scan_ref(*ins[:5], return_last_state=True, **kw)
    ref.backward(dout)
    npkw = dict(D=D.numpy() if use_D else None, z=z.numpy() if use_z else None,
                delta_bias=bias.numpy() if softplus else None, delta_softplus=softplus)
    out, clast = scan_fwd(u.numpy(), delta.numpy(), A.numpy(), B.numpy(), C.numpy(), **npkw)
    assert np.abs(out - ref.detach().numpy()).max() < 1e-12 * max(1, np.abs(out).max())
    assert np.abs(clast - last.detach().numpy()).max() < 1e-12 * max(1, np.abs(clast).max())
    gr = scan_bwd(u.numpy(), delta.numpy(), A.numpy(), B.numpy(), C.numpy(), dout.numpy(), **npkw)
    names = ["u", "delta", "A", "B", "C", "D", "z", "delta_bias"]
    for name, t in zip(names, ins):
        if name not in gr:
            continue
        want = t.grad.numpy()
        assert np.abs(gr[name] - want).max() <= 1e-10 * max(1.0, np.abs(want).max()), name
