"""GPU: the HIP Mamba selective scan (dna_amd.mamba.selective_scan_fn) against the float64 CPU
restatement of mamba_ssm's selective_scan_ref (oracle/selective_scan_ref.py; parity unpinned:
mamba_ssm is not available to run). Tolerances: fp32 -- max relative error 1e-4 (forward) /
1e-3 (gradients, fp32 atomics for dB/dC); bf16 inputs -- 3e-2."""
import pytest
import torch

from oracle.selective_scan_ref import selective_scan_ref

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _inputs(b, d, l, n, seed=0, dtype=torch.float32):
    g = torch.Generator().manual_seed(seed)
    u = torch.randn(b, d, l, generator=g)
    delta = torch.randn(b, d, l, generator=g) * 0.5 - 1.0
    A = -torch.exp(torch.randn(d, n, generator=g) * 0.5)
    B = torch.randn(b, n, l, generator=g)
    C = torch.randn(b, n, l, generator=g)
    D = torch.randn(d, generator=g)
    z = torch.randn(b, d, l, generator=g)
    bias = torch.randn(d, generator=g) * 0.1
    return [t.to(dtype) if t.dim() == 3 else t for t in (u, delta, A, B, C, D, z, bias)]


def _rel(a, b):
    return float((a.double() - b.double()).abs().max() / (b.double().abs().max() + 1e-30))


@pytest.mark.parametrize("b,d,l,n,use_z", [(2, 5, 700, 16, True), (1, 3, 1024, 8, False),
                                           (3, 2, 64, 4, True), (1, 4, 2048, 16, True),
                                           # dim % 16 == 0 / % 8 == 0: LDS-staged block kernels
                                           (2, 16, 1300, 16, True), (1, 8, 777, 8, False),
                                           (2, 32, 1536, 4, True)])
def test_selective_scan_fwd_bwd_vs_oracle(b, d, l, n, use_z):
    from dna_amd.mamba import selective_scan_fn
    u, delta, A, B, C, D, z, bias = _inputs(b, d, l, n, seed=l + n)
    z = z if use_z else None
    ref_in = [t.double().requires_grad_(True) if t is not None else None
              for t in (u, delta, A, B, C, D, z, bias)]
    ref, ref_last = selective_scan_ref(*ref_in[:5], D=ref_in[5], z=ref_in[6], delta_bias=ref_in[7],
                                       delta_softplus=True, return_last_state=True)
    dout = torch.randn(b, d, l, generator=torch.Generator().manual_seed(9))
    ref.backward(dout.double())
    dev_in = [t.to(DEV).requires_grad_(True) if t is not None else None
              for t in (u, delta, A, B, C, D, z, bias)]
    out, last = selective_scan_fn(*dev_in[:5], D=dev_in[5], z=dev_in[6], delta_bias=dev_in[7],
                                  delta_softplus=True, return_last_state=True)
    assert _rel(out.detach().cpu(), ref.detach()) < 1e-4
    assert _rel(last.cpu(), ref_last.detach()) < 1e-4
    out.backward(dout.to(DEV))
    for name, mine, theirs in zip(("u", "delta", "A", "B", "C", "D", "z", "bias"), dev_in, ref_in):
        if mine is None:
            continue
        assert _rel(mine.grad.cpu(), theirs.grad) < 1e-3, name


@pytest.mark.parametrize("d", [4, 16])
def test_selective_scan_bf16(d):
    from dna_amd.mamba import selective_scan_fn
    u, delta, A, B, C, D, z, bias = _inputs(2, d, 1500, 16, seed=3)
    ref = selective_scan_ref(u.bfloat16().float(), delta.bfloat16().float(), A,
                             B.bfloat16().float(), C.bfloat16().float(), D, z.bfloat16().float(),
                             bias, delta_softplus=True)
    out = selective_scan_fn(*(t.to(DEV).bfloat16() for t in (u, delta)), A.to(DEV),
                            *(t.to(DEV).bfloat16() for t in (B, C)), D=D.to(DEV),
                            z=z.to(DEV).bfloat16(), delta_bias=bias.to(DEV), delta_softplus=True)
    assert out.dtype == torch.bfloat16 and _rel(out.float().cpu(), ref.float()) < 3e-2

