"""CPU restatement of the Mamba selective scan used by Caduceus.

TEST INFRASTRUCTURE ONLY: imported by tests/ as the checker; the product path
(dna_amd.mamba.selective_scan_fn) runs the HIP kernels of dna_amd/csrc/selective_scan.hip.

PARITY UNPINNED: the reference calls `mamba_ssm` (Caduceus BiMambaWrapper ->
mamba_ssm.modules.mamba_simple.Mamba, reference src/models/caduceus/modeling_caduceus.py:10,
:68-121), which is neither vendored in /root/reference nor installed here, so no reference
output could be produced. This file restates the published reference implementation of
mamba_ssm (`selective_scan_ref`, mamba_ssm/ops/selective_scan_interface.py, mamba-ssm 1.x/2.x)
for the Mamba-1 call Mamba.forward makes (A real [D, N], B/C input-dependent [batch, N, L],
one group):
    delta = softplus(delta + delta_bias)            (if delta_softplus)
    x_t   = exp(delta_t * A) * x_{t-1} + delta_t * B_t * u_t        (per channel d, state n)
    y_t   = sum_n C_t[n] x_t[n] + D u_t ;  out = y * silu(z)        (if z is given)
Backward: torch autograd of this float64 restatement.
"""
import torch
import torch.nn.functional as F


def selective_scan_ref(u, delta, A, B, C, D=None, z=None, delta_bias=None, delta_softplus=False,
                       return_last_state=False):
    """u, delta, z [b, d, l]; A [d, n]; B, C [b, n, l]; D, delta_bias [d] -> out [b, d, l]."""
    dtype_in = u.dtype
    u = u.double()
    delta = delta.double()
    if delta_bias is not None:
        delta = delta + delta_bias[..., None].double()
    if delta_softplus:
        delta = F.softplus(delta)
    A = A.double()
    B = B.double()
    C = C.double()
    b, d, l = u.shape
    x = u.new_zeros((b, d, A.shape[1]))
    deltaA = torch.exp(torch.einsum("bdl,dn->bdln", delta, A))
    deltaB_u = torch.einsum("bdl,bnl,bdl->bdln", delta, B, u)
    ys = []
    for i in range(l):
        x = deltaA[:, :, i] * x + deltaB_u[:, :, i]
        ys.append(torch.einsum("bdn,bn->bd", x, C[:, :, i]))
    y = torch.stack(ys, dim=2)
    out = y if D is None else y + u * D.double()[:, None]
    if z is not None:
        out = out * F.silu(z.double())
    out = out.to(dtype_in)
    return (out, x) if return_last_state else out
