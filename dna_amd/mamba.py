"""Mamba selective scan on MI355X: `selective_scan_fn` with mamba_ssm's signature and semantics.

Caduceus (reference src/models/caduceus/modeling_caduceus.py:68-121) runs two Mamba blocks
(forward and reverse-complement direction) whose core op is mamba_ssm's `selective_scan_fn`
(external, not vendored in the reference; parity unpinned -- see oracle/selective_scan_ref.py).
This is that op for the Mamba-1 call Mamba.forward makes: A real [dim, d_state], B/C
input-dependent [batch, d_state, len], D and delta_bias per channel, optional z gating,
delta_softplus. Forward and backward run dna_amd/csrc/selective_scan.hip; no CPU fallback.
"""
import torch

from . import _native as N
from .functional import _dt, _gpu, _p, _timed


class SelectiveScan(torch.autograd.Function):
    @staticmethod
    def forward(ctx, u, delta, A, B, C, D, z, delta_bias, delta_softplus, return_last_state):
        _gpu(u, delta, A, B, C, D, z, delta_bias)
        b, d, l = u.shape
        n = A.shape[1]
        assert delta.shape == u.shape and B.shape == (b, n, l) and C.shape == (b, n, l)
        assert z is None or z.shape == u.shape
        dt = u.dtype
        u, delta = u.contiguous(), delta.contiguous().to(dt)
        B, C = B.contiguous().to(dt), C.contiguous().to(dt)
        z = None if z is None else z.contiguous().to(dt)
        A32 = A.detach().float().contiguous()
        D32 = None if D is None else D.detach().float().contiguous()
        db32 = None if delta_bias is None else delta_bias.detach().float().contiguous()
        out = torch.empty_like(u)
        states = torch.empty(N.lib().dna_selective_scan_states(b, d, l, n), device=u.device,
                             dtype=torch.float32)
        last = torch.empty(b, d, n, device=u.device, dtype=torch.float32) if return_last_state else None
        with _timed("selective_scan_fwd", b * d * l * 3 * u.element_size(), "byte"):
            N.call("dna_selective_scan_fwd", u.data_ptr(), delta.data_ptr(), A32.data_ptr(),
                   B.data_ptr(), C.data_ptr(), _p(D32), _p(z), _p(db32), int(bool(delta_softplus)),
                   _dt(u), b, d, l, n, out.data_ptr(), states.data_ptr(), _p(last), N.stream_ptr())
        ctx.save_for_backward(u, delta, A32, B, C, D32, z, db32, states)
        ctx.cfg = (bool(delta_softplus), A.dtype, B.dtype, C.dtype, D is not None,
                   delta_bias is not None)
        if return_last_state:
            ctx.mark_non_differentiable(last)
            return out, last
        return out

    @staticmethod
    def backward(ctx, dout, *rest):
        u, delta, A32, B, C, D32, z, db32, states = ctx.saved_tensors
        softplus, adt, bdt, cdt, has_D, has_bias = ctx.cfg
        b, d, l = u.shape
        n = A32.shape[1]
        dout = dout.contiguous().to(u.dtype)
        du, ddelta = torch.empty_like(u), torch.empty_like(u)
        dz = torch.empty_like(u) if z is not None else None
        dA = torch.zeros_like(A32)
        dB = torch.zeros(b, n, l, device=u.device, dtype=torch.float32)
        dC = torch.zeros_like(dB)
        dD = torch.zeros(d, device=u.device, dtype=torch.float32) if has_D else None
        dbias = torch.zeros(d, device=u.device, dtype=torch.float32) if has_bias else None
        with _timed("selective_scan_bwd", b * d * l * 5 * u.element_size(), "byte"):
            N.call("dna_selective_scan_bwd", u.data_ptr(), delta.data_ptr(), A32.data_ptr(),
                   B.data_ptr(), C.data_ptr(), _p(D32), _p(z), _p(db32), int(softplus), _dt(u),
                   b, d, l, n, states.data_ptr(), dout.data_ptr(), du.data_ptr(), ddelta.data_ptr(),
                   dA.data_ptr(), dB.data_ptr(), dC.data_ptr(), _p(dD), _p(dz), _p(dbias),
                   N.stream_ptr())
        return (du, ddelta, dA.to(adt), dB.to(bdt), dC.to(cdt), dD, dz, dbias, None, None)


def selective_scan_fn(u, delta, A, B, C, D=None, z=None, delta_bias=None, delta_softplus=False,
                      return_last_state=False):
    """mamba_ssm.ops.selective_scan_interface.selective_scan_fn (Mamba-1 form: real A, one group)."""
    if A.is_complex():
        raise NotImplementedError("complex A (S4D-style) is not used by Mamba/Caduceus")
    if B.dim() != 3 or C.dim() != 3:
        raise NotImplementedError("B/C must be input-dependent [batch, d_state, len] (Mamba form)")
    return SelectiveScan.apply(u, delta, A, B, C, D, z, delta_bias, delta_softplus, return_last_state)
