"""Mamba selective scan on MI355X: `selective_scan_fn` with mamba_ssm's signature and semantics.

Caduceus (reference src/models/caduceus/modeling_caduceus.py:68-121) runs two Mamba blocks
(forward and reverse-complement direction) whose core op is mamba_ssm's `selective_scan_fn`
(external, not vendored in the reference; parity unpinned -- see oracle/selective_scan_ref.py).
This is that op for the Mamba-1 call Mamba.forward makes: A real [dim, d_state], B/C
input-dependent [batch, d_state, len], D and delta_bias per channel, optional z gating,
delta_softplus. Forward and backward run dna_amd/csrc/selective_scan.hip; no CPU fallback.

Around it: `Mamba` (mamba_ssm.modules.mamba_simple.Mamba 1.x, restated: same parameters, names
and forward math on its non-fused path) with the depthwise causal conv1d + SiLU on the HIP
kernel of dna_amd/csrc/causal_conv.hip, x_proj / dt_proj channel-major on the strided MFMA GEMM
(dna_amd/csrc/gemm_strided.hip, `ChannelLinear`), and `BiMambaWrapper` (the reference's own wrapper,
modeling_caduceus.py:68-121: forward + flipped reverse Mamba, tied in/out projections, "add" or
"ew_multiply").
"""
import math
import os

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import _native as N
from . import functional as DF
from .functional import _dt, _gpu, _p, _timed, strided_gemm as _strided_gemm


_XDBL_SPLIT = os.environ.get("DNA_XDBL_SPLIT", "1") != "0"  # 0: autograd's slice nodes (A/B)
_NEGEXP = os.environ.get("DNA_NEGEXP", "1") != "0"  # 0: -torch.exp(A_log) through autograd (A/B)


class GradSink:
    """Hand-off of the scan's du to the x_proj backward (Mamba.forward): x feeds both the scan
    (u) and x_proj, so autograd would add the two gradients of x in a separate pass over
    [b, E, L]. With a sink the scan returns no gradient for u and leaves du here; x_proj's
    backward then accumulates its data gradient into du in the GEMM epilogue and returns the sum
    as the gradient of x -- the same total, one pass less. x_proj's backward necessarily runs
    after the scan's (it needs dB / dC)."""
    __slots__ = ("du", "dB", "dC", "want_bc")

    def __init__(self):
        self.du = None
        # with XdblSplit: the scan also leaves its fp32 dB / dC here, and the split's backward
        # converts them straight into the x_dbl gradient (no separate .to(bf16) passes)
        self.dB = self.dC = None
        self.want_bc = False


class SelectiveScan(torch.autograd.Function):
    @staticmethod
    def forward(ctx, u, delta, A, B, C, D, z, delta_bias, delta_softplus, return_last_state,
                sink=None):
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
        # algorithmic HBM bytes: u, delta (+ z), B, C in, out
        nbytes = (b * d * l * (4 if z is not None else 3) + 2 * b * n * l) * u.element_size()
        with _timed("selective_scan_fwd", nbytes, "byte"):
            N.call("dna_selective_scan_fwd", u.data_ptr(), delta.data_ptr(), A32.data_ptr(),
                   B.data_ptr(), C.data_ptr(), _p(D32), _p(z), _p(db32), int(bool(delta_softplus)),
                   _dt(u), b, d, l, n, out.data_ptr(), states.data_ptr(), _p(last), N.stream_ptr())
        ctx.save_for_backward(u, delta, A32, B, C, D32, z, db32, states)
        ctx.cfg = (bool(delta_softplus), A.dtype, B.dtype, C.dtype, D is not None,
                   delta_bias is not None)
        ctx.sink = sink
        ctx.refs = (D, delta_bias)  # the parameters themselves when passed as such (fp32)
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
        # the kernel sums dA / dB / dC / dD / d(delta_bias) with atomics: zeroed buffers, one fill
        # for the small ones and one for dB + dC; dD and d(delta_bias) of FlatParams-owned
        # parameters are added straight into their fp32 gradient slices instead (no buffer, no
        # AccumulateGrad add)
        D_ref, bias_ref = ctx.refs
        dD_direct = has_D and DF._param_grads_direct((D_ref,))
        db_direct = has_bias and DF._param_grads_direct((bias_ref,))
        nA = A32.numel()
        small = torch.zeros(nA + (d if has_D and not dD_direct else 0)
                            + (d if has_bias and not db_direct else 0),
                            device=u.device, dtype=torch.float32)
        dA = small[:nA].view_as(A32)
        o = nA
        if not has_D:
            dD = None
        elif dD_direct:
            dD = D_ref.grad
        else:
            dD, o = small[o:o + d], o + d
        if not has_bias:
            dbias = None
        elif db_direct:
            dbias = bias_ref.grad
        else:
            dbias = small[o:o + d]
        dBC = torch.zeros(2, b, n, l, device=u.device, dtype=torch.float32)
        dB, dC = dBC[0], dBC[1]
        # u, delta, dout (+ z), B, C in; du, ddelta (+ dz) out; dB, dC fp32 out
        nz = 2 if z is not None else 0
        nbytes = (b * d * l * (5 + nz) + 2 * b * n * l) * u.element_size() + 2 * b * n * l * 4
        with _timed("selective_scan_bwd", nbytes, "byte"):
            N.call("dna_selective_scan_bwd", u.data_ptr(), delta.data_ptr(), A32.data_ptr(),
                   B.data_ptr(), C.data_ptr(), _p(D32), _p(z), _p(db32), int(softplus), _dt(u),
                   b, d, l, n, states.data_ptr(), dout.data_ptr(), du.data_ptr(), ddelta.data_ptr(),
                   dA.data_ptr(), dB.data_ptr(), dC.data_ptr(), _p(dD), _p(dz), _p(dbias),
                   N.stream_ptr())
        if ctx.sink is not None and ctx.sink.want_bc:
            ctx.sink.dB, ctx.sink.dC = dB, dC
            gB = gC = None
        else:
            gB, gC = dB.to(bdt), dC.to(cdt)
        if ctx.sink is not None:
            ctx.sink.du = du
            du = None
        for direct, q in ((dD_direct, D_ref), (db_direct, bias_ref)):
            if direct:
                notify = getattr(q, "_dna_notify", None)
                if notify is not None:
                    notify(q)
        return (du, ddelta, dA.to(adt), gB, gC, None if dD_direct else dD, dz,
                None if db_direct else dbias, None, None, None)


def selective_scan_fn(u, delta, A, B, C, D=None, z=None, delta_bias=None, delta_softplus=False,
                      return_last_state=False):
    """mamba_ssm.ops.selective_scan_interface.selective_scan_fn (Mamba-1 form: real A, one group)."""
    if A.is_complex():
        raise NotImplementedError("complex A (S4D-style) is not used by Mamba/Caduceus")
    if B.dim() != 3 or C.dim() != 3:
        raise NotImplementedError("B/C must be input-dependent [batch, d_state, len] (Mamba form)")
    return SelectiveScan.apply(u, delta, A, B, C, D, z, delta_bias, delta_softplus, return_last_state)


class CausalConv1d(torch.autograd.Function):
    """act(conv1d(x, w, b, padding=K-1, groups=C)[..., :L]) on x [B, C, L] (any batch stride,
    unit channel/position strides), act = SiLU or identity (dna_causal_conv1d_fwd/bwd)."""

    @staticmethod
    def forward(ctx, x, weight, bias, silu):
        _gpu(x, weight)
        B, C, L = x.shape
        if x.stride(2) != 1 or x.stride(1) != L:
            x = x.contiguous()
        if L % 8 == 0 and (x.data_ptr() % 16 or x.stride(0) % 8):
            # the backward's 16-B path (taken for every L % 8 == 0) needs 16-B aligned rows
            x = x.clone(memory_format=torch.contiguous_format)
        K = weight.shape[-1]
        w = weight.detach().reshape(C, K).float().contiguous()
        b = None if bias is None else bias.detach().float().contiguous()
        out = torch.empty(B, C, L, device=x.device, dtype=x.dtype)
        with _timed("causal_conv_fwd", 2 * B * C * L * x.element_size(), "byte"):
            N.call("dna_causal_conv1d_fwd", x.data_ptr(), x.stride(0), _dt(x), w.data_ptr(), _p(b),
                   B, C, L, K, int(bool(silu)), out.data_ptr(), N.stream_ptr())
        ctx.save_for_backward(x, w, b)
        ctx.cfg = (bool(silu), weight.shape, weight.dtype, bias is not None)
        ctx.refs = (weight, bias)
        return out

    @staticmethod
    def backward(ctx, dout):
        x, w, b = ctx.saved_tensors
        silu, wshape, wdtype, has_b = ctx.cfg
        B, C, L = x.shape
        K = w.shape[1]
        dout = dout.contiguous().to(x.dtype)
        if L % 8 == 0 and dout.data_ptr() % 16:
            dout = dout.clone()
        dx = torch.empty(B, C, L, device=x.device, dtype=x.dtype)
        rows = N.lib().dna_causal_conv1d_part_rows(B, L)
        part = torch.empty(rows, C * (K + 1), device=x.device, dtype=torch.float32)
        with _timed("causal_conv_bwd", 3 * B * C * L * x.element_size(), "byte"):
            N.call("dna_causal_conv1d_bwd", x.data_ptr(), x.stride(0), _dt(x), w.data_ptr(), _p(b),
                   dout.data_ptr(), B, C, L, K, int(silu), dx.data_ptr(), dx.stride(0),
                   part.data_ptr(), N.stream_ptr())
        s = part.sum(0) if (C * (K + 1)) % 64 else None
        if s is None:
            s = torch.empty(C * (K + 1), device=x.device, dtype=torch.float32)
            N.call("dna_colsum_f32", part.data_ptr(), rows, C * (K + 1), s.data_ptr(), 0, N.stream_ptr())
        s = s.view(C, K + 1)
        wref, bref = ctx.refs
        if DF._param_grads_direct((wref, bref)):
            # FlatParams-owned: the [C][K+1] sums go straight into the fp32 gradient slices (two
            # strided adds instead of two copies and two AccumulateGrad adds)
            wref.grad.view(C, K).add_(s[:, :K])
            if bref is not None:
                bref.grad.add_(s[:, K])
            for q in (wref, bref):
                notify = getattr(q, "_dna_notify", None) if q is not None else None
                if notify is not None:
                    notify(q)
            return dx, None, None, None
        db = s[:, K].contiguous() if has_b else None
        return dx, s[:, :K].reshape(wshape).to(wdtype), db, None


class NegExp(torch.autograd.Function):
    """A = -exp(A_log) (mamba_ssm Mamba.forward) with a one-kernel backward, dA_log = dA * A,
    added straight into a FlatParams-owned A_log's fp32 gradient (no separate neg / mul /
    AccumulateGrad launches)."""

    @staticmethod
    def forward(ctx, a_log):
        A = torch.exp(a_log.float()).neg_()
        ctx.save_for_backward(A)
        ctx.ref = a_log
        return A

    @staticmethod
    def backward(ctx, dA):
        (A,) = ctx.saved_tensors
        ref = ctx.ref
        if ref.dtype == torch.float32 and DF._param_grads_direct((ref,)):
            ref.grad.addcmul_(dA, A)
            notify = getattr(ref, "_dna_notify", None)
            if notify is not None:
                notify(ref)
            return None
        return (dA * A).to(ref.dtype)


class XdblSplit(torch.autograd.Function):
    """(x_dbl[:, :R], x_dbl[:, R:R+N], x_dbl[:, R+N:]) as views; the backward writes the three
    slice gradients into one [b, R + 2N, L] buffer (one copy each, converting dtype on the way)
    -- autograd's three SliceBackward nodes zero-fill a full-size tensor apiece and add them."""

    @staticmethod
    def forward(ctx, x_dbl, R, Ns, sink=None):
        ctx.set_materialize_grads(False)  # a slice without gradient arrives as None, not zeros
        ctx.cfg = (x_dbl.shape, x_dbl.dtype, x_dbl.device, R, Ns)
        ctx.sink = sink
        if sink is not None:
            sink.want_bc = True
        return x_dbl[:, :R], x_dbl[:, R:R + Ns], x_dbl[:, R + Ns:]

    @staticmethod
    def backward(ctx, g_dt, g_b, g_c):
        shape, dtype, dev, R, Ns = ctx.cfg
        sink = ctx.sink
        if sink is not None:  # the scan's fp32 dB / dC, converted by the copies below
            g_b = sink.dB if g_b is None else g_b
            g_c = sink.dC if g_c is None else g_c
            sink.dB = sink.dC = None
        g = torch.empty(shape, device=dev, dtype=dtype)
        for gi, lo, hi in ((g_dt, 0, R), (g_b, R, R + Ns), (g_c, R + Ns, shape[1])):
            if gi is None:
                g[:, lo:hi].zero_()
            else:
                g[:, lo:hi].copy_(gi)
        return g, None, None, None


class ChannelLinear(torch.autograd.Function):
    """y[b, M, L] = W[M, K] . x[b, K, L] with x channel-major (unit position stride, any channel /
    batch stride): the x_proj and dt_proj products of mamba_ssm Mamba.forward (`x_proj(rearrange(x,
    "b d l -> (b l) d"))`, `dt_proj.weight @ dt.t()`) computed without transposing x, so B / C /
    delta come out in the [b, ·, L] layout the scan reads. Forward and backward on
    dna_gemm_bf16_strided (bf16, under autocast) or dna_gemm_f32_strided (fp32); dW's contraction
    over b and L runs as fp32 split-K slices summed by dna_sum_slices_accum."""

    @staticmethod
    def forward(ctx, x, weight, sink=None):
        _gpu(x, weight)
        b, K, L = x.shape
        M = weight.shape[0]
        assert weight.shape[1] == K
        if torch.is_autocast_enabled("cuda"):
            dt = torch.get_autocast_dtype("cuda")
        else:
            dt = torch.promote_types(x.dtype, weight.dtype)
        if dt not in (torch.bfloat16, torch.float32):
            raise NotImplementedError(f"ChannelLinear: {dt}")
        xin = x.to(dt)
        if xin.stride(2) != 1:
            xin = xin.contiguous()
        w = _lowp(weight, dt)
        y = torch.empty(b, M, L, device=x.device, dtype=dt)
        with _timed("mamba_proj", (b * K * L + b * M * L) * xin.element_size(), "byte"):
            _strided_gemm(w, (K, 1, 0), xin, (xin.stride(1), 1, xin.stride(0)), y, (L, M * L),
                          M, L, K, b)
        ctx.save_for_backward(xin, w)
        ctx.cfg = (x.dtype, weight.dtype)
        ctx.sink = sink
        ctx.weight = weight
        return y

    @staticmethod
    def backward(ctx, dy):
        xin, w = ctx.saved_tensors
        xdt, wdt = ctx.cfg
        du = None
        if ctx.sink is not None:  # the scan's du for the same x (GradSink)
            du, ctx.sink.du = ctx.sink.du, None
        b, K, L = xin.shape
        M = w.shape[0]
        dy = dy.to(xin.dtype)
        if dy.stride(2) != 1:
            dy = dy.contiguous()
        dx = dw = None
        es = xin.element_size()
        if ctx.needs_input_grad[0]:  # dx[b, K, L] = W^T[K, M] . dy[b, M, L]
            acc = (du is not None and du.dtype == xin.dtype == torch.bfloat16 and du.is_contiguous()
                   and du.shape == (b, K, L))
            dx = du if acc else torch.empty(b, K, L, device=xin.device, dtype=xin.dtype)
            with _timed("mamba_proj", (b * M * L + (3 if acc else 1) * b * K * L) * es, "byte"):
                _strided_gemm(w, (1, K, 0), dy, (dy.stride(1), 1, dy.stride(0)), dx, (L, K * L),
                              K, L, M, b, accumulate=acc)
            if du is not None and not acc:
                dx = dx + du.to(dx.dtype)
        if ctx.needs_input_grad[1]:  # dW[M, K] = sum_b dy[b] . x[b]^T (contraction over L)
            s = int(N.lib().dna_gemm_strided_splits(M, K, L, b))
            part = torch.empty(b * s, M, K, device=xin.device, dtype=torch.float32)
            with _timed("mamba_proj", (b * M * L + b * K * L) * es, "byte"):
                _strided_gemm(dy, (dy.stride(1), 1, dy.stride(0)), xin,
                              (1, xin.stride(1), xin.stride(0)), part, (K, M * K), M, K, L, b, s,
                              out_f32=True)
            dw = _finish_wgrad(part, ctx.weight, (M, K), wdt)
        return (None if dx is None else dx.to(xdt)), dw, None


def _wgrad_tokens(dy, sa, x, sb, M, Nn, T, batch, part=None, row0=0, rows_total=None):
    """fp32 split-K slices of dW[m][n] = sum_{b, t} A(m, t) B(t, n) (the Mamba projections' weight
    gradients: contraction over every token) on the strided MFMA GEMM. Returns (part, splits);
    slices are [z][rows_total][Nn], this call filling rows row0 .. row0 + M."""
    s = int(N.lib().dna_gemm_strided_splits(M, Nn, T, batch))
    rt = M if rows_total is None else rows_total
    if part is None:
        part = torch.empty(batch * s, rt, Nn, device=dy.device, dtype=torch.float32)
    assert part.shape[0] == batch * s
    DF.strided_gemm(dy, sa, x, sb, part[:, row0:], (Nn, rt * Nn), M, Nn, T, batch, s, out_f32=True)
    return part, s


def _lowp(weight, dt):
    """The weight in the compute dtype: the trainer's persistent bf16 copy when one exists
    (ModuleTrainer: FlatParams' shadow, rewritten by the fused AdamW step -- the same bits as
    autocast's cast), else a cast."""
    lp = getattr(weight, "_dna_lp", None)
    if dt == torch.bfloat16 and lp is not None:
        return lp
    return weight.detach().to(dt).contiguous()


def _finish_wgrad(part, weight, shape, dtype):
    """A weight gradient from its fp32 split-K slices: summed straight into the flat fp32 .grad
    when a FlatParams trainer owns the parameter (ModuleTrainer enables it; the bucket reducer is
    notified and autograd gets None, so its AccumulateGrad add -- two per tied BiMamba
    projection -- never runs), else returned."""
    g = weight.grad if getattr(weight, "_dna_direct", False) else None
    if g is not None and g.dtype == torch.float32 and g.is_contiguous() and \
            tuple(g.shape) == tuple(shape):
        N.call("dna_sum_slices_accum", part.data_ptr(), part.shape[0], g.numel(), g.data_ptr(),
               N.stream_ptr())
        notify = getattr(weight, "_dna_notify", None)
        if notify is not None:
            notify(weight)
        return None
    return _sum_parts(part, shape, dtype)


def _sum_parts(part, shape, dtype):
    out = torch.empty(shape, device=part.device, dtype=torch.float32)
    N.call("dna_sum_slices", part.data_ptr(), part.shape[0], out.numel(), out.data_ptr(),
           N.stream_ptr())
    return out.to(dtype)


class DhSink:
    """Hand-off between the two in_proj backwards of a fused BiMambaWrapper (both directions read
    the same hidden states): the first backward to run writes its dh (in forward position order)
    here and returns no gradient; the second accumulates its dh into the same buffer in the
    GEMM epilogue and returns the sum -- autograd's add of the two gradients never runs."""
    __slots__ = ("dh",)

    def __init__(self):
        self.dh = None


def _rows_from_end(t, b, L, d):
    """[b, L, d]-strided view of t whose data_ptr is row L-1 of batch 0: with row stride -d the
    GEMMs walk the sequence backwards (the BiMamba reverse direction, no flipped copy)."""
    return t.view(b, L, d)[:, L - 1:]


class InProj(torch.autograd.Function):
    """in_proj of mamba_ssm Mamba.forward, channel-major as the reference computes it
    (`in_proj.weight @ rearrange(hidden, "b l d -> d (b l)")`), returning x and z ([b, E, L]
    views of one [b, 2E, L] product) so the backward takes dx and dz apart (no cat of the two
    halves). The forward on the weight-stationary projection kernel (csrc/proj_cm.hip) or the
    strided MFMA GEMM; the data gradient dh = g_x^T W_x + g_z^T W_z contracts over both halves
    in one pass (dna_gemm_bf16_strided_cat); the weight gradient -- a contraction over all b*L
    tokens into [2E, d] -- as fp32 split-K slices.
    reverse: the sequence is read backwards (position l of x / z is h[L-1-l]), which is the
    BiMambaWrapper reverse direction `mamba_rev(hidden.flip(1))` without the flipped copy; its dh
    is written back in forward order. sink (bf16): see DhSink."""

    @staticmethod
    def forward(ctx, h, weight, reverse=False, sink=None):
        _gpu(h, weight)
        b, L, d = h.shape
        E2 = weight.shape[0]
        if torch.is_autocast_enabled("cuda"):
            dt = torch.get_autocast_dtype("cuda")
        else:
            dt = torch.promote_types(h.dtype, weight.dtype)
        if dt not in (torch.bfloat16, torch.float32):
            raise NotImplementedError(f"InProj: {dt}")
        if (reverse or sink is not None) and dt != torch.bfloat16:
            raise NotImplementedError("InProj: reverse / sink need bf16 (autocast)")
        h2 = h.reshape(b * L, d).to(dt).contiguous()
        w = _lowp(weight, dt)
        xz = torch.empty(b, E2, L, device=h.device, dtype=dt)
        with _timed("mamba_proj", (b * L * d + b * E2 * L) * h2.element_size(), "byte"):
            # xz[b][c][l] = sum_j W[c][j] h[b][l'][j],  l' = l or L-1-l
            if dt == torch.bfloat16 and d in (64, 128, 256):
                # register-resident weight, h streamed (csrc/proj_cm.hip)
                N.call("dna_proj_cm_bf16", w.data_ptr(), h2.data_ptr(), None, E2, L, d, b,
                       int(reverse), xz.data_ptr(), N.stream_ptr())
            elif reverse:
                _strided_gemm(w, (d, 1, 0), _rows_from_end(h2, b, L, d), (1, -d, L * d), xz,
                              (L, E2 * L), E2, L, d, b)
            else:
                _strided_gemm(w, (d, 1, 0), h2, (1, d, L * d), xz, (L, E2 * L), E2, L, d, b)
        ctx.save_for_backward(h2, w)
        ctx.cfg = (b, L, h.dtype, weight.dtype, bool(reverse))
        ctx.sink = sink
        ctx.weight = weight
        E = E2 // 2
        return xz[:, :E], xz[:, E:]

    @staticmethod
    def backward(ctx, dx, dz):
        h2, w = ctx.saved_tensors
        b, L, hdt, wdt, rev = ctx.cfg
        sink = ctx.sink
        E2, d = w.shape
        E = E2 // 2
        T = b * L
        dt = h2.dtype
        es = h2.element_size()
        halves = [(i, g.to(dt).contiguous()) for i, g in enumerate((dx, dz)) if g is not None]
        dh = dw = None
        if ctx.needs_input_grad[0]:
            # dh[b][l'][j] = sum_c g[b][c][l] W[c][j]: A(m = l, k = c) = g[b][c][l]; the rows of
            # the reverse direction land at l' = L-1-l (C walked backwards from row L-1)
            acc = sink is not None and sink.dh is not None
            dh = sink.dh if acc else torch.empty(b, L, d, device=h2.device, dtype=dt)
            cbase, ldc = (_rows_from_end(dh, b, L, d), -d) if rev else (dh, d)
            if not halves:
                if not acc:
                    dh.zero_()
            elif len(halves) == 2 and dt == torch.bfloat16 and E % 32 == 0:
                # the two-operand contraction splits K at E, which must be a whole number of
                # the kernel's 32-deep K-steps (dna_gemm_bf16_strided_cat); other E take the
                # concatenated operand below
                with _timed("mamba_proj", (2 * T * E + (3 if acc else 1) * T * d) * es, "byte"):
                    N.call("dna_gemm_bf16_strided_cat", halves[0][1].data_ptr(),
                           halves[1][1].data_ptr(), E, 1, L, E * L, w.data_ptr(), d, 1, 0,
                           cbase.data_ptr(), ldc, L * d, 2 if acc else 0, None, None, L, d, E2,
                           b, 1, N.stream_ptr())
            else:
                if len(halves) == 2:  # fp32 parity mode / E % 32 != 0: one operand of both halves
                    g, wi = torch.cat([halves[0][1], halves[1][1]], 1), w
                else:
                    i, g = halves[0]
                    wi = w[i * E:(i + 1) * E]
                K = g.shape[1]
                with _timed("mamba_proj", (T * K + (3 if acc else 1) * T * d) * es, "byte"):
                    _strided_gemm(g, (1, L, K * L), wi, (d, 1, 0), cbase, (ldc, L * d), L, d, K,
                                  b, accumulate=acc)
            if sink is not None:
                if acc:
                    sink.dh = None
                else:  # the other direction's backward accumulates into it and returns the sum
                    sink.dh = dh
                    dh = None
            if dh is not None:
                dh = dh.to(hdt)
        if ctx.needs_input_grad[1]:
            if not halves:
                dw = torch.zeros_like(w, dtype=wdt)
            else:
                s = int(N.lib().dna_gemm_strided_splits(E, d, L, b))
                # both halves written in full when dx and dz are both there; else the missing
                # half's rows must read as zero
                alloc = torch.empty if len(halves) == 2 else torch.zeros
                part = alloc(s * b, E2, d, device=h2.device, dtype=torch.float32)
                hb, sbk = (_rows_from_end(h2, b, L, d), -d) if rev else (h2, d)
                for i, g in halves:  # dW[c][j] = sum_{b,l} g[b][c][l] h[b][l'][j]
                    _wgrad_tokens(g, (L, 1, E * L), hb, (sbk, 1, L * d), E, d, L, b, part, i * E, E2)
                dw = _finish_wgrad(part, ctx.weight, (E2, d), wdt)
        return dh, dw, None, None


class OutProj(torch.autograd.Function):
    """out_proj of mamba_ssm Mamba.forward on the scan output y [b, E, L] (channel-major):
    out [b, L, d] = y^T . W^T (+ bias, rounded to the compute dtype first as autocast's
    F.linear does). All three products on the strided MFMA GEMM: the forward reads y with unit
    token stride (no transpose), the data gradient goes straight into the channel-major
    [b, E, L] layout the scan's backward reads, the weight gradient (contraction over all b*L
    tokens into [d, E]) as fp32 split-K slices.
    into (bf16, the BiMambaWrapper "add" strategy): the reverse direction's output is added to
    the forward direction's output `into` in place, position l of y landing at L-1-l --
    `out + mamba_rev(hidden.flip(1)).flip(1)` without the two flips and the add."""

    @staticmethod
    def forward(ctx, y, weight, bias, into=None):
        _gpu(y, weight)
        b, E, L = y.shape
        if torch.is_autocast_enabled("cuda"):
            dt = torch.get_autocast_dtype("cuda")
        else:
            dt = torch.promote_types(y.dtype, weight.dtype)
        if dt not in (torch.bfloat16, torch.float32):
            raise NotImplementedError(f"OutProj: {dt}")
        yc = y.to(dt)
        if yc.stride(2) != 1 or yc.stride(1) != L:
            yc = yc.contiguous()
        w = _lowp(weight, dt)
        d = w.shape[0]
        bn = None if bias is None else bias.detach().to(dt).float().contiguous()
        if into is not None:
            if dt != torch.bfloat16 or into.dtype != dt or not into.is_contiguous() or \
                    into.shape != (b, L, d):
                raise NotImplementedError("OutProj(into=...): bf16 [b, L, d] contiguous target")
            out, cbase, ldc = into, _rows_from_end(into, b, L, d), -d
        else:
            out = torch.empty(b, L, d, device=y.device, dtype=dt)
            cbase, ldc = out, d
        with _timed("mamba_proj", (b * E * L + (3 if into is not None else 1) * b * L * d)
                    * yc.element_size(), "byte"):
            # out[b][l'][o] (+)= sum_e y[b][e][l] W[o][e] (+ bias[o])
            _strided_gemm(yc, (1, L, yc.stride(0)), w, (1, E, 0), cbase, (ldc, L * d), L, d, E, b,
                          bias_n=bn, accumulate=into is not None)
        ctx.save_for_backward(yc, w)
        ctx.cfg = (y.dtype, weight.dtype, None if bias is None else bias.dtype, into is not None)
        ctx.weight = weight
        if into is not None:
            ctx.mark_dirty(into)
        return out

    @staticmethod
    def backward(ctx, dout):
        yc, w = ctx.saved_tensors
        ydt, wdt, bdt, rev = ctx.cfg
        b, E, L = yc.shape
        d = w.shape[0]
        dt = yc.dtype
        dout = dout.to(dt).contiguous()
        # the reverse direction's output rows are l' = L-1-l: its dout is read backwards
        db_, sd = (_rows_from_end(dout, b, L, d), -d) if rev else (dout, d)
        dy = dw = db = None
        with torch.autocast("cuda", enabled=False):
            if ctx.needs_input_grad[0]:  # dy[b][e][l] = sum_o W[o][e] dout[b][l'][o], channel-major
                dy = torch.empty(b, E, L, device=dout.device, dtype=dt)
                DF.strided_gemm(w, (1, E, 0), db_, (1, sd, L * d), dy, (L, E * L), E, L, d, b)
                dy = dy.to(ydt)
            if ctx.needs_input_grad[1]:  # dW[o][e] = sum_{b,l} dout[b][l'][o] y[b][e][l]
                part, _ = _wgrad_tokens(db_, (1, sd, L * d), yc, (1, yc.stride(1), yc.stride(0)),
                                        d, E, L, b)
                dw = _finish_wgrad(part, ctx.weight, (d, E), wdt)
            if bdt is not None and ctx.needs_input_grad[2]:
                db = dout.float().sum((0, 1)).to(bdt)
        return dy, dw, db, (dout if rev else None)


class Mamba(nn.Module):
    """mamba_ssm.modules.mamba_simple.Mamba (1.x) as Caduceus builds it (BiMambaWrapper,
    modeling_caduceus.py:88-91): same constructor, parameter names/shapes and initialisation;
    forward = the reference's non-fused path (in_proj -> causal depthwise conv1d + SiLU -> x_proj
    -> dt_proj -> selective_scan_fn(delta_softplus, z gating, D) -> out_proj), with the conv and the
    scan on HIP kernels. mamba_ssm is not vendored in the reference: parity unpinned."""

    def __init__(self, d_model, d_state=16, d_conv=4, expand=2, dt_rank="auto", dt_min=0.001,
                 dt_max=0.1, dt_init="random", dt_scale=1.0, dt_init_floor=1e-4, conv_bias=True,
                 bias=False, use_fast_path=True, layer_idx=None, device=None, dtype=None):
        super().__init__()
        fk = {"device": device, "dtype": dtype}
        self.d_model, self.d_state, self.d_conv, self.expand = d_model, d_state, d_conv, expand
        self.d_inner = int(expand * d_model)
        self.dt_rank = math.ceil(d_model / 16) if dt_rank == "auto" else dt_rank
        self.use_fast_path = use_fast_path
        self.layer_idx = layer_idx
        self.in_proj = nn.Linear(d_model, self.d_inner * 2, bias=bias, **fk)
        self.conv1d = nn.Conv1d(self.d_inner, self.d_inner, bias=conv_bias, kernel_size=d_conv,
                                groups=self.d_inner, padding=d_conv - 1, **fk)
        self.activation = "silu"
        self.act = nn.SiLU()
        self.x_proj = nn.Linear(self.d_inner, self.dt_rank + d_state * 2, bias=False, **fk)
        self.dt_proj = nn.Linear(self.dt_rank, self.d_inner, bias=True, **fk)
        dt_init_std = self.dt_rank ** -0.5 * dt_scale
        if dt_init == "constant":
            nn.init.constant_(self.dt_proj.weight, dt_init_std)
        elif dt_init == "random":
            nn.init.uniform_(self.dt_proj.weight, -dt_init_std, dt_init_std)
        else:
            raise NotImplementedError(dt_init)
        dt = torch.exp(torch.rand(self.d_inner, **fk) * (math.log(dt_max) - math.log(dt_min))
                       + math.log(dt_min)).clamp(min=dt_init_floor)
        inv_dt = dt + torch.log(-torch.expm1(-dt))
        with torch.no_grad():
            self.dt_proj.bias.copy_(inv_dt)
        self.dt_proj.bias._no_reinit = True
        A = torch.arange(1, d_state + 1, dtype=torch.float32, device=device).repeat(self.d_inner, 1)
        self.A_log = nn.Parameter(torch.log(A))
        self.A_log._no_weight_decay = True
        self.D = nn.Parameter(torch.ones(self.d_inner, device=device))
        self.D._no_weight_decay = True
        # stays torch's Linear: on the persistent MFMA GEMM (hyena.HipLinear) the config-E step was
        # slower, 92.0 vs 88.8 ms (its input is a transposed view that needs a copy first;
        # profiles/r02/session4/cfge_*linear.txt)
        self.out_proj = nn.Linear(self.d_inner, d_model, bias=bias, **fk)

    def forward(self, hidden_states, inference_params=None, reverse=False, out_into=None,
                dh_sink=None):
        """reverse + out_into (bf16 autocast): run on hidden_states read backwards and add the
        output, flipped back, into out_into in place; dh_sink: see DhSink (BiMambaWrapper)."""
        if inference_params is not None:
            raise NotImplementedError("Mamba: inference_params (recurrent decoding)")
        if reverse != (out_into is not None):
            raise ValueError("Mamba: reverse goes with out_into (the flipped-back accumulation)")
        batch, seqlen, _ = hidden_states.shape
        # in_proj computed channel-major, as the reference does (W @ x^T -> [b, 2E, l])
        x, z = InProj.apply(hidden_states, self.in_proj.weight, reverse, dh_sink)
        if self.in_proj.bias is not None:
            bx, bz = self.in_proj.bias.chunk(2)
            x, z = x + bx.to(x.dtype)[:, None], z + bz.to(z.dtype)[:, None]
        A = NegExp.apply(self.A_log) if _NEGEXP else -torch.exp(self.A_log.float())
        x = CausalConv1d.apply(x.contiguous(), self.conv1d.weight, self.conv1d.bias, True)
        # x_proj and dt_proj channel-major on the strided MFMA GEMM (ChannelLinear): x_dbl
        # [b, R + 2N, L] = x_proj.weight . x, delta [b, E, L] = dt_proj.weight . x_dbl[:, :R]
        if self.x_proj.bias is not None:
            raise NotImplementedError("Mamba: x_proj with a bias (mamba_ssm builds it bias-free)")
        sink = GradSink()  # the scan's du summed into x_proj's dx in its GEMM epilogue
        x_dbl = ChannelLinear.apply(x, self.x_proj.weight, sink)
        R, Ns = self.dt_rank, self.d_state
        if _XDBL_SPLIT:
            xdt, Bm, Cm = XdblSplit.apply(x_dbl, R, Ns, sink)
        else:
            xdt, Bm, Cm = x_dbl[:, :R], x_dbl[:, R:R + Ns], x_dbl[:, R + Ns:]
        dt = ChannelLinear.apply(xdt, self.dt_proj.weight)
        y = SelectiveScan.apply(x, dt, A, Bm, Cm, self.D.float(), z.contiguous(),
                                self.dt_proj.bias.float(), True, False, sink)
        return OutProj.apply(y, self.out_proj.weight, self.out_proj.bias, out_into)


class FlipL(torch.autograd.Function):
    """x.flip(dims=(1,)) of a [B, L, C] CUDA tensor by a 16-B row copy (dna_flip_rows); the
    backward is the same flip. torch's flip kernel ran at ~2.9 TB/s on these shapes."""

    @staticmethod
    def forward(ctx, x):
        return _flip_rows(x)

    @staticmethod
    def backward(ctx, g):
        return _flip_rows(g) if _flip_rows_ok(g.contiguous()) else g.flip(dims=(1,))


def _flip_rows_ok(x):
    return (x.is_cuda and x.dim() >= 2 and x.numel() > 0 and x.is_contiguous()
            and (x[0, 0].numel() * x.element_size()) % 16 == 0 and x.data_ptr() % 16 == 0)


def _flip_rows(x):
    x = x.contiguous()
    out = torch.empty_like(x)
    B, L = x.shape[0], x.shape[1]
    N.call("dna_flip_rows", x.data_ptr(), B, L, x[0, 0].numel() * x.element_size(), out.data_ptr(),
           N.stream_ptr())
    return out


def flip_l(x):
    """x.flip(dims=(1,)) (FlipL on CUDA tensors whose rows are whole 16-B chunks)."""
    if _flip_rows_ok(x):
        return FlipL.apply(x)
    return x.flip(dims=(1,))


class BiMambaWrapper(nn.Module):
    """The reference's BiMambaWrapper (modeling_caduceus.py:68-121) over `Mamba` above."""

    def __init__(self, d_model: int, bidirectional: bool = True, bidirectional_strategy="add",
                 bidirectional_weight_tie: bool = True, **mamba_kwargs):
        super().__init__()
        if bidirectional and bidirectional_strategy is None:
            bidirectional_strategy = "add"
        if bidirectional and bidirectional_strategy not in ["add", "ew_multiply"]:
            raise NotImplementedError(f"`{bidirectional_strategy}` strategy for bi-directionality is not implemented!")
        self.bidirectional = bidirectional
        self.bidirectional_strategy = bidirectional_strategy
        self.mamba_fwd = Mamba(d_model=d_model, **mamba_kwargs)
        if bidirectional:
            self.mamba_rev = Mamba(d_model=d_model, **mamba_kwargs)
            if bidirectional_weight_tie:  # in/out projections shared by both directions
                self.mamba_rev.in_proj.weight = self.mamba_fwd.in_proj.weight
                self.mamba_rev.in_proj.bias = self.mamba_fwd.in_proj.bias
                self.mamba_rev.out_proj.weight = self.mamba_fwd.out_proj.weight
                self.mamba_rev.out_proj.bias = self.mamba_fwd.out_proj.bias
        else:
            self.mamba_rev = None

    def _fused_add(self, hidden_states):
        # both directions on the reversed-read / in-place-accumulate projections: no flipped
        # copies of the input, the output or their gradients, no add kernels (bf16 autocast)
        return (self.bidirectional and self.bidirectional_strategy == "add"
                and hidden_states.is_cuda and torch.is_autocast_enabled("cuda")
                and torch.get_autocast_dtype("cuda") == torch.bfloat16
                and os.environ.get("DNA_BIMAMBA_FUSED", "1") != "0")

    def forward(self, hidden_states, inference_params=None):
        if inference_params is None and self._fused_add(hidden_states):
            sink = DhSink()
            out = self.mamba_fwd(hidden_states, dh_sink=sink)
            return self.mamba_rev(hidden_states, reverse=True, out_into=out, dh_sink=sink)
        out = self.mamba_fwd(hidden_states, inference_params=inference_params)
        if self.bidirectional:
            out_rev = flip_l(self.mamba_rev(flip_l(hidden_states), inference_params=inference_params))
            if self.bidirectional_strategy == "add":
                out = out + out_rev
            elif self.bidirectional_strategy == "ew_multiply":
                out = out * out_rev
            else:
                raise NotImplementedError(self.bidirectional_strategy)
        return out
