"""HyenaDNA long convolution on MI355X: `fftconv` with the reference's signature and semantics,
and the Hyena operator modules around it (HyenaFilter, HyenaOperator).

Mirrors `fftconv_ref(u, k, D, dropout_mask, gelu=True, k_rev=None, bidirectional=False)`
(reference src/models/sequence/hyena.py:60-92) in the form `HyenaFilter.forward` calls it
(:253-280: dropout_mask=None, gelu=False): u [..., D, L] (any leading dims, e.g. the operator's
[b, 1, D, 1, L]), k [D, L], D (bias) broadcastable per channel. Forward and backward run the HIP
kernels of dna_amd/csrc/fftconv.hip (four-step FFT of size 2L, fp32 internally); there is no CPU
or torch.fft fallback -- without the native library or a GPU tensor this raises.
"""
import ctypes
import math
import os

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import _native as N
from . import functional as DF
from .functional import Linear as _LinearFn
from .functional import _dt, _gpu, _p, _timed

_TORCH_LINEAR = os.environ.get("DNA_HYENA_TORCH_LINEAR", "0") == "1"  # A/B switch: torch Linear


def hip_linear(x, weight, bias=None, gelu=False):
    """F.linear(x, weight, bias) with autocast nn.Linear's dtype flow on hand-written kernels:
    under CUDA bf16 autocast with K % 64 == 0 and N % 256 == 0 the persistent MFMA GEMM
    (`dna_linear_fwd`, dgrad on a transposed bf16 weight copy, fp32 split-K weight gradient);
    every other CUDA case -- fp32, skinny or ragged N such as a 16-token character vocabulary --
    the strided MFMA GEMM (`functional.strided_linear`). CPU tensors (module-level CPU tests)
    and DNA_HYENA_TORCH_LINEAR=1 (A/B) keep torch's linear. gelu=True (the Mlp's fc1 ahead of
    GeluLinear): on the persistent path the output also carries `_dna_gelu` = gelu_tanh of it
    from the same launch (dna_linear_gelu_fwd)."""
    K, Nout = weight.shape[1], weight.shape[0]
    if _TORCH_LINEAR or not x.is_cuda:
        return F.linear(x, weight, bias)
    if (K % 64 or Nout % 256 or not torch.is_autocast_enabled("cuda")
            or torch.get_autocast_dtype("cuda") != torch.bfloat16):
        return DF.strided_linear(x, weight, bias)
    w_lp = weight.to(torch.bfloat16)
    y = _LinearFn.apply(x.reshape(-1, K).to(torch.bfloat16), weight, w_lp, bias,
                        w_lp.t().contiguous(), None, gelu)
    out = y.view(*x.shape[:-1], Nout)
    act = getattr(y, "_dna_gelu", None)
    if act is not None:
        out._dna_gelu = act.view(out.shape)
    return out


class HipLinear(nn.Linear):
    """nn.Linear (same parameters / state_dict) running `hip_linear`: the projections of the
    Hyena operator (in_proj / out_proj, hyena.py:311-509), the HyenaDNA Block's Mlp (fc1 / fc2)
    and the LM heads. The reference runs them as autocast nn.Linear (bf16 GEMM of the bf16-cast
    input and weight, bf16 output, fp32 weight / bias gradients): same operands, same output
    dtype."""

    def forward(self, x):
        return hip_linear(x, self.weight, self.bias)


def _bytes_per_elem(t):
    return t.element_size()


class FFTConv(torch.autograd.Function):
    @staticmethod
    def forward(ctx, u, k, bias, bidirectional):
        _gpu(u, k)
        L = u.shape[-1]
        if u.dim() > 3:
            # HyenaOperator layout [b, heads, D, num_blocks, L]: the reference broadcasts k_f as
            # [D, 1, L+1] (hyena.py:80-82), i.e. the channel is dim -3
            if u.shape[-2] != 1:
                raise NotImplementedError("fftconv: num_blocks > 1")
            D, lead = u.shape[-3], u.shape[:-3]
        else:
            D, lead = u.shape[-2], u.shape[:-2]
        B = 1
        for s in lead:
            B *= s
        u = u.contiguous()
        kf = k.detach().to(torch.float32).contiguous()
        assert kf.shape == (D, L), f"filter {tuple(k.shape)} != ({D}, {L})"
        b32 = None if bias is None else bias.detach().to(torch.float32).reshape(-1).contiguous()
        if b32 is not None:
            assert b32.numel() == D, "bias must have one value per channel"
        lib = N.lib()
        nk = lib.dna_fftconv_kspec_elems(L)
        if nk == 0:
            raise N.NativeError(f"fftconv: L={L} unsupported (power of 2 in [64, 131072])")
        kspec = torch.empty(D, nk, device=u.device, dtype=torch.float32)
        wsz = lib.dna_fftconv_workspace(B, D, L)
        ws = torch.empty(wsz, device=u.device, dtype=torch.uint8)
        y = torch.empty_like(u)
        # keep the input spectrum for dk when the filter needs a gradient
        uspec = (torch.empty(((B + 1) // 2) * D, nk, device=u.device, dtype=torch.float32)
                 if ctx.needs_input_grad[1] else None)
        with _timed("fftconv_fwd", B * D * L * 2 * _bytes_per_elem(u), "byte"):
            N.call("dna_fftconv_filter", kf.data_ptr(), _p(b32), D, L, int(bool(bidirectional)),
                   kspec.data_ptr(), ws.data_ptr(), wsz, N.stream_ptr())
            N.call("dna_fftconv_fwd", u.data_ptr(), _dt(u), kspec.data_ptr(), B, D, L,
                   int(bool(bidirectional)), y.data_ptr(), _p(uspec), ws.data_ptr(), wsz,
                   N.stream_ptr())
        ctx.save_for_backward(u, kspec, uspec)
        ctx.cfg = (B, D, L, bool(bidirectional), bias is not None, k.dtype, None if bias is None else bias.shape)
        return y

    @staticmethod
    def backward(ctx, dy):
        u, kspec, uspec = ctx.saved_tensors
        B, D, L, bi, has_bias, kdtype, bshape = ctx.cfg
        dy = dy.contiguous().to(u.dtype)
        need_u, need_k, need_b = ctx.needs_input_grad[0], ctx.needs_input_grad[1], ctx.needs_input_grad[2]
        du = torch.empty_like(u) if need_u else None
        dk = torch.empty(D, L, device=u.device, dtype=torch.float32) if need_k else None
        db = torch.empty(D, device=u.device, dtype=torch.float32) if (need_b and has_bias) else None
        lib = N.lib()
        wsz = lib.dna_fftconv_workspace(B, D, L)
        ws = torch.empty(wsz, device=u.device, dtype=torch.uint8)
        with _timed("fftconv_bwd", B * D * L * 3 * _bytes_per_elem(u), "byte"):
            N.call("dna_fftconv_bwd", dy.data_ptr(), u.data_ptr(), _dt(u), kspec.data_ptr(),
                   _p(uspec), B, D, L, int(bi), _p(du), _p(dk), _p(db), ws.data_ptr(), wsz,
                   N.stream_ptr())
        return (du, None if dk is None else dk.to(kdtype),
                None if db is None else db.reshape(bshape), None)


def bidirectional_pad_before(L):
    """fftconv_ref pads L//2 zeros on each side of u (total L + 2*(L//2)) and transforms at
    n = 2L (hyena.py:68-72): u starts at padded_length//2 - L//2 of the size-2L window."""
    padded = L + 2 * (L // 2)
    return padded // 2 - L // 2


def _kernel_len(n):
    """Smallest length the FFT kernels take that is >= n (powers of two from 64)."""
    return max(64, 1 << (int(n) - 1).bit_length())


MAX_KERNEL_LEN = 131072


def fftconv(u, k, D, dropout_mask=None, gelu=False, k_rev=None, bidirectional=False):
    """`fftconv_ref` on the GPU (hyena.py:60-92). Supported: dropout_mask=None, gelu=False,
    k_rev=None (the HyenaFilter call); output dtype = u's dtype, as in the reference.

    Any sequence length L, with the reference's exact semantics:
      * L a power of two in [64, 131072]: the native causal / bidirectional kernels;
      * causal, other L: u and k zero-padded to the next kernel length (a linear convolution is
        unchanged by trailing zeros), output sliced to L;
      * bidirectional, other L: the reference's circular convolution of size 2L,
        y[t] = sum_j k[j] u~[(t - j) mod 2L], equals the linear convolution of k with
        roll(u~, L) read at offset L -- run as a causal convolution of kernel length >= 2L, with
        the D*u term added as the reference adds it (u * D.unsqueeze(-1)).
    Gradients flow through the pads / roll / slices (exact)."""
    if dropout_mask is not None or gelu or k_rev is not None:
        raise NotImplementedError("fftconv: dropout_mask / gelu / k_rev (unused by HyenaFilter)")
    L = u.shape[-1]
    if L == _kernel_len(L) and L <= MAX_KERNEL_LEN:
        return FFTConv.apply(u, k, D, bidirectional)
    if not bidirectional:
        Lp = _kernel_len(L)
        if Lp > MAX_KERNEL_LEN:
            raise NotImplementedError(f"fftconv: L={L} > {MAX_KERNEL_LEN}")
        y = FFTConv.apply(F.pad(u, (0, Lp - L)), F.pad(k, (0, Lp - L)), D, False)
        return y[..., :L]
    N = 2 * L
    pb = bidirectional_pad_before(L)
    ut = F.pad(u, (pb, N - L - pb))
    v = torch.cat([ut[..., L:], ut[..., :L]], dim=-1)          # roll(u~, L)
    Lp = _kernel_len(N)
    if Lp > MAX_KERNEL_LEN:
        raise NotImplementedError(f"fftconv: bidirectional L={L} needs kernel length {Lp} > {MAX_KERNEL_LEN}")
    y = FFTConv.apply(F.pad(v, (0, Lp - N)), F.pad(k, (0, Lp - L)), None, False)[..., L:N]
    if D is not None:
        y = y + u * D.unsqueeze(-1)
    return y.to(u.dtype)


# --------------------------------------------------------------------------- Hyena operator
# The modules around the long convolution, with the reference's constructor arguments, module
# tree and state_dict keys (src/models/sequence/hyena.py:100-509), so reference checkpoints load
# unchanged. The projections, the short depthwise conv and the tiny implicit-filter MLP are plain
# torch ops (the MLP runs on [L, emb_dim]); the long convolution is the HIP `fftconv` above.
class ShortConvSplit(torch.autograd.Function):
    """Depthwise causal short conv of the in_proj output + split + first gate, fused
    (dna_hyena_shortconv_fwd/bwd): u [B, L, C] token-major -> xs [B, order-1, d, L] (x_0 ..
    x_{order-2}) and vx = v * x_{order-1} [B, d, L], channel-major for the long conv."""

    @staticmethod
    def forward(ctx, u, weight, bias, order, d):
        _gpu(u, weight, bias)
        u = u.contiguous()
        B, L, C = u.shape
        K = weight.shape[-1]
        w = weight.detach().reshape(C, K).float().contiguous()
        bb = bias.detach().float().contiguous()
        xs = torch.empty(B, order - 1, d, L, device=u.device, dtype=u.dtype)
        vx = torch.empty(B, d, L, device=u.device, dtype=u.dtype)
        with _timed("hyena_shortconv_fwd", B * L * C * u.element_size() + order * B * d * L * u.element_size(), "byte"):
            N.call("dna_hyena_shortconv_fwd", u.data_ptr(), _dt(u), w.data_ptr(), bb.data_ptr(), B, L,
                   d, order, K, xs.data_ptr(), vx.data_ptr(), N.stream_ptr())
        ctx.save_for_backward(u, w, bb)
        ctx.cfg = (order, d, K, weight.shape, weight.dtype)
        return xs, vx

    @staticmethod
    def backward(ctx, dxs, dvx):
        u, w, bb = ctx.saved_tensors
        order, d, K, wshape, wdtype = ctx.cfg
        B, L, C = u.shape
        if dxs is None:
            dxs = torch.zeros(B, order - 1, d, L, device=u.device, dtype=u.dtype)
        if dvx is None:
            dvx = torch.zeros(B, d, L, device=u.device, dtype=u.dtype)
        dxs = dxs.contiguous().to(u.dtype)
        dvx = dvx.contiguous().to(u.dtype)
        du = torch.empty_like(u)
        nrow = N.lib().dna_hyena_shortconv_part_elems(B, L, d, order, K) // (C * (K + 1))
        part = torch.empty(nrow, C * (K + 1), device=u.device, dtype=torch.float32)
        with _timed("hyena_shortconv_bwd", 3 * B * L * C * u.element_size(), "byte"):
            N.call("dna_hyena_shortconv_bwd", u.data_ptr(), _dt(u), w.data_ptr(), bb.data_ptr(), B, L,
                   d, order, K, dxs.data_ptr(), dvx.data_ptr(), du.data_ptr(), part.data_ptr(),
                   N.stream_ptr())
            s = torch.empty(C * (K + 1), device=u.device, dtype=torch.float32)
            N.call("dna_colsum_f32", part.data_ptr(), nrow, C * (K + 1), s.data_ptr(), 0, N.stream_ptr())
        s = s.view(C, K + 1)
        return du, s[:, :K].reshape(wshape).to(wdtype), s[:, K].contiguous(), None, None


class GateOut(torch.autograd.Function):
    """y = (v_conv * x_0) rearranged to [B, L, d] for out_proj (dna_hyena_gate_out_fwd/bwd)."""

    @staticmethod
    def forward(ctx, yc, xs):
        _gpu(yc, xs)
        yc = yc.contiguous()
        B, d, L = yc.shape
        xs = xs.to(yc.dtype)
        y = torch.empty(B, L, d, device=yc.device, dtype=yc.dtype)
        bstride = xs.stride(0)
        assert xs.is_contiguous()
        with _timed("hyena_gate_fwd", 3 * B * d * L * yc.element_size(), "byte"):
            N.call("dna_hyena_gate_out_fwd", yc.data_ptr(), xs.data_ptr(), _dt(yc), B, L, d, bstride,
                   y.data_ptr(), N.stream_ptr())
        ctx.save_for_backward(yc, xs)
        return y

    @staticmethod
    def backward(ctx, dy):
        yc, xs = ctx.saved_tensors
        B, d, L = yc.shape
        dy = dy.contiguous().to(yc.dtype)
        dyc = torch.empty_like(yc)
        dxs = torch.empty_like(xs) if xs.shape[1] == 1 else torch.zeros_like(xs)
        with _timed("hyena_gate_bwd", 5 * B * d * L * yc.element_size(), "byte"):
            N.call("dna_hyena_gate_out_bwd", dy.data_ptr(), yc.data_ptr(), xs.data_ptr(), _dt(yc), B, L,
                   d, xs.stride(0), dyc.data_ptr(), dxs.data_ptr(), N.stream_ptr())
        return dyc, dxs


class Sin(nn.Module):
    """sin(freq * x), freq [1, dim] initialised to w (hyena.py:100-110)."""

    def __init__(self, dim, w=10, train_freq=True):
        super().__init__()
        self.freq = nn.Parameter(w * torch.ones(1, dim)) if train_freq else w * torch.ones(1, dim)

    def forward(self, x):
        return torch.sin(self.freq * x)


class _OptimModule(nn.Module):
    """register(): lr == 0 -> buffer, else parameter tagged with its optimizer overrides
    (reference src/utils/train.py:142-156)."""

    def register(self, name, tensor, lr=None, wd=0.0):
        if lr == 0.0:
            self.register_buffer(name, tensor)
        else:
            self.register_parameter(name, nn.Parameter(tensor))
            optim = {}
            if lr is not None:
                optim["lr"] = lr
            if wd is not None:
                optim["weight_decay"] = wd
            setattr(getattr(self, name), "_optim", optim)


class PositionalEmbedding(_OptimModule):
    """Complex-exponential time features of the implicit filter (hyena.py:113-137)."""

    def __init__(self, emb_dim: int, seq_len: int, lr_pos_emb: float = 1e-5, **kwargs):
        super().__init__()
        self.seq_len = seq_len
        t = torch.linspace(0, 1, seq_len)[None, :, None]
        bands = (emb_dim - 1) // 2
        t_rescaled = torch.linspace(0, seq_len - 1, seq_len)[None, :, None]
        w = 2 * math.pi * t_rescaled / seq_len
        f = torch.linspace(1e-4, bands - 1, bands)[None, None]
        z = torch.exp(-1j * f * w)
        self.register("z", torch.cat([t, z.real, z.imag], dim=-1), lr=lr_pos_emb)
        self.register("t", t, lr=0.0)

    def forward(self, L):
        return self.z[:, :L], self.t[:, :L]


class ExponentialModulation(_OptimModule):
    """h * (exp(-t |deltas|) + shift) (hyena.py:140-163)."""

    def __init__(self, d_model, fast_decay_pct=0.3, slow_decay_pct=1.5, target=1e-2,
                 modulation_lr=0.0, shift: float = 0.0, **kwargs):
        super().__init__()
        self.shift = shift
        max_decay = math.log(target) / fast_decay_pct
        min_decay = math.log(target) / slow_decay_pct
        self.register("deltas", torch.linspace(min_decay, max_decay, d_model)[None, None],
                      lr=modulation_lr)

    def forward(self, t, x):
        return x * (torch.exp(-t * self.deltas.abs()) + self.shift)


class ModulateT(torch.autograd.Function):
    """k [O, C/O, L] fp32 = transpose(h [L, C] * (exp(-t |deltas|) + shift)), the
    ExponentialModulation of the implicit filter fused with the filter layout the long
    convolution reads (dna_hyena_modulate_t_fwd / _bwd; reference hyena.py:140-163, :438-441).
    deltas is a constant here (registered with lr 0 in every reference config)."""

    @staticmethod
    def forward(ctx, h, tpos, deltas, shift, O):
        _gpu(h, tpos, deltas)
        L, C = h.shape
        h = h.contiguous()
        k = torch.empty(O, C // O, L, device=h.device, dtype=torch.float32)
        N.call("dna_hyena_modulate_t_fwd", h.data_ptr(), _dt(h), tpos.data_ptr(), deltas.data_ptr(),
               float(shift), L, C, O, k.data_ptr(), N.stream_ptr())
        ctx.save_for_backward(tpos, deltas)
        ctx.cfg = (L, C, O, float(shift), h.dtype)
        return k

    @staticmethod
    def backward(ctx, dk):
        tpos, deltas = ctx.saved_tensors
        L, C, O, shift, hdt = ctx.cfg
        dk = dk.contiguous().float()
        dh = torch.empty(L, C, device=dk.device, dtype=hdt)
        N.call("dna_hyena_modulate_t_bwd", dk.data_ptr(), tpos.data_ptr(), deltas.data_ptr(), shift,
               L, C, O, dh.data_ptr(), _dt(dh), N.stream_ptr())
        return dh, None, None, None, None


_FILTER_FUSED = os.environ.get("DNA_HYENA_FILTER_FUSED", "1") != "0"  # A/B switch


def _ptr_array(ts):
    arr = (ctypes.c_void_p * len(ts))(*[t.data_ptr() for t in ts])
    return arr, ctypes.addressof(arr)


class FilterMLP(torch.autograd.Function):
    """HyenaFilter.filter_t under bf16 autocast as two kernels (csrc/hyena_filter.hip): the
    positional MLP Linear(E, 64) -> Sin -> [Linear(64, 64) -> Sin] x 2 -> Linear(64, C), the
    ExponentialModulation and the transpose to the long convolution's k [O][C / O][L] in one
    forward launch; the backward recomputes the MLP per 64-position tile and leaves per-block
    weight-gradient partials for one dna_sum_slices. Same dtype flow as the module path under
    autocast (reference hyena.py:162-247 with torch's autocast casts): bf16 Linear operands and
    outputs, fp32 Sin, dW / db rounded to bf16 once after the fp32 sum, the freq gradient fp32."""

    @staticmethod
    def forward(ctx, z, tpos, deltas, shift, O, w1, b1, w4, freq, *inner):
        _gpu(z, w1, w4)
        L, E = z.shape
        C = w4.shape[0]
        wi, bi = list(inner[0::2]), list(inner[1::2])
        NI = len(wi)
        k = torch.empty(O, C // O, L, device=z.device, dtype=torch.float32)
        wa, wp = _ptr_array(wi)
        ba, bp = _ptr_array(bi)
        with _timed("hyena_filter_fwd", L * (E + C) * 4, "byte"):
            N.call("dna_hyena_filter_fwd", z.data_ptr(), w1.data_ptr(), b1.data_ptr(), wp, bp, NI,
                   w4.data_ptr(), freq.data_ptr(), tpos.data_ptr(), deltas.data_ptr(), float(shift), L,
                   E, C, O, k.data_ptr(), N.stream_ptr())
        ctx.save_for_backward(z, tpos, deltas, w1, b1, w4, freq, *inner)
        ctx.cfg = (float(shift), O, NI)
        return k

    @staticmethod
    def backward(ctx, dk):
        z, tpos, deltas, w1, b1, w4, freq, *inner = ctx.saved_tensors
        shift, O, NI = ctx.cfg
        wi, bi = list(inner[0::2]), list(inner[1::2])
        L, E = z.shape
        C = w4.shape[0]
        F_ = w1.shape[0]
        dk = dk.contiguous().float()
        lib = N.lib()
        total = int(lib.dna_hyena_filter_part_elems(L, E, NI, C))
        P = int(lib.dna_hyena_filter_part_stride(E, NI, C))
        part = torch.empty(total, device=dk.device, dtype=torch.float32)
        dz = torch.empty(L, E, device=dk.device, dtype=torch.float32) if ctx.needs_input_grad[0] else None
        wa, wp = _ptr_array(wi)
        ba, bp = _ptr_array(bi)
        with _timed("hyena_filter_bwd", L * (E + C) * 4, "byte"):
            N.call("dna_hyena_filter_bwd", z.data_ptr(), w1.data_ptr(), b1.data_ptr(), wp, bp, NI,
                   w4.data_ptr(), freq.data_ptr(), tpos.data_ptr(), deltas.data_ptr(), shift, L, E, C,
                   O, dk.data_ptr(), part.data_ptr(), _p(dz), N.stream_ptr())
            # slice sum; the weight / bias entries (all but the trailing freq) rounded to bf16, the
            # grad of autocast's bf16 copies
            g = torch.empty(P, device=dk.device, dtype=torch.float32)
            N.call("dna_hyena_filter_finish", part.data_ptr(), total // P, P, P - F_, g.data_ptr(),
                   N.stream_ptr())
        o = 0
        dw4 = g[o:o + C * F_].view(C, F_); o += C * F_
        dwi = [g[o + i * F_ * F_:o + (i + 1) * F_ * F_].view(F_, F_) for i in range(NI)]; o += NI * F_ * F_
        dbi = [g[o + i * F_:o + (i + 1) * F_] for i in range(NI)]; o += NI * F_
        dw1 = g[o:o + F_ * E].view(F_, E); o += F_ * E
        db1 = g[o:o + F_]; o += F_
        dfreq = g[o:o + F_].view_as(freq)
        dinner = []
        for a_, b_ in zip(dwi, dbi):
            dinner += [a_, b_]
        return (dz, None, None, None, None, dw1, db1, dw4, dfreq, *dinner)


def _fused_filter_ok(f, h0, L, O):
    """The implicit filter runs as FilterMLP: CUDA, bf16 autocast, the reference layout
    (Linear(E, 64), then two Linear(64, 64), Linear(64, C, no bias), one shared Sin), C in
    {64, 128, 256, 512}, L % 64 == 0, modulation with a constant deltas, not normalized."""
    if not (_FILTER_FUSED and h0.is_cuda and torch.is_autocast_enabled("cuda")
            and torch.get_autocast_dtype("cuda") == torch.bfloat16):
        return False
    mods = list(f.implicit_filter)
    if len(mods) != 7 or L % 64 or not f.modulate or f.normalized or f.modulation.deltas.requires_grad:
        return False
    lins, acts = mods[0::2], mods[1::2]
    if not all(isinstance(m, nn.Linear) for m in lins) or not all(a is acts[0] for a in acts):
        return False
    if not isinstance(acts[0], Sin) or not isinstance(acts[0].freq, torch.Tensor) or acts[0].freq.numel() != 64:
        return False
    E = lins[0].in_features
    C = lins[-1].out_features
    return (E <= 8 and lins[0].out_features == 64 and all(m.in_features == 64 and m.out_features == 64
                                                           for m in lins[1:-1])
            and lins[-1].in_features == 64 and lins[-1].bias is None and C in (64, 128, 256, 512)
            and C % O == 0 and all(m.bias is not None for m in lins[:-1])
            and all(p.dtype == torch.float32 for m in lins for p in m.parameters()))


def _split_k_linear(x, lin):
    """nn.Linear over the L positions of the implicit filter MLP ([1, L, K] -> [1, L, N], K 3-5
    and N 64-256) on the strided MFMA GEMM (`functional.strided_linear`). As one library GEMM
    its weight gradient is a 64 x 64 (or 256 x 64) output reduced over all L = 65,536 positions,
    which hipBLASLt ran as one or four workgroups (~210 us per call, 12 % of the config-D step);
    here the contraction is split over the CUs. CPU tensors keep the plain linear (parity tests of
    the module on the CPU)."""
    if not x.is_cuda or x.dim() != 3 or x.shape[0] != 1:
        return lin(x)
    return DF.strided_linear(x, lin.weight, lin.bias)


class HyenaFilter(_OptimModule):
    """Implicit long filter + the long convolution (hyena.py:166-280). `forward` runs the HIP
    FFT convolution (the reference's `fftconv_ref` path, fused_fft_conv=False)."""

    def __init__(self, d_model, emb_dim=3, order=16, fused_fft_conv=False, seq_len=1024, lr=1e-3,
                 lr_pos_emb=1e-5, dropout=0.0, w=1, wd=0, bias=True, num_inner_mlps=2,
                 linear_mixer=False, modulate: bool = True, normalized=False, bidirectional=False,
                 **kwargs):
        super().__init__()
        if emb_dim % 2 == 0 or emb_dim < 3:
            raise ValueError("emb_dim must be odd and greater or equal to 3 (time, sine and cosine)")
        self.d_model, self.emb_dim, self.seq_len, self.modulate = d_model, emb_dim, seq_len, modulate
        self.use_bias = bias
        self.fused_fft_conv = fused_fft_conv
        self.bias = nn.Parameter(torch.randn(d_model))
        self.dropout = nn.Dropout(dropout)
        self.bidirectional = bidirectional
        act = Sin(dim=order, w=w)  # one module (one freq) reused by every activation, as in the reference
        self.pos_emb = PositionalEmbedding(emb_dim, seq_len, lr_pos_emb)
        if linear_mixer is False:
            self.implicit_filter = nn.Sequential(nn.Linear(emb_dim, order), act)
            for _ in range(num_inner_mlps):
                self.implicit_filter.append(nn.Linear(order, order))
                self.implicit_filter.append(act)
            self.implicit_filter.append(nn.Linear(order, d_model, bias=False))
        else:
            self.implicit_filter = nn.Sequential(nn.Linear(emb_dim, d_model, bias=False))
        self.modulation = ExponentialModulation(d_model, **kwargs)
        self.normalized = normalized
        for c in self.implicit_filter.children():
            for name, _ in c.state_dict().items():
                setattr(getattr(c, name), "_optim", {"weight_decay": wd, "lr": lr})

    def filter(self, L, *args, **kwargs):
        z, t = self.pos_emb(L)
        h = z
        for layer in self.implicit_filter:
            h = _split_k_linear(h, layer) if isinstance(layer, nn.Linear) else layer(h)
        if self.modulate:
            h = self.modulation(t, h)
        if self.normalized:
            h = h / torch.norm(h, dim=-1, p=1, keepdim=True)
        return h

    def filter_t(self, L, O):
        """filter(L)[0] as the long convolution reads it: k [O, d_model / O, L] with
        k[o][v][l] = filter(L)[0][l][v * O + o]. On the GPU the modulation and the transpose are
        one kernel (ModulateT); otherwise the reshape / permute of the reference."""
        z, t = self.pos_emb(L)
        if z.dim() == 3 and z.shape[0] == 1 and _fused_filter_ok(self, z, L, O):
            lins = list(self.implicit_filter)[0::2]
            act = self.implicit_filter[1]
            inner = []
            for m in lins[1:-1]:
                inner += [m.weight, m.bias]
            return FilterMLP.apply(z[0], t.reshape(-1).float().contiguous(),
                                   self.modulation.deltas.reshape(-1).float().contiguous(),
                                   self.modulation.shift, O, lins[0].weight, lins[0].bias,
                                   lins[-1].weight, act.freq.reshape(-1), *inner)
        h = z
        for layer in self.implicit_filter:
            h = _split_k_linear(h, layer) if isinstance(layer, nn.Linear) else layer(h)
        deltas = self.modulation.deltas
        if (self.modulate and not self.normalized and h.is_cuda and h.dim() == 3 and h.shape[0] == 1
                and not deltas.requires_grad and h.dtype in (torch.float32, torch.bfloat16)):
            tpos = t.reshape(-1).float().contiguous()
            return ModulateT.apply(h[0], tpos, deltas.reshape(-1).float().contiguous(),
                                   self.modulation.shift, O)
        if self.modulate:
            h = self.modulation(t, h)
        if self.normalized:
            h = h / torch.norm(h, dim=-1, p=1, keepdim=True)
        return h[0].reshape(L, h.shape[-1] // O, O).permute(2, 1, 0)

    def forward(self, x, L, k=None, bias=None, *args, **kwargs):
        if k is None:
            k = self.filter(L)
        k = k[0] if type(k) is tuple else k
        if bias is None:
            bias = self.bias
        bias = bias if self.use_bias else 0 * bias
        return fftconv(x, k, bias, bidirectional=self.bidirectional).to(dtype=x.dtype)


class HyenaOperator(nn.Module):
    """Hyena operator (hyena.py:311-509): in_proj -> short depthwise conv -> order-1 gated long
    convolutions -> out_proj. Supported as in every reference HyenaDNA config: num_heads = 1,
    num_blocks = 1, inner_factor = 1, outer_mixing = post_order_ffn = False, activation "id";
    other settings raise."""

    def __init__(self, d_model, l_max, order=2, filter_order=64, num_heads=1, inner_factor=1,
                 num_blocks=1, fused_bias_fc=False, outer_mixing=False, dropout=0.0,
                 filter_dropout=0.0, filter_cls="hyena-filter", post_order_ffn=False,
                 jit_filter=False, short_filter_order=3, activation="id", return_state=False,
                 bidirectional=False, layer_idx=None, device=None, dtype=None, **filter_args):
        super().__init__()
        if (num_heads, inner_factor, num_blocks) != (1, 1, 1) or outer_mixing or post_order_ffn:
            raise NotImplementedError("HyenaOperator: num_heads/inner_factor/num_blocks = 1, no "
                                      "outer_mixing / post_order_ffn (all reference configs)")
        if activation not in (None, "id", "identity", "linear"):
            raise NotImplementedError(f"HyenaOperator: activation {activation!r}")
        if fused_bias_fc:
            raise NotImplementedError("fused_bias_fc (flash_attn FusedDense)")
        if filter_cls not in ("hyena-filter", None):
            raise NotImplementedError(f"filter_cls {filter_cls!r}")
        if order < 2:
            raise ValueError(f"Order must be at least 2, (got {order})")
        self.d_model, self.order, self.l_max = d_model, order, l_max
        self.num_heads, self.inner_factor, self.num_blocks = num_heads, inner_factor, num_blocks
        self.head_dim = d_model // num_heads
        self.block_dim = l_max // num_blocks
        self.filter_order, self.short_filter_order = filter_order, short_filter_order
        self.return_state, self.bidirectional = return_state, bidirectional
        self.activation = nn.Identity()
        self.dropout = nn.Dropout(dropout)
        self.out_proj = HipLinear(d_model * inner_factor, d_model)
        self.in_proj = HipLinear(d_model, (order + 1) * d_model)
        total_width = d_model * inner_factor * (order + 1)
        self.short_filter = nn.Conv1d(total_width, total_width, kernel_size=short_filter_order,
                                      groups=total_width, padding=short_filter_order - 1)
        self.filter_fn = HyenaFilter(self.head_dim * inner_factor * (order - 1), order=filter_order,
                                     seq_len=l_max, channels=1, dropout=filter_dropout,
                                     bidirectional=bidirectional, **filter_args)

    def forward(self, u, *args, **kwargs):
        l = u.size(-2)
        l_filter = min(l, self.l_max)
        K = self.short_filter_order
        if self.d_model % 64 == 0 and 2 <= K <= 4 and self.order <= 4 and l == l_filter:
            return self._forward_fused(u, l_filter)
        # other widths: torch ops around the HIP long convolution
        u = self.in_proj(u).transpose(1, 2)                                   # b d l
        uc = self.short_filter(u)[..., :l_filter]
        b, C = uc.shape[0], uc.shape[1]
        uc = uc.reshape(b, 1, C, 1, l_filter)                                 # b ho v z l
        *x, v = uc.split(self.d_model, dim=2)
        k = self.filter_fn.filter(l_filter)
        k = k[0].reshape(l_filter, self.head_dim, self.order - 1).permute(2, 1, 0)   # o v l
        bias = self.filter_fn.bias.reshape(self.head_dim, self.order - 1).t()          # o v
        for o, x_i in enumerate(reversed(x[1:])):
            v = self.dropout(v * x_i)
            v = self.filter_fn(v, l_filter, k=k[o], bias=bias[o, None, :, None])
        y = self.activation((v * x[0]).reshape(b, self.d_model, l_filter).transpose(1, 2))
        y = self.out_proj(y)
        if self.return_state:
            return y, None
        return y

    def _forward_fused(self, x, L):
        """d_model % 64 == 0: in_proj -> fused short conv / split / gate (HIP) -> long convs
        (HIP) -> fused gate + transpose (HIP) -> out_proj. Same math as forward's torch path."""
        d, order = self.d_model, self.order
        u = self.in_proj(x)                                                   # [B, L, C] token-major
        xs, v = ShortConvSplit.apply(u, self.short_filter.weight, self.short_filter.bias, order, d)
        k = self.filter_fn.filter_t(L, order - 1)                              # o v l
        # order 2: the one filter as a view (no select node, whose backward is a zero fill + copy)
        ks = [k.view(k.shape[1], L)] if order == 2 else [k[o] for o in range(order - 1)]
        bias = self.filter_fn.bias.reshape(self.head_dim, order - 1).t()       # o v
        for o in range(order - 1):
            if o > 0:  # reversed(x[1:]): x_{order-1} was gated in the fused kernel
                v = v * xs[:, order - 1 - o]
            v = self.dropout(v)
            v = self.filter_fn(v, L, k=ks[o], bias=bias[o])
        y = self.activation(GateOut.apply(v, xs))
        y = self.out_proj(y)
        if self.return_state:
            return y, None
        return y

    @property
    def d_output(self):
        return self.d_model
