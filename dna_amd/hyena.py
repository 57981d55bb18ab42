"""HyenaDNA long convolution on MI355X: `fftconv` with the reference's signature and semantics.

Mirrors `fftconv_ref(u, k, D, dropout_mask, gelu=True, k_rev=None, bidirectional=False)`
(reference src/models/sequence/hyena.py:60-92) in the form `HyenaFilter.forward` calls it
(:253-280: dropout_mask=None, gelu=False): u [..., D, L] (any leading dims, e.g. the operator's
[b, 1, D, 1, L]), k [D, L], D (bias) broadcastable per channel. Forward and backward run the HIP
kernels of dna_amd/csrc/fftconv.hip (four-step FFT of size 2L, fp32 internally); there is no CPU
or torch.fft fallback -- without the native library or a GPU tensor this raises.
"""
import torch

from . import _native as N
from .functional import _dt, _gpu, _p, _timed


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


def fftconv(u, k, D, dropout_mask=None, gelu=False, k_rev=None, bidirectional=False):
    """`fftconv_ref` on the GPU (hyena.py:60-92). Supported: dropout_mask=None, gelu=False,
    k_rev=None (the HyenaFilter call); output dtype = u's dtype, as in the reference."""
    if dropout_mask is not None or gelu or k_rev is not None:
        raise NotImplementedError("fftconv: dropout_mask / gelu / k_rev (unused by HyenaFilter)")
    return FFTConv.apply(u, k, D, bidirectional)
