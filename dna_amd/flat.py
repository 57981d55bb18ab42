"""One flat HBM buffer for all parameters, gradients and the bf16 compute copy.

All 117,074,176 DNABERT-2 parameters become views into one fp32 buffer (468 MB), their .grad
views into one fp32 gradient buffer, and a persistent bf16 copy (234 MB) feeds the GEMMs and is
refreshed by the fused AdamW kernel -- so the optimizer is one launch, gradient buckets for the
RCCL all-reduce are contiguous slices (zero-copy), and no per-step weight casts run.

Layout: parameters in REVERSE registration order (head and last layer first), each slice aligned
to 64 elements; backward produces gradients roughly front-to-back through this buffer, so the
all-reduce buckets (dna_amd/ddp.py) become ready in order. The tied embedding/decoder weight is
one parameter and therefore one slice (it sits at the end: its last contribution comes from the
embedding backward, the final op of the backward pass).
"""
import torch

ALIGN = 64  # elements (256 B fp32 / 128 B bf16): keeps every slice 16-B aligned for vector loads


class FlatParams:
    def __init__(self, module: torch.nn.Module, device=None, shadow_dtype=torch.bfloat16):
        params = list(module.parameters())[::-1]
        device = torch.device(device) if device is not None else params[0].device
        self.params = params
        self.slices = []
        off = 0
        for p in params:
            n = p.numel()
            self.slices.append((off, n, tuple(p.shape)))
            off += (n + ALIGN - 1) // ALIGN * ALIGN
        self.numel = off
        self.n_params = sum(p.numel() for p in params)
        self.flat = torch.zeros(off, dtype=torch.float32, device=device)
        self.grad = torch.zeros(off, dtype=torch.float32, device=device)
        self._index = {}
        with torch.no_grad():
            for p, (o, n, shape) in zip(params, self.slices):
                self.flat[o:o + n].copy_(p.detach().reshape(-1))
                p.data = self.flat[o:o + n].view(shape)
                p.grad = self.grad[o:o + n].view(shape)
                self._index[id(p)] = (o, n, shape)
        self.shadow = None
        # transposed bf16 copies of the projection weights (parameters flagged `_dna_transpose`
        # by the model): the data gradient dx = dy . W runs as a K-major GEMM on W^T
        self.transposed = [p for p in params if getattr(p, "_dna_transpose", False) and p.dim() == 2]
        self.shadow_t = None
        if shadow_dtype is not None:
            self.shadow = torch.empty(off, dtype=shadow_dtype, device=device)
            if self.transposed and self.shadow.is_cuda and shadow_dtype == torch.bfloat16:
                self.shadow_t = torch.empty(off, dtype=shadow_dtype, device=device)
            self.refresh_shadow()
        if hasattr(module, "_lp_provider"):
            module._lp_provider = self.lp if self.shadow is not None else None
        if hasattr(module, "_lpt_provider"):
            module._lpt_provider = self.lpt if self.shadow_t is not None else None

    def slice_of(self, p):
        return self._index[id(p)]

    def lp(self, p):
        o, n, shape = self._index[id(p)]
        return self.shadow[o:o + n].view(shape)

    def lpt(self, p):
        """Transposed bf16 copy [in, out] of a flagged 2-D weight [out, in]."""
        o, n, shape = self._index[id(p)]
        return self.shadow_t[o:o + n].view(shape[1], shape[0])

    @torch.no_grad()
    def refresh_shadow(self):
        """Re-derive the bf16 copy after any parameter change made outside FusedAdamW."""
        if self.shadow is not None:
            self.shadow.copy_(self.flat)
            self.refresh_transposed()

    def refresh_transposed(self):
        """W^T bf16 copies from the bf16 shadow (after every optimizer step: FusedAdamW calls it)."""
        if self.shadow_t is None:
            return
        from . import _native as N
        st = N.stream_ptr(self.shadow.device)
        for p in self.transposed:
            o, n, (r, c) = self._index[id(p)]
            N.call("dna_transpose_bf16", self.shadow[o:o + n].data_ptr(), r, c,
                   self.shadow_t[o:o + n].data_ptr(), st)

    def zero_grad(self):
        self.grad.zero_()

    def enable_direct_grad(self, on=True):
        """Let fused backward kernels accumulate weight gradients straight into the flat .grad
        views (dna_amd.functional.Linear) instead of returning them to AccumulateGrad. Only valid
        for loss.backward() into these .grad buffers (not torch.autograd.grad)."""
        for p in self.params:
            p._dna_direct = bool(on)
