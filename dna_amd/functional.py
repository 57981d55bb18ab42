"""Autograd Functions over the dna_amd C ABI (HIP kernels on the current torch stream).

Each Function is one fused HIP op with a hand-written backward; the forward, data-gradient and
weight-gradient GEMMs run the MFMA kernels of csrc/gemm.hip (hipBLASLt through torch only for
shapes those kernels do not take, or as the DNA_GEMM_IMPL / DNA_WGRAD_IMPL=torch A/B arm).
No CPU fallback: every op raises if the native library is missing or a tensor is not on a GPU.
"""
import math
import os

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import _native as N

_DT = {torch.float32: N.F32, torch.bfloat16: N.BF16}


def _dt(t):
    try:
        return _DT[t.dtype]
    except KeyError:
        raise TypeError(f"dna_amd: unsupported dtype {t.dtype} (fp32 / bf16 only)")


def _gpu(*ts):
    for t in ts:
        if t is not None and not t.is_cuda:
            raise RuntimeError("dna_amd ops run on the GPU only (no CPU fallback); "
                               f"got a tensor on {t.device}")


def _p(t):
    return None if t is None else t.data_ptr()


class LibraryFallbackError(RuntimeError):
    """A projection left the hand-written kernels for a torch/hipBLASLt GEMM under
    DNA_STRICT_NATIVE=1 (bench.py sets it: the timed step must stay native)."""


_FALLBACK_SEEN = set()


def library_fallback(what, *shapes):
    """Called wherever a projection is about to run on torch.mm / addmm / bmm instead of the
    hand-written MFMA kernels (shapes the kernels do not take, or the DNA_GEMM_IMPL /
    DNA_WGRAD_IMPL=torch A/B arms). DNA_STRICT_NATIVE=1 turns it into an error; otherwise each
    (site, shapes) pair is counted once in `_FALLBACK_SEEN` (tests and bench read it)."""
    key = (what,) + tuple(tuple(s) for s in shapes)
    if os.environ.get("DNA_STRICT_NATIVE", "0") == "1":
        raise LibraryFallbackError(f"dna_amd: {what} {shapes} would run on a library GEMM "
                                   "(DNA_STRICT_NATIVE=1)")
    _FALLBACK_SEEN.add(key)


class OpTimer:
    """Optional HIP-event timing of ops on the stream they launch on (bench.py roofline).
    Disabled (None) by default: zero overhead on the product path."""
    active = None

    def __init__(self):
        self.pending = []  # (name, units, start_event, end_event)

    def __enter__(self):
        OpTimer.active = self
        return self

    def __exit__(self, *exc):
        OpTimer.active = None

    def summary(self):
        """{name: (launches, mean_ms, units_per_launch, kind)} after a device synchronize;
        kind "flop" (MFMA-bound: algorithmic FLOPs) or "byte" (HBM-bound: algorithmic bytes)."""
        acc = {}
        for name, units, kind, a, b in self.pending:
            n, t, u, _ = acc.get(name, (0, 0.0, 0.0, kind))
            acc[name] = (n + 1, t + a.elapsed_time(b), u + units, kind)
        return {k: (n, t / n, u / n, kind) for k, (n, t, u, kind) in acc.items()}


class _timed:
    __slots__ = ("name", "units", "kind", "t", "a")

    def __init__(self, name, units, kind="flop"):
        self.name, self.units, self.kind, self.t = name, units, kind, OpTimer.active

    def __enter__(self):
        if self.t is not None:
            self.a = torch.cuda.Event(enable_timing=True)
            self.a.record()

    def __exit__(self, *exc):
        if self.t is not None:
            b = torch.cuda.Event(enable_timing=True)
            b.record()
            self.t.pending.append((self.name, self.units, self.kind, self.a, b))


class DropoutRNG:
    """Counter-based dropout stream: every dropout site draws (seed, offset) and advances the
    offset by the number of Philox4x32 groups it consumes, so backward regenerates the mask.
    MLMTrainer derives the seed from train.seed and the rank; checkpoints keep (seed, offset)."""

    def __init__(self, seed=2222):
        self.seed = int(seed) & 0xFFFFFFFFFFFFFFFF
        self.offset = 0

    def take(self, n_elements):
        off = self.offset
        self.offset += (int(n_elements) + 3) // 4 + 1
        return self.seed, off


# ----------------------------------------------------------------------------------- embeddings
class EmbeddingLN(torch.autograd.Function):
    """dropout(LN(E[ids] + type_row)) -> (y fp32, y_bf16|None)   (bert_layers.py:62-107)."""

    @staticmethod
    def forward(ctx, ids, E, tt, gamma, beta, eps, p, seed, off, want_f32, want_bf16):
        _gpu(ids, E, tt, gamma, beta)
        ctx.set_materialize_grads(False)
        T, (V, d) = ids.numel(), E.shape
        y = torch.empty(T, d, device=E.device, dtype=torch.float32) if want_f32 else None
        yb = torch.empty(T, d, device=E.device, dtype=torch.bfloat16) if want_bf16 else None
        mean = torch.empty(T, device=E.device, dtype=torch.float32)
        rstd = torch.empty_like(mean)
        ids = ids.contiguous()
        N.call("dna_embed_ln_fwd", ids.data_ptr(), E.data_ptr(), tt[0].data_ptr(),
               gamma.data_ptr(), beta.data_ptr(), T, d, V, eps, p, seed, off, _p(y), _p(yb),
               mean.data_ptr(), rstd.data_ptr(), N.stream_ptr())
        ctx.save_for_backward(ids, E, tt, gamma, mean, rstd)
        ctx.cfg = (eps, p, seed, off)
        return y, yb

    @staticmethod
    def backward(ctx, dy, dyb):
        ids, E, tt, gamma, mean, rstd = ctx.saved_tensors
        _, p, seed, off = ctx.cfg
        T, (V, d) = ids.numel(), E.shape
        dtt = torch.zeros_like(tt)
        dg = torch.empty_like(gamma)
        db = torch.empty_like(gamma)
        nws = N.lib().dna_ln_bwd_workspace(T, d)
        ws = torch.empty(max(nws, 16), device=E.device, dtype=torch.uint8)
        dy = None if dy is None else dy.contiguous()
        dyb = None if dyb is None else dyb.contiguous()
        # per-token row gradients, then an id-sorted segmented sum into the table (frequent
        # tokens would otherwise serialise thousands of atomic row adds on one row)
        drows = torch.empty(T, d, device=E.device, dtype=torch.float32)
        N.call("dna_embed_ln_bwd_rows", _p(dy), _p(dyb), ids.data_ptr(), E.data_ptr(),
               tt[0].data_ptr(), gamma.data_ptr(), mean.data_ptr(), rstd.data_ptr(), T, d, V,
               p, seed, off, drows.data_ptr(), dtt[0].data_ptr(), dg.data_ptr(), db.data_ptr(),
               ws.data_ptr(), nws, N.stream_ptr())
        sorted_ids, perm = torch.sort(ids, stable=True)  # fixed summation order run to run
        dE = torch.zeros_like(E)
        nsw = N.lib().dna_embed_grad_segsum_workspace(T, d)
        sw = torch.empty(max(nsw // 4, 4), device=E.device, dtype=torch.float32)
        N.call("dna_embed_grad_segsum", drows.data_ptr(), sorted_ids.data_ptr(), perm.data_ptr(),
               T, d, V, 0, dE.data_ptr(), sw.data_ptr(), nsw, N.stream_ptr())
        # the tied decoder's weight gradient may still be adding into E.grad on the wgrad side
        # stream; AccumulateGrad adds dE into the same buffer on this stream next
        join_side_stream()
        return None, dE, dtt, dg, db, None, None, None, None, None, None


class EmbeddingFn(torch.autograd.Function):
    """E[ids] with the table gradient of dna_embed_grad_segsum (ids sorted once, rows summed per
    run of equal ids in a fixed order: deterministic, no atomics) instead of torch's
    embedding_dense_backward -- with a 16-symbol character vocabulary every id owns thousands of
    rows, which that path serialises (0.65 ms per HyenaDNA step at L = 65,536)."""

    @staticmethod
    def forward(ctx, ids, E, padding_idx):
        _gpu(ids, E)
        ctx.save_for_backward(ids)
        ctx.cfg = (E.shape, padding_idx)
        return F.embedding(ids, E, padding_idx)

    @staticmethod
    def backward(ctx, dy):
        (ids,) = ctx.saved_tensors
        (V, d), pad = ctx.cfg
        flat = ids.reshape(-1).contiguous()
        T = flat.numel()
        drows = dy.reshape(T, d).float().contiguous()
        sorted_ids, perm = torch.sort(flat, stable=True)
        dE = torch.zeros(V, d, device=dy.device, dtype=torch.float32)
        nsw = N.lib().dna_embed_grad_segsum_workspace(T, d)
        sw = torch.empty(max(nsw // 4, 4), device=dy.device, dtype=torch.float32)
        N.call("dna_embed_grad_segsum", drows.data_ptr(), sorted_ids.data_ptr(), perm.data_ptr(),
               T, d, V, -1 if pad is None else pad, dE.data_ptr(), sw.data_ptr(), nsw,
               N.stream_ptr())
        join_side_stream()  # a tied head's weight gradient may be on the wgrad side stream
        return None, dE, None


def embedding(ids, weight, padding_idx=None):
    """F.embedding(ids, weight, padding_idx) with EmbeddingFn's backward for fp32 CUDA tables of
    width 64k <= 1024 (torch's otherwise)."""
    V, d = weight.shape
    if (ids.is_cuda and weight.dtype == torch.float32 and d % 64 == 0 and d <= 1024
            and ids.dtype in (torch.int64, torch.int32) and torch.is_grad_enabled()
            and weight.requires_grad):
        if padding_idx is not None and padding_idx < 0:
            padding_idx += V
        return EmbeddingFn.apply(ids.long(), weight, padding_idx)
    return F.embedding(ids, weight, padding_idx)


class HipEmbedding(nn.Embedding):
    """nn.Embedding (same parameter / state_dict) whose table gradient is the deterministic
    segmented sum (functional.embedding); max_norm / scale_grad_by_freq / sparse keep torch's."""

    def forward(self, ids):
        if self.max_norm is not None or self.scale_grad_by_freq or self.sparse:
            return super().forward(ids)
        return embedding(ids, self.weight, self.padding_idx)


def strided_gemm(A, sa, B, sb, C, sc, M, Nc, K, batch, splits=1, out_f32=None, bias_n=None,
                 accumulate=False):
    """C[z][m][n] = sum_k A(m, k) B(k, n) (+ bias_n[n], fp32) on dna_gemm_bf16_strided /
    dna_gemm_f32_strided (z = batch * splits + split). sa = (sam, sak, saz), sb = (sbk, sbn, sbz),
    sc = (ldc, scz); strides in elements. accumulate (bf16 operands, splits == 1): C += A B in the
    epilogue."""
    bn = None if bias_n is None else bias_n.data_ptr()
    if A.dtype == torch.bfloat16:
        assert B.dtype == torch.bfloat16
        f32 = C.dtype == torch.float32 if out_f32 is None else out_f32
        N.call("dna_gemm_bf16_strided", A.data_ptr(), *sa, B.data_ptr(), *sb, C.data_ptr(), *sc,
               int(f32) | (2 if accumulate else 0), None, bn, M, Nc, K, batch, splits,
               N.stream_ptr())
    else:
        if accumulate:
            raise NotImplementedError("strided_gemm: accumulate needs bf16 operands")
        assert A.dtype == B.dtype == C.dtype == torch.float32
        N.call("dna_gemm_f32_strided", A.data_ptr(), *sa, B.data_ptr(), *sb, C.data_ptr(), *sc,
               bn, M, Nc, K, batch, splits, N.stream_ptr())


class StridedLinear(torch.autograd.Function):
    """y[L, N] = x[L, K] . w[N, K]^T + b on the strided MFMA GEMM (dna_gemm_bf16_strided /
    dna_gemm_f32_strided) for skinny projections over many tokens (the HyenaDNA implicit-filter
    MLP, the char-vocabulary LM heads): the weight gradient's L-long contraction runs as fp32
    split-K slices summed once by dna_sum_slices_accum (rounded once, as one GEMM with fp32
    accumulation would), the bias gradient as an fp32 column sum. x / w / b in one dtype."""

    @staticmethod
    def forward(ctx, x, w, b):
        _gpu(x, w, b)
        L, K = x.shape
        Nn = w.shape[0]
        x = x.contiguous()
        w = w.contiguous()
        y = torch.empty(L, Nn, device=x.device, dtype=x.dtype)
        bf = None if b is None else b.float().contiguous()
        with _timed("strided_linear", (L * (K + Nn)) * x.element_size(), "byte"):
            strided_gemm(x, (K, 1, 0), w, (1, K, 0), y, (Nn, 0), L, Nn, K, 1, bias_n=bf)
        ctx.save_for_backward(x, w)
        ctx.has_b = b is not None
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        L, K = x.shape
        Nn = w.shape[0]
        dy = dy.contiguous().to(x.dtype)
        dx = None
        if ctx.needs_input_grad[0]:  # dx[L, K] = dy[L, N] . w[N, K]
            dx = torch.empty(L, K, device=x.device, dtype=x.dtype)
            strided_gemm(dy, (Nn, 1, 0), w, (K, 1, 0), dx, (K, 0), L, K, Nn, 1)
        s = int(N.lib().dna_gemm_strided_splits(Nn, K, L, 1))
        part = torch.empty(s, Nn, K, device=x.device, dtype=torch.float32)
        if x.dtype == torch.bfloat16:  # dW[N, K] = sum_l dy[l, n] x[l, k]
            strided_gemm(dy, (1, Nn, 0), x, (K, 1, 0), part, (K, Nn * K), Nn, K, L, 1, s,
                            out_f32=True)
        else:
            strided_gemm(dy, (1, Nn, 0), x, (K, 1, 0), part, (K, Nn * K), Nn, K, L, 1, s)
        dw = torch.empty(Nn, K, device=x.device, dtype=torch.float32)
        N.call("dna_sum_slices", part.data_ptr(), s, Nn * K, dw.data_ptr(), N.stream_ptr())
        db = dy.float().sum(0).to(dy.dtype) if ctx.has_b else None
        return dx, dw.to(w.dtype), db


def strided_linear(x, weight, bias=None):
    """F.linear(x, weight, bias) with nn.Linear's dtype flow (under autocast x, W and b in the
    autocast dtype, output in it, bias added inside the product) on StridedLinear; x [..., K]."""
    w, b = weight, bias
    if torch.is_autocast_enabled(x.device.type):
        dt = torch.get_autocast_dtype(x.device.type)
        x, w, b = x.to(dt), w.to(dt), (b.to(dt) if b is not None else None)
    else:
        b = b.to(x.dtype) if b is not None else None
        w = w.to(x.dtype)
    if x.dtype not in (torch.bfloat16, torch.float32):
        raise NotImplementedError(f"strided_linear in {x.dtype}")
    lead = x.shape[:-1]
    with torch.autocast(x.device.type, enabled=False):
        y = StridedLinear.apply(x.reshape(-1, x.shape[-1]), w, b)
    return y.reshape(*lead, w.shape[0])


# ----------------------------------------------------------------------------------- fused LN
_PARAM_DIRECT = os.environ.get("DNA_PARAM_GRAD_DIRECT", "1") != "0"  # 0: AccumulateGrad (A/B)


def _param_grads_direct(params):
    """Every parameter of the tuple (None entries skipped) is FlatParams-owned with direct
    gradients on (dna_amd.flat.enable_direct_grad) and holds its fp32 .grad view: the kernel may
    then add its gradient there itself. Only for loss.backward() into those buffers."""
    ps = [q for q in params if q is not None]
    return _PARAM_DIRECT and bool(ps) and all(getattr(q, "_dna_direct", False) and q.grad is not None
                            and q.grad.dtype == torch.float32 and q.grad.is_contiguous()
                            for q in ps)


class FusedLayerNorm(torch.autograd.Function):
    """LN(dropout(act(x + bias)) + residual) -> (y fp32|None, y_bf16|None).

    BertSelfOutput (bert_layers.py:209-214), GeGLU-MLP tail (:298-300), head transform
    (:524-528, act=gelu, eps=1e-12)."""

    @staticmethod
    def forward(ctx, x, bias, residual, gamma, beta, eps, act, p, seed, off, want_f32, want_bf16):
        _gpu(x, bias, residual, gamma, beta)
        ctx.set_materialize_grads(False)
        x = x.contiguous()
        n, d = x.shape
        y = torch.empty(n, d, device=x.device, dtype=torch.float32) if want_f32 else None
        yb = torch.empty(n, d, device=x.device, dtype=torch.bfloat16) if want_bf16 else None
        mean = torch.empty(n, device=x.device, dtype=torch.float32)
        rstd = torch.empty_like(mean)
        residual = None if residual is None else residual.contiguous()
        es = x.element_size()
        nbytes = n * (d * (es + (4 if residual is not None else 0) + (4 if want_f32 else 0)
                           + (2 if want_bf16 else 0)) + 8)
        with _timed("ln_fwd", nbytes, "byte"):
            N.call("dna_ln_fwd", x.data_ptr(), _dt(x), _p(bias), act, p, seed, off, _p(residual),
                   gamma.data_ptr(), beta.data_ptr(), n, d, eps, _p(y), _p(yb), mean.data_ptr(),
                   rstd.data_ptr(), N.stream_ptr())
        # backward from the fp32 output (x_hat = (y - beta) / gamma, dna_ln_bwd_from_y): one fp32
        # row read instead of x + the residual, and neither is kept alive for the backward
        ctx.from_y = y is not None and act == N.ACT_NONE and _LN_BWD_FROM_Y
        if ctx.from_y:
            ctx.save_for_backward(y, bias, gamma, beta, rstd)
            ctx.shape = (n, d, x.dtype, residual is not None)
            # the parameters themselves (their .grad / FlatParams flags), for _param_grads_direct
            ctx.params = (bias, gamma, beta)
        else:
            ctx.save_for_backward(x, bias, residual, gamma, mean, rstd)
        ctx.cfg = (act, p, seed, off)
        return y, yb

    @staticmethod
    def backward(ctx, dy, dyb):
        if ctx.from_y:
            return FusedLayerNorm._backward_from_y(ctx, dy, dyb)
        x, bias, residual, gamma, mean, rstd = ctx.saved_tensors
        act, p, seed, off = ctx.cfg
        n, d = x.shape
        dx = torch.empty_like(x)
        dres = torch.empty(n, d, device=x.device, dtype=torch.float32) if residual is not None else None
        dg = torch.empty_like(gamma)
        db = torch.empty_like(gamma)
        dbias = torch.empty_like(bias) if bias is not None else None
        nws = N.lib().dna_ln_bwd_workspace(n, d)
        ws = torch.empty(max(nws, 16), device=x.device, dtype=torch.uint8)
        dy = None if dy is None else dy.contiguous()
        dyb = None if dyb is None else dyb.contiguous()
        es = x.element_size()
        # reads dy / dy_bf16, x, residual; writes dx and (with a residual) d(residual) fp32
        nbytes = n * (d * ((4 if dy is not None else 0) + (2 if dyb is not None else 0) + 2 * es
                           + (8 if residual is not None else 0)) + 8)
        with _timed("ln_bwd", nbytes, "byte"):
            N.call("dna_ln_bwd", _p(dy), _p(dyb), x.data_ptr(), _dt(x), _p(bias), act, p, seed,
                   off, _p(residual), gamma.data_ptr(), mean.data_ptr(), rstd.data_ptr(), n, d,
                   _p(dres), dx.data_ptr(), dg.data_ptr(), db.data_ptr(), _p(dbias), ws.data_ptr(),
                   nws, N.stream_ptr())
        return dx, dbias, dres, dg, db, None, None, None, None, None, None, None

    @staticmethod
    def _backward_from_y(ctx, dy, dyb):
        y, bias, gamma, beta, rstd = ctx.saved_tensors
        act, p, seed, off = ctx.cfg
        n, d, xdt, has_res = ctx.shape
        dx = torch.empty(n, d, device=y.device, dtype=xdt)
        dres = torch.empty(n, d, device=y.device, dtype=torch.float32) if has_res else None
        direct = _param_grads_direct(ctx.params)
        if direct:
            # dgamma / dbeta / dbias added straight into the flat fp32 gradient (dna_amd.flat)
            # by the partial-sum pass, instead of three AccumulateGrad adds
            pb, pg, pbe = ctx.params
            dg, db, dbias = pg.grad, pbe.grad, (pb.grad if pb is not None else None)
        else:
            dg = torch.empty_like(gamma)
            db = torch.empty_like(gamma)
            dbias = torch.empty_like(bias) if bias is not None else None
        nws = N.lib().dna_ln_bwd_workspace(n, d)
        ws = torch.empty(max(nws, 16), device=y.device, dtype=torch.uint8)
        dy = None if dy is None else dy.contiguous()
        dyb = None if dyb is None else dyb.contiguous()
        es = dx.element_size()
        # reads dy / dy_bf16 and y; writes dx and (with a residual) d(residual) fp32
        nbytes = n * (d * ((4 if dy is not None else 0) + (2 if dyb is not None else 0) + 4 + es
                           + (4 if has_res else 0)) + 4)
        with _timed("ln_bwd", nbytes, "byte"):
            N.call("dna_ln_bwd_from_y_acc" if direct else "dna_ln_bwd_from_y", _p(dy), _p(dyb),
                   y.data_ptr(), _dt(dx), p, seed, off, gamma.data_ptr(), beta.data_ptr(),
                   rstd.data_ptr(), n, d, _p(dres), dx.data_ptr(), dg.data_ptr(), db.data_ptr(),
                   _p(dbias), ws.data_ptr(), nws, N.stream_ptr())
        if direct:
            for q in ctx.params:
                notify = getattr(q, "_dna_notify", None) if q is not None else None
                if notify is not None:
                    notify(q)
            return dx, None, dres, None, None, None, None, None, None, None, None, None
        return dx, dbias, dres, dg, db, None, None, None, None, None, None, None


# DNA_LN_BWD_FROM_Y=0: the LayerNorm backward recomputes x_hat from x (+ bias, dropout) + the
# residual instead of from the fp32 output (A/B switch)
_LN_BWD_FROM_Y = os.environ.get("DNA_LN_BWD_FROM_Y", "1") != "0"


class AddLayerNorm(torch.autograd.Function):
    """Pre-norm residual add + LN: (x, residual fp32) -> (sum = x + residual fp32, LN(sum) fp32
    or bf16) in one pass (dna_add_ln_fwd); beta None = RMSNorm (mamba_ssm's fused add + RMSNorm
    of the Caduceus Blocks). The flash_attn Block's `residual = dropout(x) +
    residual; norm(residual)` with residual_in_fp32 and dropout p = 0 (HyenaDNA's Blocks,
    long_conv_lm.py:205-267): same fp32 sum, same LN. The backward adds the gradient of `sum`
    from the residual stream to the LN's input gradient in the same kernel (dna_add_ln_bwd), so
    the add node, autograd's gradient accumulation and the cast of x's gradient are gone."""

    @staticmethod
    def forward(ctx, x, residual, gamma, beta, eps, want_bf16):
        _gpu(x, residual, gamma, beta)
        ctx.set_materialize_grads(False)
        x, residual = x.contiguous(), residual.contiguous()
        n, d = x.shape
        rms = beta is None  # RMSNorm (AddRMSNorm)
        s = torch.empty(n, d, device=x.device, dtype=torch.float32)
        y = torch.empty(n, d, device=x.device, dtype=torch.bfloat16 if want_bf16 else torch.float32)
        mean = None if rms else torch.empty(n, device=x.device, dtype=torch.float32)
        rstd = torch.empty(n, device=x.device, dtype=torch.float32)
        nbytes = n * (d * (x.element_size() + 8 + y.element_size()) + 8)
        with _timed("ln_fwd", nbytes, "byte"):
            N.call("dna_add_ln_fwd", x.data_ptr(), _dt(x), residual.data_ptr(), gamma.data_ptr(),
                   _p(beta), n, d, eps, int(rms), s.data_ptr(),
                   None if want_bf16 else y.data_ptr(), y.data_ptr() if want_bf16 else None,
                   _p(mean), rstd.data_ptr(), N.stream_ptr())
        ctx.save_for_backward(x, residual, gamma, mean, rstd)
        ctx.rms = rms
        return s, y

    @staticmethod
    def backward(ctx, ds, dy):
        x, residual, gamma, mean, rstd = ctx.saved_tensors
        rms = ctx.rms
        n, d = x.shape
        dx = torch.empty_like(x)
        dres = torch.empty(n, d, device=x.device, dtype=torch.float32)
        dg = torch.empty_like(gamma)
        db = None if rms else torch.empty_like(gamma)
        nws = N.lib().dna_ln_bwd_workspace(n, d)
        ws = torch.empty(max(nws, 16), device=x.device, dtype=torch.uint8)
        dy = None if dy is None else dy.contiguous()
        ds = None if ds is None else ds.contiguous().float()
        dyf = dy if (dy is not None and dy.dtype == torch.float32) else None
        dyb = dy if (dy is not None and dy.dtype == torch.bfloat16) else None
        nbytes = n * (d * ((4 if dyf is not None else 0) + (2 if dyb is not None else 0)
                           + (4 if ds is not None else 0) + 2 * x.element_size() + 8) + 8)
        with _timed("ln_bwd", nbytes, "byte"):
            N.call("dna_add_ln_bwd", _p(dyf), _p(dyb), _p(ds), x.data_ptr(), _dt(x),
                   residual.data_ptr(), gamma.data_ptr(), _p(mean), rstd.data_ptr(), n, d, int(rms),
                   dres.data_ptr(), dx.data_ptr(), dg.data_ptr(), _p(db), ws.data_ptr(),
                   nws, N.stream_ptr())
        return dx, dres, dg, db, None, None


class RMSNormFn(torch.autograd.Function):
    """x * rsqrt(mean(x^2) + eps) * gamma -> (y fp32|None, y_bf16|None): mamba_ssm's RMSNorm
    as the Caduceus Blocks / norm_f apply it (modeling_caduceus.py:25-65, :214-216)."""

    @staticmethod
    def forward(ctx, x, gamma, eps, want_f32, want_bf16):
        _gpu(x, gamma)
        ctx.set_materialize_grads(False)
        x = x.contiguous()
        n, d = x.shape
        y = torch.empty(n, d, device=x.device, dtype=torch.float32) if want_f32 else None
        yb = torch.empty(n, d, device=x.device, dtype=torch.bfloat16) if want_bf16 else None
        rstd = torch.empty(n, device=x.device, dtype=torch.float32)
        nbytes = n * (d * (x.element_size() + (4 if want_f32 else 0) + (2 if want_bf16 else 0)) + 4)
        with _timed("rms_fwd", nbytes, "byte"):
            N.call("dna_rms_fwd", x.data_ptr(), _dt(x), gamma.data_ptr(), n, d, eps, _p(y), _p(yb),
                   rstd.data_ptr(), N.stream_ptr())
        ctx.save_for_backward(x, gamma, rstd)
        return y, yb

    @staticmethod
    def backward(ctx, dy, dyb):
        x, gamma, rstd = ctx.saved_tensors
        n, d = x.shape
        dx = torch.empty_like(x)
        dg = torch.empty_like(gamma)
        nws = N.lib().dna_ln_bwd_workspace(n, d)
        ws = torch.empty(max(nws, 16), device=x.device, dtype=torch.uint8)
        dy = None if dy is None else dy.contiguous()
        dyb = None if dyb is None else dyb.contiguous()
        nbytes = n * (d * ((4 if dy is not None else 0) + (2 if dyb is not None else 0)
                           + 2 * x.element_size()) + 4)
        with _timed("rms_bwd", nbytes, "byte"):
            N.call("dna_rms_bwd", _p(dy), _p(dyb), x.data_ptr(), _dt(x), gamma.data_ptr(),
                   rstd.data_ptr(), n, d, dx.data_ptr(), dg.data_ptr(), ws.data_ptr(), nws,
                   N.stream_ptr())
        return dx, dg, None, None, None


# ----------------------------------------------------------------------------------- attention
class AlibiAttention(torch.autograd.Function):
    """softmax(q k^T * scale - slope_h |i-j| + pad_bias) v on packed qkv [T, 3*H*D]."""

    @staticmethod
    def forward(ctx, qkv, key_valid, slopes, b, S, H, scale, bias_grad=False):
        _gpu(qkv, key_valid, slopes)
        qkv = qkv.contiguous()
        T = qkv.shape[0]
        D = qkv.shape[1] // (3 * H)
        out = torch.empty(T, H * D, device=qkv.device, dtype=qkv.dtype)
        lse = torch.empty(b, H, S, device=qkv.device, dtype=torch.float32)
        with _timed("attn_fwd", 4.0 * b * H * S * S * D):
            N.call("dna_attn_fwd", qkv.data_ptr(), _p(key_valid), slopes.data_ptr(), b, S, H, D,
                   _dt(qkv), scale, out.data_ptr(), lse.data_ptr(), N.stream_ptr())
        ctx.save_for_backward(qkv, out, lse, key_valid, slopes)
        ctx.cfg = (b, S, H, D, scale)
        ctx.bias_grad = bias_grad and qkv.dtype == torch.bfloat16
        return out

    @staticmethod
    def backward(ctx, dout):
        qkv, out, lse, key_valid, slopes = ctx.saved_tensors
        b, S, H, D, scale = ctx.cfg
        dqkv = torch.empty_like(qkv)
        delta = torch.empty(b * H * S, device=qkv.device, dtype=torch.float32)
        dout = dout.contiguous()
        part = None
        if ctx.bias_grad:  # column sums of dqkv (the packed projection's bias gradient), fused
            rows = N.lib().dna_attn_dbias_part_rows(b, S)
            part = torch.empty(rows, qkv.shape[1], device=qkv.device, dtype=torch.float32)
        with _timed("attn_bwd", 10.0 * b * H * S * S * D):
            N.call("dna_attn_bwd_ex", qkv.data_ptr(), out.data_ptr(), dout.data_ptr(),
                   lse.data_ptr(), _p(key_valid), slopes.data_ptr(), b, S, H, D, _dt(qkv), scale,
                   dqkv.data_ptr(), delta.data_ptr(), _p(part), N.stream_ptr())
        if part is not None:
            colsum = torch.empty(qkv.shape[1], device=qkv.device, dtype=torch.float32)
            N.call("dna_colsum_f32", part.data_ptr(), part.shape[0], part.shape[1],
                   colsum.data_ptr(), 0, N.stream_ptr())
            # picked up by Linear.backward of the projection that produced qkv (same tensor
            # object: nothing sits between the two nodes), instead of a dy.sum(0) pass
            dqkv._dna_colsum = colsum
        return dqkv, None, None, None, None, None, None, None


def alibi_attention(qkv, key_valid, slopes, b, S, H, scale=None, bias_grad=False):
    """bias_grad: also produce the column sums of dqkv in backward (bf16 path), for the bias of
    the linear layer that made qkv (see Linear.backward)."""
    D = qkv.shape[1] // (3 * H)
    return AlibiAttention.apply(qkv, key_valid, slopes, b, S, H,
                                scale if scale is not None else 1.0 / math.sqrt(D), bias_grad)


# ----------------------------------------------------------------------------------- GeGLU
def _geglu_forward(g, p, seed, off):
    """(a, fac): the GeGLU output and the backward factors fac = [d a / d g1 | d a / d g2]
    (dropout folded in; csrc/common.h geglu_fwd_fac), so the backward is dg = da * fac. From
    the gated_layers epilogue, which wrote fac in g's place (Linear, geglu=...), or the separate
    pass (dna_geglu_fwd; fac in a new buffer, g is left as it is)."""
    pre = getattr(g, "_dna_geglu", None)
    if pre is not None and pre[1] == (p, seed, off):
        a = pre[0]  # computed in the producing GEMM's epilogue (Linear, geglu=...)
        del g._dna_geglu
        return a, g
    g = g.contiguous()
    n, F2 = g.shape
    a = torch.empty(n, F2 // 2, device=g.device, dtype=g.dtype)
    fac = torch.empty_like(g)
    with _timed("geglu_fwd", n * F2 // 2 * 5 * g.element_size(), "byte"):
        N.call("dna_geglu_fwd", g.data_ptr(), _dt(g), n, F2 // 2, p, seed, off, a.data_ptr(),
               fac.data_ptr(), N.stream_ptr())
    return a, fac


class GeGLU(torch.autograd.Function):
    """dropout(gelu(g[:, :F]) * g[:, F:])   (bert_layers.py:292-296)."""

    @staticmethod
    def forward(ctx, g, p, seed, off):
        _gpu(g)
        a, fac = _geglu_forward(g, p, seed, off)
        ctx.save_for_backward(fac)
        return a

    @staticmethod
    def backward(ctx, da):
        (fac,) = ctx.saved_tensors
        n, F2 = fac.shape
        dg = torch.empty_like(fac)
        da = da.contiguous()
        with _timed("geglu_bwd", n * F2 // 2 * 5 * fac.element_size(), "byte"):
            N.call("dna_geglu_bwd", da.data_ptr(), fac.data_ptr(), _dt(fac), n, F2 // 2,
                   dg.data_ptr(), N.stream_ptr())
        return dg, None, None, None


# ----------------------------------------------------------------------------------- loss
class MaskedCrossEntropy(torch.autograd.Function):
    """sum_r CE(logits[r], target[r]) / denom  (fp32 math on bf16 or fp32 logits)."""

    @staticmethod
    def forward(ctx, logits, target, denom):
        _gpu(logits, target)
        logits = logits.contiguous()
        M, V = logits.shape
        loss = torch.empty(M, device=logits.device, dtype=torch.float32)
        lse = torch.empty_like(loss)
        target = target.contiguous()
        N.call("dna_xent_fwd", logits.data_ptr(), _dt(logits), target.data_ptr(), M, V,
               loss.data_ptr(), lse.data_ptr(), N.stream_ptr())
        ctx.save_for_backward(logits, target, lse)
        ctx.denom = float(denom)
        return loss.sum() / ctx.denom

    @staticmethod
    def backward(ctx, dloss):
        logits, target, lse = ctx.saved_tensors
        M, V = logits.shape
        dl = torch.empty_like(logits)
        dloss = dloss.detach().to(torch.float32).contiguous().reshape(1)
        N.call("dna_xent_bwd", logits.data_ptr(), _dt(logits), target.data_ptr(), lse.data_ptr(),
               dloss.data_ptr(), 1.0 / ctx.denom, M, V, dl.data_ptr(), N.stream_ptr())
        return dl, None, None


# ----------------------------------------------------------------------------------- GEMM
def _gemm_impl():
    """"hip" (default): forward and data-gradient GEMMs on csrc/gemm.hip; "torch": hipBLASLt
    through torch.mm (A/B switch, DNA_GEMM_IMPL)."""
    return os.environ.get("DNA_GEMM_IMPL", "hip")


def _hip_gemm_ok(x, w_lp, n_out, k_red):
    return (x.dtype == torch.bfloat16 and w_lp.dtype == torch.bfloat16 and x.is_cuda
            and k_red % 64 == 0 and n_out % 8 == 0 and _gemm_impl() == "hip")


def _f32_gemm_ok(x, w):
    """fp32 parity mode: exact-fp32 MFMA kernels (csrc/gemm_f32.hip) for every projection."""
    return (x.dtype == torch.float32 and w.dtype == torch.float32 and x.is_cuda
            and _gemm_impl() == "hip")


def _hip_linear_f32(x, w, bias):
    """y[M, N] = x[M, K] . w[N, K]^T (+ b), fp32 in / fp32 out (dna_linear_fwd_f32)."""
    x, w = x.contiguous(), w.contiguous()
    M, K = x.shape
    Nn = w.shape[0]
    y = torch.empty(M, Nn, device=x.device, dtype=torch.float32)
    b = None if bias is None else bias.float().contiguous()
    N.call("dna_linear_fwd_f32", x.data_ptr(), w.data_ptr(), _p(b), M, Nn, K, y.data_ptr(),
           N.stream_ptr())
    return y


def _hip_dgrad_f32(dy, w):
    """dx[M, K] = dy[M, N] . w[N, K], fp32 (dna_linear_dgrad_f32)."""
    dy, w = dy.contiguous(), w.contiguous()
    M, Nn = dy.shape
    K = w.shape[1]
    dx = torch.empty(M, K, device=dy.device, dtype=torch.float32)
    N.call("dna_linear_dgrad_f32", dy.data_ptr(), w.data_ptr(), M, Nn, K, dx.data_ptr(),
           N.stream_ptr())
    return dx


def _hip_wgrad_f32_parts(dy, x):
    """fp32 split-K partials [s, m, n] of dy^T x (dna_linear_wgrad_f32)."""
    dy, x = dy.contiguous(), x.contiguous()
    rows, m = dy.shape
    n = x.shape[1]
    s = N.lib().dna_linear_wgrad_f32_splits(rows, m, n)
    parts = torch.empty(s, m, n, device=dy.device, dtype=torch.float32)
    N.call("dna_linear_wgrad_f32", dy.data_ptr(), x.data_ptr(), rows, m, n, s, parts.data_ptr(),
           N.stream_ptr())
    return parts, s


def _geglu_fused_ok(x, w_lp):
    F2, K = w_lp.shape
    return (os.environ.get("DNA_GEGLU_FUSED", "1") != "0" and _hip_gemm_ok(x, w_lp, F2, K)
            and F2 % 256 == 0 and K >= 128)


def _hip_geglu_linear(x, w_nk, p, seed, off):
    """fac[M, 2F] (the GeGLU backward factors of g = x . w^T, in g's place) and
    a[M, F] = dropout(gelu(g1) g2) in one launch (dna_geglu_linear_fwd)."""
    x = x.contiguous()
    M, K = x.shape
    F2 = w_nk.shape[0]
    fac = torch.empty(M, F2, device=x.device, dtype=torch.bfloat16)
    a = torch.empty(M, F2 // 2, device=x.device, dtype=torch.bfloat16)
    N.call("dna_geglu_linear_fwd", x.data_ptr(), w_nk.data_ptr(), None, M, F2 // 2, K, float(p),
           seed, off, fac.data_ptr(), a.data_ptr(), N.stream_ptr())
    return fac, a


def _gelu_fc1_ok(x, w_lp):
    """dna_linear_gelu_fwd applies (the persistent kernel's lean body: N % 256, N <= 8192,
    K % 128); DNA_GELU_FC1_FUSED=0: torch's separate GELU pass (A/B)."""
    Nn, K = w_lp.shape
    return (os.environ.get("DNA_GELU_FC1_FUSED", "1") != "0" and _hip_gemm_ok(x, w_lp, Nn, K)
            and Nn % 256 == 0 and Nn <= 8192 and K % 128 == 0 and Nn * K * 2 < 2 ** 31)


def _hip_linear_gelu(x, w_nk, bias):
    """h = x . w_nk^T (+ fp32 bias) and act = bf16(gelu_tanh(h)) from one launch
    (dna_linear_gelu_fwd)."""
    x = x.contiguous()
    M, K = x.shape
    Nn = w_nk.shape[0]
    h = torch.empty(M, Nn, device=x.device, dtype=torch.bfloat16)
    act = torch.empty_like(h)
    N.call("dna_linear_gelu_fwd", x.data_ptr(), w_nk.data_ptr(), _p(bias), M, Nn, K, h.data_ptr(),
           act.data_ptr(), N.stream_ptr())
    return h, act


def _hip_linear(x, w_nk, bias):
    """y[M, N] = x[M, K] . w_nk[N, K]^T (+ fp32 bias): the persistent MFMA GEMM (dna_linear_fwd)."""
    x = x.contiguous()
    M, K = x.shape
    Nn = w_nk.shape[0]
    y = torch.empty(M, Nn, device=x.device, dtype=torch.bfloat16)
    N.call("dna_linear_fwd", x.data_ptr(), w_nk.data_ptr(), _p(bias), M, Nn, K, y.data_ptr(),
           N.stream_ptr())
    return y


def bias_grad(dy, bias=None):
    """fp32 sum over rows of dy [rows, cols] (a Linear's bias gradient): bf16 CUDA gradients
    with cols % 64 == 0 on the native two-stage column sum (dna_colsum_bf16, deterministic);
    everything else torch's sum."""
    rows, cols = dy.shape
    if (dy.dtype == torch.bfloat16 and dy.is_cuda and cols % 64 == 0 and rows >= 1
            and dy.is_contiguous() and dy.data_ptr() % 16 == 0):
        # bias: the parameter; under FlatParams direct gradients the column sum is added straight
        # into its fp32 .grad view (the kernel's accumulate mode) and None is returned -- no
        # AccumulateGrad add launch per bias and step (DNA_BIAS_GRAD_DIRECT=0: returned, A/B)
        direct = (bias is not None and os.environ.get("DNA_BIAS_GRAD_DIRECT", "1") != "0"
                  and _param_grads_direct((bias,)) and bias.grad.numel() == cols)
        out = bias.grad if direct else torch.empty(cols, device=dy.device, dtype=torch.float32)
        nws = N.lib().dna_colsum_bf16_workspace(rows, cols)
        ws = torch.empty(nws, device=dy.device, dtype=torch.uint8)
        with _timed("colsum", rows * cols * 2, "byte"):
            N.call("dna_colsum_bf16", dy.data_ptr(), rows, cols, out.data_ptr(), int(direct),
                   ws.data_ptr(), nws, N.stream_ptr())
        if direct:
            notify = getattr(bias, "_dna_notify", None)
            if notify is not None:
                notify(bias)
            return None
        return out
    return dy.sum(0, dtype=torch.float32)


class GeluLinear(torch.autograd.Function):
    """o = gelu_tanh(h) . w^T + b as one autograd node (the flash_attn Mlp's act + fc2 in the
    HyenaDNA Blocks, activation F.gelu(approximate="tanh")): forward = torch's GELU kernel then the
    persistent GEMM; backward = fc2's data gradient with the GELU backward in its epilogue
    (dna_gelu_linear_dgrad_p: dh = bf16(dy . w) * gelu'(h), the intermediate da never stored),
    weight gradient from a = gelu(h), bias gradient by the native column sum."""

    @staticmethod
    def forward(ctx, h, w, b, w_lp, w_lpt, act=None):
        _gpu(h)
        h = h.contiguous()
        # act: gelu(h) from fc1's GEMM epilogue (dna_linear_gelu_fwd), else torch's GELU pass
        a = act if act is not None else F.gelu(h, approximate="tanh")
        flops = 2.0 * h.shape[0] * w_lp.shape[0] * w_lp.shape[1]
        with _timed("gemm_hip", flops):
            o = _hip_linear(a, w_lp, None if b is None else b.float())
        ctx.save_for_backward(h, a, w_lpt)
        ctx.weight = w
        ctx.bias = b
        ctx.has_b = b is not None
        return o

    @staticmethod
    def backward(ctx, do):
        h, a, w_lpt = ctx.saved_tensors
        do = do.contiguous()
        M, F_ = h.shape
        Nn = do.shape[1]
        flops = 2.0 * M * Nn * F_
        dh = torch.empty_like(h)
        with _timed("gemm_gelu_bwd", flops):
            N.call("dna_gelu_linear_dgrad_p", do.data_ptr(), w_lpt.data_ptr(), h.data_ptr(), M, F_,
                   Nn, dh.data_ptr(), N.stream_ptr())
        dw = _weight_grad(ctx.weight, do, a, flops)
        db = bias_grad(do, ctx.bias) if ctx.has_b else None
        return dh, dw, db, None, None, None


def gelu_linear_ok(h, w):
    """GeluLinear applies: bf16 CUDA activations, the persistent kernel's shapes (fc2's output
    and input widths % 256: the forward is then the same GEMM hip_linear runs), the hand-written
    GEMM path enabled."""
    Nn, F_ = w.shape
    return (h.is_cuda and h.dtype == torch.bfloat16 and Nn % 256 == 0
            and F_ % 256 == 0 and _gemm_impl() == "hip"
            and os.environ.get("DNA_GELU_BWD_FUSED", "1") != "0")


def gelu_linear(h, w, b, act=None):
    """F.linear(F.gelu(h, approximate="tanh"), w, b) under bf16 autocast (GeluLinear); act:
    gelu(h) already computed by fc1's epilogue (hyena.hip_linear(..., gelu=True))."""
    lead, F_ = h.shape[:-1], h.shape[-1]
    w_lp = w.to(torch.bfloat16)
    y = GeluLinear.apply(h.reshape(-1, F_), w, b, w_lp, w_lp.t().contiguous(),
                         None if act is None else act.reshape(-1, F_))
    return y.view(*lead, w.shape[0])


class Linear(torch.autograd.Function):
    """y = x @ w_lp^T (+ b): forward and dgrad on the compute dtype copy `w_lp` of the fp32
    master weight `w` -- bf16: the hand-written MFMA kernel (csrc/gemm.hip), the data gradient
    on the transposed copy `w_lpt` (dx = dy . w = dy . (w^T)^T, both operands K-major); the
    weight gradient in fp32 from the token-major MFMA kernel (dna_linear_wgrad_p chunk partials
    folded into the flat gradient by dna_sum_slices_accum)."""

    @staticmethod
    def forward(ctx, x, w, w_lp, b, w_lpt, geglu=None, gelu=False):
        ctx.save_for_backward(x, w_lp, w_lpt)
        ctx.weight = w
        ctx.bias = b
        ctx.has_b = b is not None
        flops = 2.0 * x.shape[0] * w_lp.shape[0] * w_lp.shape[1]
        if geglu is not None and b is None and _geglu_fused_ok(x, w_lp):
            # g = x . w^T and a = dropout(gelu(g1) g2) in one launch (the GeGLU epilogue of the
            # persistent GEMM). The tensor returned in g's place holds the GeGLU backward factors
            # (g itself is never stored); `a` rides on it for the GeGLU node that follows, which
            # must be its only consumer (bit-identical to the separate dna_geglu_fwd pass, which
            # then does not run)
            with _timed("gemm_geglu", flops):
                g, a = _hip_geglu_linear(x, w_lp, *geglu)
            g._dna_geglu = (a, tuple(geglu))
            return g
        if gelu and _gelu_fc1_ok(x, w_lp):
            # h and gelu_tanh(h) from one launch; gelu(h) rides on h for the GeluLinear node
            # that follows (it carries the GELU backward: this node's gradient stays dh)
            with _timed("gemm_gelu", flops):
                h, act = _hip_linear_gelu(x, w_lp, b if (b is None or b.dtype == torch.float32) else b.float())
            h._dna_gelu = act
            return h
        if _hip_gemm_ok(x, w_lp, w_lp.shape[0], w_lp.shape[1]):
            with _timed("gemm_hip", flops):
                return _hip_linear(x, w_lp, b if (b is None or b.dtype == torch.float32) else b.float())
        if _f32_gemm_ok(x, w_lp):
            with _timed("gemm_f32", flops):
                return _hip_linear_f32(x, w_lp, b)
        library_fallback("linear forward", x.shape, w_lp.shape)
        with _timed("gemm", flops):
            if b is not None:
                return torch.addmm(b.to(x.dtype), x, w_lp.t())
            return torch.mm(x, w_lp.t())

    @staticmethod
    def backward(ctx, dy):
        x, w_lp, w_lpt = ctx.saved_tensors
        colsum = getattr(dy, "_dna_colsum", None)
        dy = dy.contiguous()
        if colsum is not None:
            dy._dna_colsum = colsum
        flops = 2.0 * x.shape[0] * w_lp.shape[0] * w_lp.shape[1]
        dx = None
        if ctx.needs_input_grad[0]:
            if w_lpt is not None and _hip_gemm_ok(dy, w_lpt, w_lpt.shape[0], w_lpt.shape[1]):
                with _timed("gemm_hip", flops):
                    dx = _hip_linear(dy, w_lpt, None)
            elif _f32_gemm_ok(dy, w_lp):
                with _timed("gemm_f32", flops):
                    dx = _hip_dgrad_f32(dy, w_lp)
            else:
                library_fallback("linear data gradient", dy.shape, w_lp.shape)
                with _timed("gemm", flops):
                    dx = torch.mm(dy, w_lp)
        dw = _weight_grad(ctx.weight, dy, x, flops)
        db = None
        if ctx.has_b:
            db = getattr(dy, "_dna_colsum", None)  # fused upstream (AlibiAttention.backward)
            if db is None:
                db = bias_grad(dy, ctx.bias)
        return dx, dw, None, db, None, None, None


# ------------------------------------------------------------------ weight-gradient side stream
# The weight gradient of a projection is off the backward's critical path: with a side stream
# (DNA_WGRAD_STREAM=1) it runs beside the next memory-bound kernels of the backward (GeGLU /
# LayerNorm backward). Measured at the bench shape (interleaved A/B): +1.0-1.2 % step throughput
# -- the GEMM blocks hold the CUs and the LayerNorm backward beside them stretches 0.30 -> 1.08 ms
# per launch -- so it is off by default (the per-kernel timings then stay clean).
_SIDE = {}


def _side_stream():
    if os.environ.get("DNA_WGRAD_STREAM", "0") != "1":
        return None
    dev = torch.cuda.current_device()
    st = _SIDE.get(dev)
    if st is None:
        st = _SIDE[dev] = torch.cuda.Stream(device=dev)
    return st


_JOIN_QUEUED = [False]
_KEEP = []  # dy / x of side-stream wgrads, released once the current stream has joined


def join_side_stream():
    """Make the current stream wait for every weight gradient queued on the side stream. Queued
    automatically at the end of every backward that used it (autograd engine callback), so
    whatever reads the gradients after backward() -- all-reduce, clipping, optimizer, tests --
    sees them complete; the gradient-bucket reducer also calls it before each collective."""
    _JOIN_QUEUED[0] = False
    st = _SIDE.get(torch.cuda.current_device()) if torch.cuda.is_available() else None
    if st is not None:
        torch.cuda.current_stream().wait_stream(st)
    # safe to release now: later users of these blocks run on the current stream, behind the join
    _KEEP.clear()


def _queue_join():
    if not _JOIN_QUEUED[0]:
        _JOIN_QUEUED[0] = True
        torch.autograd.Variable._execution_engine.queue_callback(join_side_stream)


def wgrad_splits(rows, m, n, target_tiles=512, max_splits=None):
    """Split-K factor for dW = dY^T X: the contraction runs over all `rows` tokens while the
    output has only (m/256)*(n/256) tiles (9..72 for DNABERT-2), far fewer than 256 CUs.
    Smallest power of two giving >= target_tiles tiles, capped at 64 (measured at b=256: Wqkv
    545 us at s=32 vs 635-738 at s=16; Wg best at 8, Wwo at 16, Wo flat from 16 to 64)."""
    if max_splits is None:
        max_splits = int(os.environ.get("DNA_WGRAD_MAX_SPLITS", 64))
    tiles = max(1, (m // 256) * (n // 256))
    s = 1
    while s < max_splits and tiles * s < target_tiles:
        s *= 2
    while s > 1 and (rows % s or rows // s < 256):
        s //= 2
    return s


def _hip_wgrad_ok(dy, x):
    """The persistent token-major weight-gradient kernel (dna_linear_wgrad_p) for every bf16
    projection with 256-multiple sides -- all of DNABERT-2's. At the bench shapes (T = 262,144)
    it is 1-22 % faster than hipBLASLt's split-K batched GEMM (0.40-0.43 of the bf16 peak vs
    0.34-0.42; profiles/r03/wgrad_ab*.jsonl). DNA_WGRAD_IMPL=torch is the A/B arm."""
    rows, m = dy.shape
    n = x.shape[1]
    # the kernel needs two 64-row K-steps per split: a handful of rows (the MLM head's masked rows
    # of a tiny micro-batch, or none) goes to the torch split-K path
    return (dy.dtype == torch.bfloat16 and x.dtype == torch.bfloat16 and dy.is_cuda
            and rows >= 128 and m % 256 == 0 and n % 256 == 0 and _gemm_impl() == "hip"
            and os.environ.get("DNA_WGRAD_IMPL", "hip") == "hip")


def _hip_wgrad_parts(dy, x):
    """fp32 split-K partials [s, m, n] of dy^T x from the persistent MFMA kernel (token-major
    operands read in place; s chosen by the library to fill the grid)."""
    dy, x = dy.contiguous(), x.contiguous()
    rows, m = dy.shape
    n = x.shape[1]
    s = N.lib().dna_linear_wgrad_p_splits(rows, m, n)
    parts = torch.empty(s, m, n, device=dy.device, dtype=torch.float32)
    N.call("dna_linear_wgrad_p", dy.data_ptr(), x.data_ptr(), rows, m, n, s, parts.data_ptr(),
           N.stream_ptr())
    return parts, s


def wgrad(dy, x):
    """fp32 dW [m, n] = dy[rows, m]^T x[rows, n] (split-K partials + fp32 sum for bf16; the
    exact-fp32 MFMA kernel's slices for fp32)."""
    if _f32_gemm_ok(x, dy):
        parts, s = _hip_wgrad_f32_parts(dy, x)
        out = torch.empty(parts.shape[1:], device=dy.device, dtype=torch.float32)
        N.call("dna_sum_slices", parts.data_ptr(), s, out.numel(), out.data_ptr(), N.stream_ptr())
        return out
    if x.dtype == torch.float32:
        library_fallback("weight gradient", dy.shape, x.shape)
        return torch.mm(dy.t(), x)
    if _hip_wgrad_ok(dy, x):
        parts, s = _hip_wgrad_parts(dy, x)
        out = torch.empty(parts.shape[1:], device=dy.device, dtype=torch.float32)
        N.call("dna_sum_slices", parts.data_ptr(), s, out.numel(), out.data_ptr(), N.stream_ptr())
        return out
    library_fallback("weight gradient", dy.shape, x.shape)
    rows, m = dy.shape
    n = x.shape[1]
    s = wgrad_splits(rows, m, n)
    if s == 1:
        return torch.mm(dy.t(), x, out_dtype=torch.float32)
    a = dy.view(s, rows // s, m).transpose(1, 2)
    b = x.view(s, rows // s, n)
    return torch.bmm(a, b, out_dtype=torch.float32).sum(0)


def wgrad_accumulate(dy, x, grad):
    """grad[m, n] += dy^T x: split-K partials (the persistent MFMA kernel; hipBLASLt batched GEMM
    for shapes it does not take, or with DNA_WGRAD_IMPL=torch) folded in by one native pass."""
    rows, m = dy.shape
    n = x.shape[1]
    assert grad.is_contiguous() and grad.dtype == torch.float32 and grad.shape == (m, n)
    if _hip_wgrad_ok(dy, x):
        parts, s = _hip_wgrad_parts(dy, x)
        N.call("dna_sum_slices_accum", parts.data_ptr(), s, m * n, grad.data_ptr(), N.stream_ptr())
        return
    library_fallback("weight gradient", dy.shape, x.shape)
    s = wgrad_splits(rows, m, n)
    if s == 1:
        parts = torch.mm(dy.t(), x, out_dtype=torch.float32)
    else:
        parts = torch.bmm(dy.view(s, rows // s, m).transpose(1, 2), x.view(s, rows // s, n),
                          out_dtype=torch.float32)
    N.call("dna_sum_slices_accum", parts.data_ptr(), s, m * n, grad.data_ptr(), N.stream_ptr())


def _weight_grad(w, dy, x, flops):
    """dW = dy^T x of the projection with fp32 master weight w: straight into the flat gradient
    buffer when a FlatParams owns w (None returned, bucket reducer notified), else returned."""
    direct = (getattr(w, "_dna_direct", False) and w.grad is not None and x.dtype != torch.float32
              and _hip_wgrad_ok(dy, x))
    side = _side_stream() if direct else None
    if side is not None:
        # wgrad beside the rest of the backward; dy / x must outlive it on the side stream
        side.wait_stream(torch.cuda.current_stream())
        _KEEP.append((dy, x))  # (record_stream instead made the allocator thrash)
        with torch.cuda.stream(side), _timed("gemm_wgrad", flops):
            wgrad_accumulate(dy, x, w.grad)
        _queue_join()
        notify = getattr(w, "_dna_notify", None)
        if notify is not None:
            notify(w)
        return None
    with _timed("gemm_wgrad", flops):
        if direct:
            # write straight into the flat fp32 gradient buffer (dna_amd.flat) and tell the
            # gradient-bucket reducer, instead of returning dW to AccumulateGrad
            wgrad_accumulate(dy, x, w.grad)
            notify = getattr(w, "_dna_notify", None)
            if notify is not None:
                notify(w)
            return None
        return wgrad(dy, x)


def geglu_out_fused_ok(g, w_lp, w_lpt):
    """GeGLUOut applies: bf16 path, the transposed wo copy present, kernel-legal shapes
    (hidden % 128, F % 256), DNA_GEGLU_BWD_FUSED not 0."""
    if w_lpt is None or os.environ.get("DNA_GEGLU_BWD_FUSED", "1") == "0":
        return False
    Nh, F = w_lp.shape
    return (g.dtype == torch.bfloat16 and _hip_gemm_ok(g, w_lp, Nh, F) and w_lpt.shape == (F, Nh)
            and g.shape[1] == 2 * F and Nh % 128 == 0 and F % 256 == 0)


class GeGLUOut(torch.autograd.Function):
    """o = dropout(gelu(g[:, :F]) * g[:, F:]) . wo^T  (bert_layers.py:292-297, the bias going to
    the LayerNorm that follows) as ONE autograd node, so its backward runs the data gradient of
    wo and the GeGLU backward in one launch (dna_geglu_linear_dgrad_p: dg straight from dy, da
    never in memory) beside wo's weight gradient. Forward: the GeGLU output `a` from the
    gated_layers epilogue (Linear, geglu=...) or the separate pass, then the persistent GEMM."""

    @staticmethod
    def forward(ctx, g, p, seed, off, w, w_lp, w_lpt):
        _gpu(g)
        g = g.contiguous()
        # the same `a` (fused epilogue or dna_geglu_fwd) and the backward factors
        a, fac = _geglu_forward(g, p, seed, off)
        n, F2 = g.shape
        flops = 2.0 * n * w_lp.shape[0] * w_lp.shape[1]
        with _timed("gemm_hip", flops):
            o = _hip_linear(a, w_lp, None)
        ctx.save_for_backward(fac, a, w_lpt)
        ctx.weight = w
        return o

    @staticmethod
    def backward(ctx, dy):
        fac, a, w_lpt = ctx.saved_tensors
        dy = dy.contiguous()
        n, F2 = fac.shape
        Nh = dy.shape[1]
        flops = 2.0 * n * Nh * (F2 // 2)
        dg = torch.empty_like(fac)
        with _timed("gemm_geglu_bwd", flops):
            N.call("dna_geglu_linear_dgrad_p", dy.data_ptr(), w_lpt.data_ptr(), fac.data_ptr(), n,
                   F2 // 2, Nh, dg.data_ptr(), N.stream_ptr())
        dw = _weight_grad(ctx.weight, dy, a, flops)
        return dg, None, None, None, dw, None, None


def geglu_out(g, p, seed, off, w, w_lp, w_lpt):
    return GeGLUOut.apply(g, p, seed, off, w, w_lp, w_lpt)


def linear(x, w, w_lp, b=None, w_lpt=None, geglu=None):
    """geglu=(p, seed, offset): the output feeds GeGLU.apply(y, p, seed, offset) next -- fuse
    that GeGLU forward into the GEMM epilogue when the shapes allow (DNA_GEGLU_FUSED=0: never)."""
    return Linear.apply(x, w, w_lp if w_lp is not None else w, b, w_lpt, geglu)
