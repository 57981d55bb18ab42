"""The hot-path HIP kernels as PyTorch operators: `torch.ops.dna_amd.<op>` (SURVEY §8(b) kernel
boundary).

Each op wraps one C-ABI entry point of include/dna_amd.h, runs on the current torch HIP stream,
writes into caller-allocated outputs (declared as mutated arguments), and raises a Python
exception on dtype / shape / contiguity / device errors -- the checks the reference's Triton slot
asserts (flash_attn_triton.py:849-855) -- instead of letting a kernel read out of bounds.

    torch.ops.dna_amd.attn_fwd(qkv, key_valid, slopes, b, S, H, scale, out, lse)
    torch.ops.dna_amd.attn_bwd(qkv, out, dout, lse, key_valid, slopes, b, S, H, scale, dqkv)
    torch.ops.dna_amd.linear_fwd(x, w, bias, y)                   y = x w^T (+ bias), bf16 MFMA
    torch.ops.dna_amd.geglu_fwd(g, p, seed, offset, a, fac)       a = dropout(gelu(g1) g2),
                                                                  fac = backward factors
    torch.ops.dna_amd.geglu_bwd(da, fac, dg)                      dg = da * fac
    torch.ops.dna_amd.xent_fwd(logits, target, loss, lse)         per-row CE
    torch.ops.dna_amd.transpose_bf16(src, dst)
and the reference's FlashAttention kernel slot with its own signature (flash_attn_triton.py:
1077-1130, called at bert_layers.py:188/192 as flash_attn_qkvpacked_func(qkv, bias)), autograd
included:

    out = dna_amd.ops.flash_attn_qkvpacked_func(qkv[b,S,3,H,D], bias=None, causal=False,
                                                softmax_scale=None)
    out, lse = torch.ops.dna_amd.flash_attn_qkvpacked(qkv, bias, causal, softmax_scale)
with the reference's bias forms ("vector" [., ., 1, S] / "matrix" [., ., S, S], batch / head
broadcast, fp32 or the qkv dtype), fp16 and bf16, any S, head_dim <= 128 (csrc/flash_slot.hip).
The model itself runs the fast path, where the ALiBi + key-pad bias enters as (slopes,
key_valid) instead of a materialised [b,H,S,S] tensor: bias[h,i,j] = -slopes[h]*|i-j| +
(key j pad ? -10000 : 0), exactly what bert_layers.py:421-448 builds:

    out = dna_amd.ops.alibi_attn_qkvpacked_func(qkv, slopes, key_valid, softmax_scale)
The model's own autograd Functions (dna_amd.functional) call the C ABI directly (no per-call
dispatcher overhead on the ~300 launches of a step).
"""
import math

import torch

from . import _native as N

_DT = {torch.float32: N.F32, torch.bfloat16: N.BF16}


def _check(cond, msg):
    if not cond:
        raise RuntimeError(f"dna_amd: {msg}")


def _cuda_contig(name, t, dtypes=None):
    _check(t.is_cuda, f"{name} must be on the GPU (no CPU fallback), got {t.device}")
    _check(t.is_contiguous(), f"{name} must be contiguous")
    if dtypes is not None:
        _check(t.dtype in dtypes, f"{name} dtype {t.dtype} not in {dtypes}")


def _p(t):
    return None if t is None else t.data_ptr()


# ------------------------------------------------------------------------------- attention
@torch.library.custom_op("dna_amd::attn_fwd", mutates_args=("out", "lse"))
def attn_fwd(qkv: torch.Tensor, key_valid: torch.Tensor | None, slopes: torch.Tensor, b: int,
             S: int, H: int, scale: float, out: torch.Tensor, lse: torch.Tensor) -> None:
    _cuda_contig("qkv", qkv, (torch.bfloat16, torch.float32))
    _check(qkv.dim() == 2 and qkv.shape[0] == b * S and qkv.shape[1] % (3 * H) == 0,
           f"qkv must be [b*S, 3*H*D], got {tuple(qkv.shape)}")
    D = qkv.shape[1] // (3 * H)
    _cuda_contig("out", out, (qkv.dtype,))
    _check(tuple(out.shape) == (b * S, H * D), "out must be [b*S, H*D]")
    _cuda_contig("lse", lse, (torch.float32,))
    _check(lse.numel() == b * H * S, "lse must hold b*H*S floats")
    _cuda_contig("slopes", slopes, (torch.float32,))
    if key_valid is not None:
        _cuda_contig("key_valid", key_valid, (torch.uint8, torch.bool))
        _check(key_valid.numel() == b * S, "key_valid must hold b*S entries")
    N.call("dna_attn_fwd", qkv.data_ptr(), _p(key_valid), slopes.data_ptr(), b, S, H, D,
           _DT[qkv.dtype], scale, out.data_ptr(), lse.data_ptr(), N.stream_ptr())


@torch.library.custom_op("dna_amd::attn_bwd", mutates_args=("dqkv",))
def attn_bwd(qkv: torch.Tensor, out: torch.Tensor, dout: torch.Tensor, lse: torch.Tensor,
             key_valid: torch.Tensor | None, slopes: torch.Tensor, b: int, S: int, H: int,
             scale: float, dqkv: torch.Tensor) -> None:
    for n, t in (("qkv", qkv), ("out", out), ("dout", dout), ("dqkv", dqkv)):
        _cuda_contig(n, t, (qkv.dtype,))
    _cuda_contig("lse", lse, (torch.float32,))
    _check(dqkv.shape == qkv.shape and dout.shape == out.shape, "dqkv / dout shapes")
    D = qkv.shape[1] // (3 * H)
    delta = torch.empty(b * H * S, device=qkv.device, dtype=torch.float32)
    N.call("dna_attn_bwd", qkv.data_ptr(), out.data_ptr(), dout.data_ptr(), lse.data_ptr(),
           _p(key_valid), slopes.data_ptr(), b, S, H, D, _DT[qkv.dtype], scale, dqkv.data_ptr(),
           delta.data_ptr(), N.stream_ptr())


@torch.library.custom_op("dna_amd::alibi_attn_qkvpacked", mutates_args=())
def alibi_attn_qkvpacked(qkv: torch.Tensor, slopes: torch.Tensor, key_valid: torch.Tensor | None,
                         softmax_scale: float | None = None) -> tuple[torch.Tensor, torch.Tensor]:
    """The model's fast path: the ALiBi + key-pad bias of bert_layers.py:421-448 from (slopes,
    key_valid), never materialised. -> (out [b, S, H, D], lse [b, H, S] fp32 natural log)."""
    _check(qkv.dim() == 5 and qkv.shape[2] == 3, f"qkv must be [b, S, 3, H, D], got {tuple(qkv.shape)}")
    b, S, _, H, D = qkv.shape
    scale = softmax_scale if softmax_scale is not None else 1.0 / math.sqrt(D)
    packed = qkv.contiguous().view(b * S, 3 * H * D)
    out = torch.empty(b * S, H * D, device=qkv.device, dtype=qkv.dtype)
    lse = torch.empty(b, H, S, device=qkv.device, dtype=torch.float32)
    kv = None if key_valid is None else key_valid.to(torch.uint8).contiguous()
    attn_fwd(packed, kv, slopes.float().contiguous(), b, S, H, scale, out, lse)
    return out.view(b, S, H, D), lse


@alibi_attn_qkvpacked.register_fake
def _(qkv, slopes, key_valid, softmax_scale=None):
    b, S, _, H, D = qkv.shape
    return qkv.new_empty(b, S, H, D), qkv.new_empty(b, H, S, dtype=torch.float32)


def _alibi_setup(ctx, inputs, output):
    qkv, slopes, key_valid, softmax_scale = inputs
    out, lse = output
    ctx.save_for_backward(qkv, slopes, key_valid if key_valid is not None else torch.empty(0),
                          out, lse)
    ctx.has_kv = key_valid is not None
    ctx.scale = softmax_scale


def _alibi_backward(ctx, dout, dlse):
    qkv, slopes, key_valid, out, lse = ctx.saved_tensors
    b, S, _, H, D = qkv.shape
    scale = ctx.scale if ctx.scale is not None else 1.0 / math.sqrt(D)
    packed = qkv.contiguous().view(b * S, 3 * H * D)
    kv = key_valid.to(torch.uint8).contiguous() if ctx.has_kv else None
    dqkv = torch.empty_like(packed)
    attn_bwd(packed, out.contiguous().view(b * S, H * D), dout.contiguous().view(b * S, H * D),
             lse, kv, slopes.float().contiguous(), b, S, H, scale, dqkv)
    return dqkv.view(qkv.shape), None, None, None


alibi_attn_qkvpacked.register_autograd(_alibi_backward, setup_context=_alibi_setup)


def alibi_attn_qkvpacked_func(qkv, slopes, key_valid=None, softmax_scale=None):
    """The fast path: out of alibi_attn_qkvpacked (bias = -slopes[h]*|i-j| + pad*-10000)."""
    return torch.ops.dna_amd.alibi_attn_qkvpacked(qkv, slopes, key_valid, softmax_scale)[0]


# ------------------------------------------------------------------- generic FlashAttention slot
_FDT = {torch.bfloat16: N.BF16, torch.float16: N.F16, torch.float32: N.F32}


def _bias_args(bias, b, H, S, qkv_dtype):
    """The reference's bias handling (flash_attn_triton.py:780-807): 4-D, fp32 or the qkv dtype,
    last dims (1, S) "vector" or (S, S) "matrix", first dims broadcastable to (b, H) -- broadcast
    as stride 0 here instead of repeat copies. -> (bias, dtype code, type, sb, sh, sq)."""
    if bias is None:
        return None, N.F32, 0, 0, 0, 0
    _check(bias.dtype in (qkv_dtype, torch.float32), f"bias dtype {bias.dtype} must be fp32 or {qkv_dtype}")
    _check(bias.is_cuda, "bias must be on the GPU")
    _check(bias.dim() == 4, f"bias must be 4-D, got {bias.dim()}-D")
    if bias.stride(-1) != 1:
        bias = bias.contiguous()
    if tuple(bias.shape[2:]) == (1, S):
        btype = 1
    elif tuple(bias.shape[2:]) == (S, S):
        btype = 2
    else:
        raise RuntimeError("Last 2 dimensions of bias must be (1, seqlen_k) or (seqlen_q, seqlen_k)")
    _check(bias.shape[0] in (1, b) and bias.shape[1] in (1, H),
           f"First 2 dimensions of bias must be broadcastible to (batch, nheads) = ({b}, {H}). "
           f"Bias has shape: {tuple(bias.shape)}")
    sb = bias.stride(0) if bias.shape[0] == b and b > 1 else 0
    sh = bias.stride(1) if bias.shape[1] == H and H > 1 else 0
    sq = bias.stride(2) if btype == 2 else 0
    return bias, _FDT[bias.dtype], btype, sb, sh, sq


def _pad_head(t, Dp):
    D = t.shape[-1]
    return t if D == Dp else torch.nn.functional.pad(t, (0, Dp - D))


def _kernel_dim(D):
    _check(D <= 128, "FlashAttention only support head dimensions up to 128")
    return 32 if D <= 32 else (64 if D <= 64 else 128)


@torch.library.custom_op("dna_amd::flash_attn_qkvpacked", mutates_args=())
def flash_attn_qkvpacked(qkv: torch.Tensor, bias: torch.Tensor | None = None, causal: bool = False,
                         softmax_scale: float | None = None) -> tuple[torch.Tensor, torch.Tensor]:
    """_flash_attn_forward over packed qkv [b, S, 3, H, D] (flash_attn_triton.py:767-860)
    -> (out [b, S, H, D], lse [b, H, ceil(S/128)*128] fp32 natural log)."""
    _check(qkv.dim() == 5 and qkv.shape[2] == 3, f"qkv must be [b, S, 3, H, D], got {tuple(qkv.shape)}")
    _check(qkv.dtype in (torch.float16, torch.bfloat16), "Only support fp16 and bf16")
    _check(qkv.is_cuda, "qkv must be on the GPU (no CPU fallback)")
    b, S, _, H, D = qkv.shape
    scale = softmax_scale if softmax_scale is not None else 1.0 / math.sqrt(D)
    Dp = _kernel_dim(D)
    x = _pad_head(qkv, Dp).contiguous()
    bias, bdt, btype, sb, sh, sq = _bias_args(bias, b, H, S, qkv.dtype)
    out = torch.empty(b, S, H, Dp, device=qkv.device, dtype=qkv.dtype)
    lse = torch.empty(b, H, N.lib().dna_flash_lse_rows(S), device=qkv.device, dtype=torch.float32)
    N.call("dna_flash_fwd", x.data_ptr(), _FDT[qkv.dtype], _p(bias), bdt, btype, sb, sh, sq, b, S, H,
           Dp, int(bool(causal)), scale, out.data_ptr(), lse.data_ptr(), N.stream_ptr())
    return (out if Dp == D else out[..., :D].contiguous()), lse


@flash_attn_qkvpacked.register_fake
def _(qkv, bias=None, causal=False, softmax_scale=None):
    b, S, _, H, D = qkv.shape
    return qkv.new_empty(b, S, H, D), qkv.new_empty(b, H, (S + 127) // 128 * 128, dtype=torch.float32)


def _flash_setup(ctx, inputs, output):
    qkv, bias, causal, softmax_scale = inputs
    out, lse = output
    ctx.save_for_backward(qkv, bias if bias is not None else torch.empty(0), out, lse)
    ctx.has_bias = bias is not None
    ctx.causal = bool(causal)
    ctx.scale = softmax_scale


def _flash_backward(ctx, dout, dlse):
    qkv, bias, out, lse = ctx.saved_tensors
    # flash_attn_triton.py:1109-1110
    _check(not (ctx.has_bias and ctx.needs_input_grad[1]),
           "FlashAttention does not support bias gradient yet")
    b, S, _, H, D = qkv.shape
    scale = ctx.scale if ctx.scale is not None else 1.0 / math.sqrt(D)
    Dp = _kernel_dim(D)
    x = _pad_head(qkv, Dp).contiguous()
    o = _pad_head(out, Dp).contiguous()
    g = _pad_head(dout, Dp).contiguous()
    bias, bdt, btype, sb, sh, sq = _bias_args(bias if ctx.has_bias else None, b, H, S, qkv.dtype)
    delta = torch.empty_like(lse)
    dqkv = torch.empty_like(x)
    N.call("dna_flash_bwd", x.data_ptr(), _FDT[qkv.dtype], _p(bias), bdt, btype, sb, sh, sq,
           o.data_ptr(), g.data_ptr(), lse.data_ptr(), b, S, H, Dp, int(ctx.causal), scale,
           delta.data_ptr(), dqkv.data_ptr(), N.stream_ptr())
    return (dqkv if Dp == D else dqkv[..., :D].contiguous()), None, None, None


flash_attn_qkvpacked.register_autograd(_flash_backward, setup_context=_flash_setup)


def flash_attn_qkvpacked_func(qkv, bias=None, causal=False, softmax_scale=None):
    """Drop-in for flash_attn_qkvpacked_func (flash_attn_triton.py:1077-1130, the reference's
    _FlashAttnQKVPackedFunc.apply): same positional signature and semantics -- qkv [b, S, 3, H, D]
    fp16 / bf16, bias broadcastible to (b, H, S, S) as "vector" [., ., 1, S] or "matrix"
    [., ., S, S] (fp32 or qkv dtype), causal, softmax_scale (default 1/sqrt(D)); returns
    out [b, S, H, D]; the backward gives dqkv (no bias gradient, as the reference)."""
    return torch.ops.dna_amd.flash_attn_qkvpacked(qkv, bias, bool(causal), softmax_scale)[0]


# ------------------------------------------------------------------------------- GEMM
@torch.library.custom_op("dna_amd::linear_fwd", mutates_args=("y",))
def linear_fwd(x: torch.Tensor, w: torch.Tensor, bias: torch.Tensor | None, y: torch.Tensor) -> None:
    _cuda_contig("x", x, (torch.bfloat16,))
    _cuda_contig("w", w, (torch.bfloat16,))
    _cuda_contig("y", y, (torch.bfloat16,))
    M, K = x.shape
    Nn = w.shape[0]
    _check(w.shape[1] == K and tuple(y.shape) == (M, Nn), "shapes: x[M,K], w[N,K], y[M,N]")
    _check(K % 64 == 0 and Nn % 8 == 0, f"K % 64 and N % 8 required (K={K}, N={Nn})")
    if bias is not None:
        _cuda_contig("bias", bias, (torch.float32,))
        _check(bias.numel() == Nn, "bias must hold N floats")
    N.call("dna_linear_fwd", x.data_ptr(), w.data_ptr(), _p(bias), M, Nn, K, y.data_ptr(),
           N.stream_ptr())


@torch.library.custom_op("dna_amd::transpose_bf16", mutates_args=("dst",))
def transpose_bf16(src: torch.Tensor, dst: torch.Tensor) -> None:
    _cuda_contig("src", src, (torch.bfloat16,))
    _cuda_contig("dst", dst, (torch.bfloat16,))
    r, c = src.shape
    _check(tuple(dst.shape) == (c, r), "dst must be src transposed")
    N.call("dna_transpose_bf16", src.data_ptr(), r, c, dst.data_ptr(), N.stream_ptr())


@torch.library.custom_op("dna_amd::geglu_linear_fwd", mutates_args=("fac", "a"))
def geglu_linear_fwd(x: torch.Tensor, w: torch.Tensor, bias: torch.Tensor | None, p: float,
                     seed: int, offset: int, fac: torch.Tensor, a: torch.Tensor) -> None:
    """g = x . w^T (+ bias), a = dropout(gelu(g[:, :F]) * g[:, F:]) and fac = the backward
    factors of geglu_fwd in one launch (gated_layers + GeGLU, bert_layers.py:292-296; g itself is
    not stored); same bits as linear_fwd + geglu_fwd."""
    _cuda_contig("x", x, (torch.bfloat16,))
    _cuda_contig("w", w, (torch.bfloat16,))
    _cuda_contig("fac", fac, (torch.bfloat16,))
    _cuda_contig("a", a, (torch.bfloat16,))
    M, K = x.shape
    F2 = w.shape[0]
    _check(w.shape[1] == K and tuple(fac.shape) == (M, F2) and tuple(a.shape) == (M, F2 // 2),
           "shapes: x[M,K], w[2F,K], fac[M,2F], a[M,F]")
    _check(K % 64 == 0 and F2 % 256 == 0, f"K % 64 and 2F % 256 required (K={K}, 2F={F2})")
    if bias is not None:
        _cuda_contig("bias", bias, (torch.float32,))
        _check(bias.numel() == F2, "bias must hold 2F floats")
    N.call("dna_geglu_linear_fwd", x.data_ptr(), w.data_ptr(), _p(bias), M, F2 // 2, K, float(p),
           seed, offset, fac.data_ptr(), a.data_ptr(), N.stream_ptr())


@torch.library.custom_op("dna_amd::geglu_linear_dgrad", mutates_args=("dg",))
def geglu_linear_dgrad(dy: torch.Tensor, wt: torch.Tensor, fac: torch.Tensor,
                       dg: torch.Tensor) -> None:
    """dg = geglu_bwd(dy . wt^T, fac) in one launch: wo's data gradient (wt = wo^T, [F, hidden])
    with the GeGLU backward in the epilogue (bert_layers.py:292-297); == linear_fwd + geglu_bwd."""
    _cuda_contig("dy", dy, (torch.bfloat16,))
    _cuda_contig("wt", wt, (torch.bfloat16,))
    _cuda_contig("fac", fac, (torch.bfloat16,))
    _cuda_contig("dg", dg, (torch.bfloat16,))
    M, H = dy.shape
    F = wt.shape[0]
    _check(wt.shape[1] == H and tuple(fac.shape) == (M, 2 * F) and dg.shape == fac.shape,
           "shapes: dy[M,H], wt[F,H], fac / dg[M,2F]")
    _check(H % 128 == 0 and H >= 256 and F % 256 == 0,
           f"hidden % 128, hidden >= 256 and F % 256 required (H={H}, F={F})")
    N.call("dna_geglu_linear_dgrad_p", dy.data_ptr(), wt.data_ptr(), fac.data_ptr(), M, F, H,
           dg.data_ptr(), N.stream_ptr())


# ------------------------------------------------------------------------------- elementwise
@torch.library.custom_op("dna_amd::geglu_fwd", mutates_args=("a", "fac"))
def geglu_fwd(g: torch.Tensor, p: float, seed: int, offset: int, a: torch.Tensor,
              fac: torch.Tensor) -> None:
    """a = dropout(gelu(g[:, :F]) * g[:, F:]); fac [rows, 2F] = the backward factors
    [d a / d g1 | d a / d g2] with the dropout folded in, for geglu_bwd (may be g itself)."""
    _cuda_contig("g", g, (torch.bfloat16, torch.float32))
    _cuda_contig("a", a, (g.dtype,))
    n, f2 = g.shape
    _check(tuple(a.shape) == (n, f2 // 2), "a must be [rows, F] for g [rows, 2F]")
    _cuda_contig("fac", fac, (g.dtype,))
    _check(fac.shape == g.shape, "fac must be shaped like g")
    N.call("dna_geglu_fwd", g.data_ptr(), _DT[g.dtype], n, f2 // 2, p, seed, offset, a.data_ptr(),
           fac.data_ptr(), N.stream_ptr())


@torch.library.custom_op("dna_amd::geglu_bwd", mutates_args=("dg",))
def geglu_bwd(da: torch.Tensor, fac: torch.Tensor, dg: torch.Tensor) -> None:
    """dg = [da * fac1 | da * fac2] (fac from geglu_fwd / geglu_linear_fwd)."""
    _cuda_contig("fac", fac, (torch.bfloat16, torch.float32))
    _cuda_contig("da", da, (fac.dtype,))
    _cuda_contig("dg", dg, (fac.dtype,))
    n, f2 = fac.shape
    _check(tuple(da.shape) == (n, f2 // 2) and dg.shape == fac.shape, "da [rows, F], dg like fac")
    N.call("dna_geglu_bwd", da.data_ptr(), fac.data_ptr(), _DT[fac.dtype], n, f2 // 2,
           dg.data_ptr(), N.stream_ptr())


@torch.library.custom_op("dna_amd::xent_fwd", mutates_args=("loss", "lse"))
def xent_fwd(logits: torch.Tensor, target: torch.Tensor, loss: torch.Tensor,
             lse: torch.Tensor) -> None:
    _cuda_contig("logits", logits, (torch.bfloat16, torch.float32))
    _cuda_contig("target", target, (torch.int64,))
    M, V = logits.shape
    _check(target.numel() == M and loss.numel() == M and lse.numel() == M, "row counts")
    N.call("dna_xent_fwd", logits.data_ptr(), _DT[logits.dtype], target.data_ptr(), M, V,
           loss.data_ptr(), lse.data_ptr(), N.stream_ptr())


OPS = ("attn_fwd", "attn_bwd", "alibi_attn_qkvpacked", "flash_attn_qkvpacked", "linear_fwd",
       "transpose_bf16", "geglu_linear_fwd", "geglu_linear_dgrad",
       "geglu_fwd", "geglu_bwd", "xent_fwd")
