"""GPU: the strided MFMA GEMM (dna_gemm_bf16_strided / dna_gemm_f32_strided) against fp32 torch
matmul on the same bf16 / fp32 operands, for every operand layout (k- or m/n-contiguous A and B),
ragged edges (M, N, K not multiples of the tile, rows not 16-B aligned), a batch, split-K slices,
biases and both output types; and ChannelLinear (the Mamba x_proj / dt_proj products) forward and
backward under bf16 autocast vs an fp32 torch restatement. Tolerances: fp32 1e-5, bf16 output
1e-2, fp32 output from bf16 inputs 2e-5 (relative to the max |ref|)."""
import pytest
import torch

from dna_amd import _native as N
from dna_amd.mamba import ChannelLinear, _strided_gemm

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _rel(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return float((a - b).abs().max() / (b.abs().max() + 1e-30))


def _operand(rows, cols, contig_rows, dtype, g, batch):
    """A logical [batch, rows, cols] operand stored with unit stride along cols (contig_rows False)
    or along rows (True); returns (storage tensor, logical view)."""
    if contig_rows:
        t = torch.randn(batch, cols, rows, generator=g).to(dtype).to(DEV)
        return t, t.transpose(1, 2)
    t = torch.randn(batch, rows, cols, generator=g).to(dtype).to(DEV)
    return t, t


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("a_mc,b_nc", [(False, False), (False, True), (True, False), (True, True)])
@pytest.mark.parametrize("M,N_,K,batch,splits", [(48, 300, 512, 2, 1), (512, 1000, 16, 1, 1),
                                                   (16, 136, 48, 3, 1), (48, 512, 1500, 2, 4),
                                                   (130, 129, 77, 1, 3)])
def test_strided_gemm_vs_torch(dtype, a_mc, b_nc, M, N_, K, batch, splits):
    g = torch.Generator().manual_seed(M * 7 + N_ + K)
    # A(m, k): unit stride along k unless a_mc; B(k, n): unit stride along k if not b_nc
    a_st, A = _operand(M, K, a_mc, dtype, g, batch)
    b_st, B = _operand(N_, K, b_nc, dtype, g, batch)       # logical [batch, N, K]
    B = B.transpose(1, 2)                                   # logical [batch, K, N]
    ref = torch.einsum("zmk,zkn->zmn", A.double(), B.double())
    out_f32 = dtype == torch.float32 or splits > 1
    C = torch.full((batch * splits, M, N_), float("nan"), device=DEV,
                   dtype=torch.float32 if out_f32 else dtype)
    sa = (A.stride(1), A.stride(2), A.stride(0))
    sb = (B.stride(1), B.stride(2), B.stride(0))
    _strided_gemm(a_st, sa, b_st, sb, C, (N_, M * N_), M, N_, K, batch, splits, out_f32=out_f32)
    got = C.view(batch, splits, M, N_).double().sum(1)
    tol = 1e-5 if dtype == torch.float32 else (2e-5 if out_f32 else 1e-2)
    assert _rel(got, ref) < tol


def test_strided_gemm_bias_and_k_zero():
    g = torch.Generator().manual_seed(1)
    A = torch.randn(64, 40, generator=g).bfloat16().to(DEV)
    B = torch.randn(40, 200, generator=g).bfloat16().to(DEV)
    bm = torch.randn(64, generator=g).to(DEV)
    bn = torch.randn(200, generator=g).to(DEV)
    C = torch.empty(64, 200, device=DEV, dtype=torch.float32)
    N.call("dna_gemm_bf16_strided", A.data_ptr(), 40, 1, 0, B.data_ptr(), 200, 1, 0,
           C.data_ptr(), 200, 0, 1, bm.data_ptr(), bn.data_ptr(), 64, 200, 40, 1, 1,
           N.stream_ptr())
    ref = A.double() @ B.double() + bm.double()[:, None] + bn.double()[None, :]
    assert _rel(C, ref) < 2e-5
    N.call("dna_gemm_bf16_strided", A.data_ptr(), 40, 1, 0, B.data_ptr(), 200, 1, 0,
           C.data_ptr(), 200, 0, 1, bm.data_ptr(), None, 64, 200, 0, 1, 1, N.stream_ptr())
    assert torch.equal(C, bm[:, None].expand(64, 200))   # K == 0: bias only


@pytest.mark.parametrize("b,K,M,L", [(2, 512, 48, 1000), (1, 16, 512, 4096), (3, 64, 36, 301)])
def test_channel_linear_autocast_vs_fp32(b, K, M, L):
    g = torch.Generator().manual_seed(L)
    x = torch.randn(b, K, L, generator=g).to(DEV).bfloat16().requires_grad_(True)
    w = (torch.randn(M, K, generator=g) / K ** 0.5).to(DEV).requires_grad_(True)
    dy = torch.randn(b, M, L, generator=g).to(DEV)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        y = ChannelLinear.apply(x, w)
    assert y.dtype == torch.bfloat16
    xr = x.detach().float().requires_grad_(True)
    wr = w.detach().bfloat16().float().requires_grad_(True)
    yr = torch.einsum("mk,bkl->bml", wr, xr)
    assert _rel(y, yr) < 1e-2
    y.backward(dy.bfloat16())
    yr.backward(dy.bfloat16().float())
    assert x.grad.dtype == torch.bfloat16 and w.grad.dtype == torch.float32
    assert _rel(x.grad, xr.grad) < 1e-2
    assert _rel(w.grad, wr.grad) < 1e-4   # fp32 slices of exact bf16 products


def test_channel_linear_sliced_input_fp32():
    """dt_proj's input is a channel slice of x_dbl (batch stride 48 L): no copy, same result."""
    g = torch.Generator().manual_seed(3)
    xd = torch.randn(2, 48, 777, generator=g).to(DEV).requires_grad_(True)
    w = torch.randn(96, 16, generator=g).to(DEV).requires_grad_(True)
    y = ChannelLinear.apply(xd[:, :16], w)
    yr = torch.einsum("mk,bkl->bml", w.double(), xd[:, :16].double())
    assert _rel(y, yr) < 1e-5
    dy = torch.randn(2, 96, 777, generator=g).to(DEV)
    y.backward(dy)
    xr = xd.detach().double().requires_grad_(True)
    wr = w.detach().double().requires_grad_(True)
    torch.einsum("mk,bkl->bml", wr, xr[:, :16]).backward(dy.double())
    assert _rel(xd.grad, xr.grad) < 1e-5 and _rel(w.grad, wr.grad) < 1e-5
    assert float(xd.grad[:, 16:].abs().max()) == 0.0


@pytest.mark.parametrize("M,N_,K,batch,bias", [(1024, 4096, 256, 1, False), (1024, 2048, 256, 2, True),
                                               (100, 1001, 64, 2, True), (300, 77, 128, 3, False),
                                               (256, 64, 256, 1, True)])
def test_proj_cm_vs_fp32(M, N_, K, batch, bias):
    """dna_proj_cm_bf16 (register-resident weight, channel-major output; the Mamba in_proj
    forward) against an fp32 matmul of the same bf16 operands: bf16 output rounding only."""
    g = torch.Generator(device=DEV).manual_seed(M + N_ + K)
    W = torch.randn(M, K, device=DEV, generator=g).to(torch.bfloat16)
    X = torch.randn(batch, N_, K, device=DEV, generator=g).to(torch.bfloat16)
    b = torch.randn(M, device=DEV, generator=g) if bias else None
    C = torch.full((batch, M, N_), float("nan"), device=DEV, dtype=torch.bfloat16)
    N.call("dna_proj_cm_bf16", W.data_ptr(), X.data_ptr(), None if b is None else b.data_ptr(),
           M, N_, K, batch, 0, C.data_ptr(), N.stream_ptr())
    ref = torch.einsum("ck,zlk->zcl", W.float(), X.float())
    if b is not None:
        ref = ref + b[None, :, None]
    err = (C.float() - ref).abs().max() / ref.abs().max()
    assert torch.isfinite(C.float()).all()
    assert err < 8e-3, err


def test_proj_cm_rejects_bad_k():
    with pytest.raises(N.NativeError, match="K=96"):
        N.call("dna_proj_cm_bf16", 16, 16, None, 64, 64, 96, 1, 0, 16, None)


@pytest.mark.parametrize("M,N_,K,batch", [(512, 4096, 48, 1), (64, 301, 16, 2)])
def test_strided_gemm_accumulate(M, N_, K, batch):
    """accumulate=True: C = bf16(A B + C) in the epilogue (the x_proj data gradient summed into
    the scan's du), against fp32 A B + C."""
    from dna_amd.functional import strided_gemm
    g = torch.Generator(device=DEV).manual_seed(M * 7 + N_)
    W = torch.randn(K, M, device=DEV, generator=g).to(torch.bfloat16)        # A(m, k) = W[k][m]
    dy = torch.randn(batch, K, N_, device=DEV, generator=g).to(torch.bfloat16)
    C0 = torch.randn(batch, M, N_, device=DEV, generator=g).to(torch.bfloat16)
    C = C0.clone()
    strided_gemm(W, (1, M, 0), dy, (N_, 1, K * N_), C, (N_, M * N_), M, N_, K, batch,
                 accumulate=True)
    ref = torch.einsum("km,zkn->zmn", W.float(), dy.float()) + C0.float()
    err = (C.float() - ref).abs().max() / ref.abs().max()
    assert err < 8e-3, err
