// Exact-fp32 projections on the f32-input MFMA (v_mfma_f32_16x16x4_f32, gfx950): the fp32
// parity mode of the encoder (north_star: logits within 1e-3 of the reference's fp32 forward)
// runs every nn.Linear of bert_layers.py (Wqkv :158, attention dense :214, gated_layers :292,
// wo :297, MLM transform :560, tied decoder :664) and its backward on hand-written kernels too,
// not on a vendor GEMM. The instruction is bit-for-bit a k-ordered fmaf chain (one rounding per
// product), at the f32 rate (64 FLOP/clk/SIMD, 157 TF dense).
//
//   fwd    y[M,N]  = x[M,K] . w[N,K]^T (+ b)     A k-contiguous,  B k-contiguous
//   dgrad  dx[M,K] = dy[M,N] . w[N,K]            A k-contiguous,  B mn-contiguous
//   wgrad  dW[N,K] = dy[T,N]^T . x[T,K]          A mn-contiguous, B mn-contiguous; split-K over
//          tokens into fp32 slices [s][N][K] reduced by dna_sum_slices_accum (deterministic)
//
// Tile 128x128x16, 256 threads = 4 waves as 2x2, each wave 64x64 = 4x4 16x16 accumulators.
// Operands are staged through registers (float4 loads where the contiguous dimension allows,
// zero-filled past the edges) into a double-buffered LDS image [k][m] / [k][n] with a padded
// row, so a k-contiguous operand's transposed write (4 lanes per row, 16 rows per wave) and
// the MFMA's operand read (16 consecutive m or n per k) are both bank-conflict free.
#include "common.h"

namespace dna {
namespace gemm32 {

// LDS row stride 148 floats (148 mod 64 = 20 banks): the k-contiguous transposed store (rows k,
// k+4, k+8, k+12 x 8 columns per 32-lane group) and the operand read (rows k, k+1 x 16 columns)
// both land on distinct banks; 148 % 4 == 0 keeps the mn-contiguous float4 stores aligned
constexpr int BM = 128, BN = 128, BK = 16, NT = 256, LDSW = BM + 20;

struct Args {
  const float* A; long long sam, sak;  // A(m, k) = A[m * sam + k * sak]
  const float* B; long long sbk, sbn;  // B(k, n) = B[k * sbk + n * sbn]
  float* C; long long ldc, slice;      // C[m * ldc + n] (+ blockIdx.z * slice)
  const float* bias;                   // [N] or null
  int M, N, K, kchunk;                 // kchunk: k range per split
  long long saz, sbz;                  // batch steps of A / B (dna_gemm_f32_strided)
  int splits;                          // blockIdx.z = batch * splits + split
};

// Loads of one 128 x 16 operand tile into 8 registers per thread, then into the LDS image
// img[k][LDSW] (row = k). KC: the operand is contiguous along k (x, w rows), else along m/n.
template <bool KC, bool VEC>
struct Tile {
  float r[8];
  __device__ __forceinline__ void load(const float* __restrict__ P, long long s_mn, long long s_k,
                                       int mn0, int MN, int k0, int kend, int t) {
    if constexpr (KC) {
      // 4 threads per row (one float4 each = 16 k), 64 rows per pass, 2 passes
#pragma unroll
      for (int p = 0; p < 2; ++p) {
        const int mn = mn0 + p * 64 + (t >> 2), k = k0 + 4 * (t & 3);
        const float* src = P + (long long)mn * s_mn + (long long)k * s_k;
        if (VEC && mn < MN && k + 3 < kend) {
          const float4 v = *reinterpret_cast<const float4*>(src);
          r[4 * p] = v.x; r[4 * p + 1] = v.y; r[4 * p + 2] = v.z; r[4 * p + 3] = v.w;
        } else {
#pragma unroll
          for (int j = 0; j < 4; ++j)
            r[4 * p + j] = (mn < MN && k + j < kend) ? src[j * s_k] : 0.f;
        }
      }
    } else {
      // 32 threads per k row (one float4 each = 128 mn), 8 rows per pass, 2 passes
#pragma unroll
      for (int p = 0; p < 2; ++p) {
        const int k = k0 + p * 8 + (t >> 5), mn = mn0 + 4 * (t & 31);
        const float* src = P + (long long)k * s_k + (long long)mn * s_mn;
        if (VEC && k < kend && mn + 3 < MN) {
          const float4 v = *reinterpret_cast<const float4*>(src);
          r[4 * p] = v.x; r[4 * p + 1] = v.y; r[4 * p + 2] = v.z; r[4 * p + 3] = v.w;
        } else {
#pragma unroll
          for (int j = 0; j < 4; ++j)
            r[4 * p + j] = (k < kend && mn + j < MN) ? src[j * s_mn] : 0.f;
        }
      }
    }
  }
  __device__ __forceinline__ void store(float* img, int t) const {
    if constexpr (KC) {
#pragma unroll
      for (int p = 0; p < 2; ++p) {
        const int mn = p * 64 + (t >> 2), k = 4 * (t & 3);
#pragma unroll
        for (int j = 0; j < 4; ++j) img[(k + j) * LDSW + mn] = r[4 * p + j];
      }
    } else {
#pragma unroll
      for (int p = 0; p < 2; ++p) {
        const int k = p * 8 + (t >> 5), mn = 4 * (t & 31);
        *reinterpret_cast<float4*>(img + k * LDSW + mn) =
            float4{r[4 * p], r[4 * p + 1], r[4 * p + 2], r[4 * p + 3]};
      }
    }
  }
};

template <bool AKC, bool BKC, bool VA, bool VB>
__global__ __launch_bounds__(NT) void gemm_f32_kernel(Args a) {
  __shared__ float smem[2][2][BK * LDSW];  // [buffer][A, B]
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int m0 = blockIdx.y * BM, n0 = blockIdx.x * BN;
  const int zb = blockIdx.z / a.splits, sp = blockIdx.z - zb * a.splits;
  const float* A = a.A + zb * a.saz;
  const float* B = a.B + zb * a.sbz;
  const int kb = sp * a.kchunk;
  const int ke = min(a.K, kb + a.kchunk);
  const int nk = (ke - kb + BK - 1) / BK;

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  Tile<AKC, VA> ta;
  Tile<BKC, VB> tb;
  if (nk > 0) {
    ta.load(A, a.sam, a.sak, m0, a.M, kb, ke, t);
    tb.load(B, a.sbn, a.sbk, n0, a.N, kb, ke, t);
    ta.store(smem[0][0], t);
    tb.store(smem[0][1], t);
  }
  __syncthreads();
  const int li = lane & 15, lk = lane >> 4;
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) {  // next tile into registers while this one computes
      ta.load(A, a.sam, a.sak, m0, a.M, kb + (kt + 1) * BK, ke, t);
      tb.load(B, a.sbn, a.sbk, n0, a.N, kb + (kt + 1) * BK, ke, t);
    }
    const float* ia = smem[cur][0] + wm * 64 + li;
    const float* ib = smem[cur][1] + wn * 64 + li;
#pragma unroll
    for (int ks = 0; ks < BK / 4; ++ks) {
      const int row = (ks * 4 + lk) * LDSW;
      float fa[4], fb[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) fa[i] = ia[row + i * 16];
#pragma unroll
      for (int j = 0; j < 4; ++j) fb[j] = ib[row + j * 16];
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(fa[i], fb[j], acc[i][j], 0, 0, 0);
    }
    if (kt + 1 < nk) {
      ta.store(smem[cur ^ 1][0], t);
      tb.store(smem[cur ^ 1][1], t);
    }
    __syncthreads();
  }

  // C/D map: lane l holds rows 4*(l>>4) + r of column l&15 of each 16x16 tile
  float* C = a.C + (long long)blockIdx.z * a.slice;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int n = n0 + wn * 64 + j * 16 + li;
    if (n >= a.N) continue;
    const float bv = a.bias ? a.bias[n] : 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + wm * 64 + i * 16 + 4 * lk + r;
        if (m < a.M) C[(long long)m * a.ldc + n] = acc[i][j][r] + bv;
      }
  }
}

template <bool AKC, bool BKC>
int launch(Args a, int splits, hipStream_t st, const char* name, int batch = 1) {
  a.splits = splits;
  // float4 paths need the contiguous stride 1, the other stride (and the batch step) a
  // multiple of 4 and 16-B bases
  const bool va = (AKC ? a.sak == 1 && a.sam % 4 == 0 : a.sam == 1 && a.sak % 4 == 0) &&
                  a.saz % 4 == 0 && ((uintptr_t)a.A & 15) == 0;
  const bool vb = (BKC ? a.sbk == 1 && a.sbn % 4 == 0 : a.sbn == 1 && a.sbk % 4 == 0) &&
                  a.sbz % 4 == 0 && ((uintptr_t)a.B & 15) == 0;
  const dim3 grid((a.N + BN - 1) / BN, (a.M + BM - 1) / BM, batch * splits);
  if (va && vb) hipLaunchKernelGGL((gemm_f32_kernel<AKC, BKC, true, true>), grid, dim3(NT), 0, st, a);
  else if (va) hipLaunchKernelGGL((gemm_f32_kernel<AKC, BKC, true, false>), grid, dim3(NT), 0, st, a);
  else if (vb) hipLaunchKernelGGL((gemm_f32_kernel<AKC, BKC, false, true>), grid, dim3(NT), 0, st, a);
  else hipLaunchKernelGGL((gemm_f32_kernel<AKC, BKC, false, false>), grid, dim3(NT), 0, st, a);
  DNA_LAUNCH_CHECK(name);
  return DNA_OK;
}

}  // namespace gemm32
}  // namespace dna

using namespace dna;
using namespace dna::gemm32;

extern "C" int dna_linear_fwd_f32(const float* x, const float* w, const float* bias, int M, int N,
                                  int K, float* y, void* stream) {
  DNA_CHECK_ARG(M >= 0 && N > 0 && K > 0, "dna_linear_fwd_f32: bad shape");
  if (M == 0) return DNA_OK;
  DNA_CHECK_ARG(x && w && y, "dna_linear_fwd_f32: null pointer");
  Args a{};
  a.A = x; a.sam = K; a.sak = 1;
  a.B = w; a.sbk = 1; a.sbn = K;
  a.C = y; a.ldc = N; a.bias = bias;
  a.M = M; a.N = N; a.K = K; a.kchunk = K;
  return launch<true, true>(a, 1, as_stream(stream), "dna_linear_fwd_f32");
}

extern "C" int dna_linear_dgrad_f32(const float* dy, const float* w, int M, int N, int K, float* dx,
                                    void* stream) {
  DNA_CHECK_ARG(M >= 0 && N > 0 && K > 0, "dna_linear_dgrad_f32: bad shape");
  if (M == 0) return DNA_OK;
  DNA_CHECK_ARG(dy && w && dx, "dna_linear_dgrad_f32: null pointer");
  Args a{};  // dx[M, K] = dy[M, N] . w[N, K]: reduction over N
  a.A = dy; a.sam = N; a.sak = 1;
  a.B = w; a.sbk = K; a.sbn = 1;
  a.C = dx; a.ldc = K;
  a.M = M; a.N = K; a.K = N; a.kchunk = N;
  return launch<true, false>(a, 1, as_stream(stream), "dna_linear_dgrad_f32");
}

extern "C" int dna_linear_wgrad_f32_splits(int T, int N, int K) {
  if (T <= 0 || N <= 0 || K <= 0) return 1;
  const int tiles = ((N + BM - 1) / BM) * ((K + BN - 1) / BN);
  int s = 1;  // enough blocks for the 256 CUs, at least 256 tokens per slice
  while (s < 64 && tiles * s < 512 && T / (2 * s) >= 256) s *= 2;
  return s;
}

extern "C" int dna_linear_wgrad_f32(const float* dy, const float* x, int T, int N, int K,
                                    int splits, float* partials, void* stream) {
  DNA_CHECK_ARG(T >= 0 && N > 0 && K > 0 && splits >= 1, "dna_linear_wgrad_f32: bad shape");
  DNA_CHECK_ARG(partials && (T == 0 || (dy && x)), "dna_linear_wgrad_f32: null pointer");
  DNA_CHECK_ARG((long long)splits * N * K < (1ll << 40), "dna_linear_wgrad_f32: too many partials");
  Args a{};  // dW[N, K] = sum_t dy[t, n] x[t, k]
  a.A = dy; a.sam = 1; a.sak = N;
  a.B = x; a.sbk = K; a.sbn = 1;
  a.C = partials; a.ldc = K; a.slice = (long long)N * K;
  a.M = N; a.N = K; a.K = T;
  a.kchunk = ((T + splits - 1) / splits + BK - 1) / BK * BK;
  if (T == 0) a.kchunk = BK;  // every slice computes zeros
  return launch<false, false>(a, splits, as_stream(stream), "dna_linear_wgrad_f32");
}

// C[z][m][n] = sum_k A(m, k) B(k, n) over a batch with split-K slices (z = batch * splits +
// split; C + z * scz): the fp32 form of dna_gemm_bf16_strided (gemm_strided.hip), for the Mamba
// projections outside autocast. A needs a unit stride along k or m, B along k or n.
extern "C" int dna_gemm_f32_strided(const float* A, long long sam, long long sak, long long saz,
                                    const float* B, long long sbk, long long sbn, long long sbz,
                                    float* C, long long ldc, long long scz, const float* bias_n,
                                    int M, int N, int K, int batch, int splits, void* stream) {
  DNA_CHECK_ARG(M >= 0 && N >= 0 && K >= 0 && batch >= 1 && splits >= 1 && splits <= 65535 / batch,
                "dna_gemm_f32_strided: bad shape");
  if (M == 0 || N == 0) return DNA_OK;
  DNA_CHECK_ARG(A && B && C, "dna_gemm_f32_strided: null pointer");
  DNA_CHECK_ARG(sak == 1 || sam == 1, "dna_gemm_f32_strided: A needs a unit stride along k or m");
  DNA_CHECK_ARG(sbk == 1 || sbn == 1, "dna_gemm_f32_strided: B needs a unit stride along k or n");
  DNA_CHECK_ARG(splits == 1 || !bias_n,
                "dna_gemm_f32_strided: a bias with split-K would be added once per slice");
  Args a{};
  a.A = A; a.sam = sam; a.sak = sak; a.saz = saz;
  a.B = B; a.sbk = sbk; a.sbn = sbn; a.sbz = sbz;
  a.C = C; a.ldc = ldc; a.slice = scz; a.bias = bias_n;
  a.M = M; a.N = N; a.K = K;
  a.kchunk = ((K + splits - 1) / splits + BK - 1) / BK * BK;
  if (a.kchunk == 0) a.kchunk = BK;
  hipStream_t st = as_stream(stream);
  if (sak == 1 && sbk == 1) return launch<true, true>(a, splits, st, "dna_gemm_f32_strided", batch);
  if (sak == 1) return launch<true, false>(a, splits, st, "dna_gemm_f32_strided", batch);
  if (sbk == 1) return launch<false, true>(a, splits, st, "dna_gemm_f32_strided", batch);
  return launch<false, false>(a, splits, st, "dna_gemm_f32_strided", batch);
}
