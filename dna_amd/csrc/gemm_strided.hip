// Strided bf16 GEMM on MFMA (v_mfma_f32_16x16x32_bf16, gfx950) for the skinny projections of
// the Mamba mixer (Caduceus, reference src/models/caduceus/modeling_caduceus.py:88-91 ->
// mamba_ssm Mamba: x_proj, dt_proj and their backward), computed CHANNEL-MAJOR so that no
// operand is ever transposed in memory:
//
//   x_dbl[b, R+2N, L] = Wx[R+2N, E] . x[b, E, L]         (x = the conv output, already [b, E, L];
//                                                          B / C come out as the [b, N, L] rows
//                                                          the scan reads)
//   delta[b, E, L]    = Wdt[E, R]   . x_dbl[b, :R, L]
//   backward: dx = W^T . dy (same form), dW = sum_b dy[b] . x[b]^T (contraction over L: split-K
//   into fp32 slices [batch * splits][M][K], summed by dna_sum_slices_accum, deterministic)
//
// The library GEMMs these replace ran the same products token-major with K = 16 / 48 or with the
// L-long contraction on 16-wide tiles, at 5-20 % of the HBM rate. These shapes are HBM-bound
// (R + 2N = 48, R = 16 against E = 512 and L = 131,072), so the kernel is a plain register-staged
// double-buffered tile loop that keeps every load 16 B wide:
//
//   C[z][m][n] = sum_k A(m, k) B(k, n),  A(m, k) = A[z_b*saz + m*sam + k*sak],
//                                        B(k, n) = B[z_b*sbz + k*sbk + n*sbn]
//   z = blockIdx.z = batch * splits + split; k in [split*kchunk, (split+1)*kchunk) ∩ [0, K)
//
// Tile 128 x 128 x 32, 256 threads = 4 waves (2 x 2), each wave 64 x 64 = 4 x 4 MFMA tiles. An
// operand contiguous along k (AKC / BKC) is staged into a [row][k] image (80-B rows: the
// ds_read_b128 fragment reads are bank-conflict free); one contiguous along m / n into a [k][row]
// image (272-B rows) read with ds_read_b64_tr_b16. The product is issued swapped (C^T = B^T A^T),
// so a lane holds 4 consecutive n of one m; a permlane16 exchange widens that to 8 (16-B stores).
#include "common.h"

namespace dna {
namespace sg {

constexpr int BM = 128, BN = 128, BK = 32, NT = 256;
constexpr int KS = BK + 8;    // [row][k] image row (elements)
constexpr int MS = BM + 8;    // [k][row] image row (elements)
constexpr int IMG = BM * KS;  // elements per image (>= BK * MS)
static_assert(IMG >= BK * MS, "image size");

typedef __attribute__((ext_vector_type(4))) short s16x4;
typedef __attribute__((ext_vector_type(8))) short s16x8;
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

struct Args {
  const bf16* A; long long sam, sak, saz;
  const bf16* B; long long sbk, sbn, sbz;
  void* C; long long ldc, scz;
  const float* bias_m;  // [M] or null
  const float* bias_n;  // [N] or null
  // optional second A operand supplying k in [K1, K) at the same strides (K1 % BK == 0): C = [A | A2] B
  // (the Mamba in_proj data gradient sums its x and z halves, held in separate tensors, in one pass)
  const bf16* A2; int K1;
  int accum;            // C += A B (read-modify-write epilogue) instead of C = A B
  int M, N, K, kchunk, splits;
  int va, vb, vc;       // 16-B operand loads / vector output stores allowed
};

// One 128 x 32 operand tile: 2 chunks of 8 elements per thread, staged through registers.
// KC: contiguous along k (rows = m or n, 4 chunks per row); else contiguous along m / n (rows =
// k, 16 chunks per row).
template <bool KC>
struct Tile {
  bf16x8 r[2];
  __device__ __forceinline__ void load(const bf16* __restrict__ P, long long s_mn, long long s_k,
                                       int mn0, int MN, int k0, int kend, int t, int vec) {
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      const int q = t + p * NT;
      int mn, k;
      if constexpr (KC) {
        mn = mn0 + (q >> 2);
        k = k0 + (q & 3) * 8;
      } else {
        k = k0 + (q >> 4);
        mn = mn0 + (q & 15) * 8;
      }
      const bf16* src = P + (long long)mn * s_mn + (long long)k * s_k;
      const bool full = KC ? (mn < MN && k + 8 <= kend) : (k < kend && mn + 8 <= MN);
      if (vec && full) {
        r[p] = *reinterpret_cast<const bf16x8*>(src);
      } else {
        const long long step = KC ? s_k : s_mn;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const bool ok = KC ? (mn < MN && k + j < kend) : (k < kend && mn + j < MN);
          r[p][j] = ok ? src[j * step] : (bf16)0.f;
        }
      }
    }
  }
  __device__ __forceinline__ void store(bf16* img, int t) const {
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      const int q = t + p * NT;
      if constexpr (KC) *reinterpret_cast<bf16x8*>(img + (q >> 2) * KS + (q & 3) * 8) = r[p];
      else *reinterpret_cast<bf16x8*>(img + (q >> 4) * MS + (q & 15) * 8) = r[p];
    }
  }
};

// MFMA operand: rows base + (lane & 15), k = 8 * (lane >> 4) + 0..7 of the 32-deep tile
template <bool KC>
__device__ __forceinline__ bf16x8 frag(const bf16* img, int base, int lane) {
  if constexpr (KC) {
    return *reinterpret_cast<const bf16x8*>(img + (base + (lane & 15)) * KS + (lane >> 4) * 8);
  } else {
    const int i = lane & 15, g = lane >> 4;
    const bf16* p = img + (8 * g + (i >> 2)) * MS + base + 4 * (i & 3);
    const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(p));
    const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(p + 4 * MS));
    return __builtin_bit_cast(bf16x8, s16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]});
  }
}

template <bool AKC, bool BKC, bool F32>
__global__ __launch_bounds__(NT, 4) void sgemm_kernel(Args a) {
  __shared__ __attribute__((aligned(16))) bf16 smem[2][2][IMG];  // [buffer][A, B]
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int m0 = blockIdx.y * BM, n0 = blockIdx.x * BN;
  const int z = blockIdx.z, zb = z / a.splits, sp = z - zb * a.splits;
  const bf16* A = a.A + zb * a.saz;
  const bf16* B = a.B + zb * a.sbz;
  // A for the k-tile at k0: with A2, tiles past K1 read A2 (rebased so the k index stays global)
  auto a_at = [&](int k0) -> const bf16* {
    if (a.A2 && k0 >= a.K1) return a.A2 + zb * a.saz - (long long)a.K1 * a.sak;
    return A;
  };
  const int kb = sp * a.kchunk;
  const int ke = min(a.K, kb + a.kchunk);
  const int nk = ke > kb ? (ke - kb + BK - 1) / BK : 0;

  f32x4 acc[4][4];  // [m tile][n tile]
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  Tile<AKC> ta;
  Tile<BKC> tb;
  if (nk > 0) {
    ta.load(a_at(kb), a.sam, a.sak, m0, a.M, kb, ke, t, a.va);
    tb.load(B, a.sbn, a.sbk, n0, a.N, kb, ke, t, a.vb);
    ta.store(smem[0][0], t);
    tb.store(smem[0][1], t);
  }
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) {  // the next tile into registers while this one computes
      ta.load(a_at(kb + (kt + 1) * BK), a.sam, a.sak, m0, a.M, kb + (kt + 1) * BK, ke, t, a.va);
      tb.load(B, a.sbn, a.sbk, n0, a.N, kb + (kt + 1) * BK, ke, t, a.vb);
    }
    bf16x8 fa[4], fb[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) fa[i] = frag<AKC>(smem[cur][0], wm * 64 + i * 16, lane);
#pragma unroll
    for (int j = 0; j < 4; ++j) fb[j] = frag<BKC>(smem[cur][1], wn * 64 + j * 16, lane);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[j], fa[i], acc[i][j], 0, 0, 0);
    if (kt + 1 < nk) {
      ta.store(smem[cur ^ 1][0], t);
      tb.store(smem[cur ^ 1][1], t);
    }
    __syncthreads();
  }

  // swapped product: lane holds n = 4 * (lane >> 4) + r of column m = lane & 15 of each tile.
  // Tiles j, j + 1 are exchanged with v_permlane16_swap so a lane holds 8 consecutive n of its m
  // (columns {0, 16, 8, 24}[lane >> 4] .. + 7 of the pair's 32): one 16-B bf16 store (two fp32)
  // per lane, 64 contiguous bytes per row and instruction.
  const long long zc = (long long)z * a.scz;
  const int cg = lane >> 4;
  const int colq = ((cg & 1) << 4) + ((cg & 2) << 2);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int m = m0 + wm * 64 + i * 16 + (lane & 15);
    const float bm = (a.bias_m && m < a.M) ? a.bias_m[m] : 0.f;
#pragma unroll
    for (int jp = 0; jp < 2; ++jp) {
      f32x4 v[2];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int nt = n0 + wn * 64 + (2 * jp + h) * 16 + 4 * cg;  // this tile's 4 columns
        v[h] = acc[i][2 * jp + h];
#pragma unroll
        for (int r = 0; r < 4; ++r) v[h][r] += bm + ((a.bias_n && nt + r < a.N) ? a.bias_n[nt + r] : 0.f);
      }
      const int n = n0 + wn * 64 + jp * 32 + colq;  // first of this lane's 8 columns
      float o[8];
      if constexpr (F32) {
        // whole-vector bit casts (a bit cast of a single vector element lvalue compiled to
        // element 0 for every r: ROCm 7.2 clang, caught by test_strided_gemm_vs_torch)
        typedef __attribute__((ext_vector_type(4))) unsigned u32x4_t;
        const u32x4_t a0 = __builtin_bit_cast(u32x4_t, v[0]), a1 = __builtin_bit_cast(u32x4_t, v[1]);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const auto sw = __builtin_amdgcn_permlane16_swap(a0[r], a1[r], false, false);
          o[r] = __uint_as_float((unsigned)sw[0]);
          o[4 + r] = __uint_as_float((unsigned)sw[1]);
        }
      } else {
        typedef __attribute__((ext_vector_type(2))) unsigned u32x2_t;
        const u32x2_t h0 = __builtin_bit_cast(u32x2_t, bf16x4{(bf16)v[0][0], (bf16)v[0][1], (bf16)v[0][2], (bf16)v[0][3]});
        const u32x2_t h1 = __builtin_bit_cast(u32x2_t, bf16x4{(bf16)v[1][0], (bf16)v[1][1], (bf16)v[1][2], (bf16)v[1][3]});
        const auto sx = __builtin_amdgcn_permlane16_swap(h0[0], h1[0], false, false);
        const auto sy = __builtin_amdgcn_permlane16_swap(h0[1], h1[1], false, false);
        typedef __attribute__((ext_vector_type(4))) unsigned u32x4_t;
        const bf16x8 hb = __builtin_bit_cast(bf16x8, u32x4_t{(unsigned)sx[0], (unsigned)sy[0], (unsigned)sx[1], (unsigned)sy[1]});
#pragma unroll
        for (int e = 0; e < 8; ++e) o[e] = (float)hb[e];  // exact: already bf16 values
        // accumulate: the unrounded sums in the same lane order (the swaps run with every lane
        // active -- inside the bounds branch a swap partner may be masked off)
        float s8[8];
        if (a.accum) {
          const u32x4_t a0 = __builtin_bit_cast(u32x4_t, v[0]), a1 = __builtin_bit_cast(u32x4_t, v[1]);
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const auto sw = __builtin_amdgcn_permlane16_swap(a0[r], a1[r], false, false);
            s8[r] = __uint_as_float((unsigned)sw[0]);
            s8[4 + r] = __uint_as_float((unsigned)sw[1]);
          }
        }
        if (m < a.M && n < a.N) {
          bf16* C = reinterpret_cast<bf16*>(a.C) + zc + (long long)m * a.ldc + n;
          if (a.accum) {  // C = bf16(A B + C): the product is rounded once, after the sum
            if (a.vc && n + 8 <= a.N) {
              const bf16x8 old = *reinterpret_cast<const bf16x8*>(C);
              bf16x8 nw;
#pragma unroll
              for (int e = 0; e < 8; ++e) nw[e] = (bf16)(s8[e] + (float)old[e]);
              *reinterpret_cast<bf16x8*>(C) = nw;
            } else {
#pragma unroll
              for (int e = 0; e < 8; ++e)
                if (n + e < a.N) C[e] = (bf16)(s8[e] + (float)C[e]);
            }
            continue;
          }
          if (a.vc && n + 8 <= a.N) *reinterpret_cast<bf16x8*>(C) = hb;
          else
#pragma unroll
            for (int e = 0; e < 8; ++e)
              if (n + e < a.N) C[e] = hb[e];
        }
        continue;
      }
      if (m < a.M && n < a.N) {
        float* C = reinterpret_cast<float*>(a.C) + zc + (long long)m * a.ldc + n;
        if (a.accum) {
#pragma unroll
          for (int e = 0; e < 8; ++e)
            if (n + e < a.N) o[e] += C[e];
        }
        if (a.vc && n + 8 <= a.N) {
          *reinterpret_cast<f32x4*>(C) = f32x4{o[0], o[1], o[2], o[3]};
          *reinterpret_cast<f32x4*>(C + 4) = f32x4{o[4], o[5], o[6], o[7]};
        } else {
#pragma unroll
          for (int e = 0; e < 8; ++e)
            if (n + e < a.N) C[e] = o[e];
        }
      }
    }
  }
}

}  // namespace sg
}  // namespace dna

using namespace dna;
using namespace dna::sg;

// split count for a long contraction: enough blocks to cover the CUs twice, >= 256 k per slice
extern "C" int dna_gemm_strided_splits(int M, int N, int K, int batch) {
  if (M <= 0 || N <= 0 || K <= 0 || batch <= 0) return 1;
  const long long tiles = (long long)((M + BM - 1) / BM) * ((N + BN - 1) / BN) * batch;
  int s = 1;
  while (s < 256 && tiles * s < 512 && K / (2 * s) >= 256) s *= 2;
  return s;
}

static int strided_impl(const void* A, const void* A2, int K1, long long sam, long long sak,
                        long long saz, const void* B, long long sbk, long long sbn, long long sbz,
                        void* C, long long ldc, long long scz, int out_f32, const float* bias_m,
                        const float* bias_n, int M, int N, int K, int batch, int splits,
                        void* stream);

extern "C" int dna_gemm_bf16_strided(const void* A, long long sam, long long sak, long long saz,
                                     const void* B, long long sbk, long long sbn, long long sbz,
                                     void* C, long long ldc, long long scz, int out_f32,
                                     const float* bias_m, const float* bias_n, int M, int N, int K,
                                     int batch, int splits, void* stream) {
  return strided_impl(A, nullptr, K, sam, sak, saz, B, sbk, sbn, sbz, C, ldc, scz, out_f32, bias_m,
                      bias_n, M, N, K, batch, splits, stream);
}

extern "C" int dna_gemm_bf16_strided_cat(const void* A, const void* A2, int K1, long long sam,
                                         long long sak, long long saz, const void* B, long long sbk,
                                         long long sbn, long long sbz, void* C, long long ldc,
                                         long long scz, int out_f32, const float* bias_m,
                                         const float* bias_n, int M, int N, int K, int batch,
                                         int splits, void* stream) {
  DNA_CHECK_ARG(A2 && K1 > 0 && K1 < K && K1 % BK == 0,
                "dna_gemm_bf16_strided_cat: need A2 and 0 < K1 < K, K1 %% %d == 0 (K1=%d K=%d)", BK,
                K1, K);
  return strided_impl(A, A2, K1, sam, sak, saz, B, sbk, sbn, sbz, C, ldc, scz, out_f32, bias_m,
                      bias_n, M, N, K, batch, splits, stream);
}

static int strided_impl(const void* A, const void* A2, int K1, long long sam, long long sak,
                        long long saz, const void* B, long long sbk, long long sbn, long long sbz,
                        void* C, long long ldc, long long scz, int out_f32, const float* bias_m,
                        const float* bias_n, int M, int N, int K, int batch, int splits,
                        void* stream) {
  DNA_CHECK_ARG(M >= 0 && N >= 0 && K >= 0 && batch >= 1 && splits >= 1 && splits <= 65535 / batch,
                "dna_gemm_bf16_strided: bad shape (M=%d N=%d K=%d batch=%d splits=%d)", M, N, K,
                batch, splits);
  if (M == 0 || N == 0) return DNA_OK;
  DNA_CHECK_ARG(A && B && C, "dna_gemm_bf16_strided: null pointer");
  DNA_CHECK_ARG(sak == 1 || sam == 1, "dna_gemm_bf16_strided: A needs a unit stride along k or m");
  DNA_CHECK_ARG(sbk == 1 || sbn == 1, "dna_gemm_bf16_strided: B needs a unit stride along k or n");
  DNA_CHECK_ARG(splits == 1 || !(bias_m || bias_n),
                "dna_gemm_bf16_strided: a bias with split-K would be added once per slice");
  Args a{};
  a.A = (const bf16*)A; a.sam = sam; a.sak = sak; a.saz = saz;
  a.A2 = (const bf16*)A2; a.K1 = K1;
  a.accum = (out_f32 & 2) != 0;
  DNA_CHECK_ARG(!a.accum || splits == 1, "dna_gemm_bf16_strided: accumulate needs splits == 1");
  out_f32 &= 1;
  a.B = (const bf16*)B; a.sbk = sbk; a.sbn = sbn; a.sbz = sbz;
  a.C = C; a.ldc = ldc; a.scz = scz;
  a.bias_m = bias_m; a.bias_n = bias_n;
  a.M = M; a.N = N; a.K = K; a.splits = splits;
  a.kchunk = ((K + splits - 1) / splits + BK - 1) / BK * BK;
  if (a.kchunk == 0) a.kchunk = BK;  // K == 0: every slice writes zeros (+ bias)
  const bool akc = sak == 1, bkc = sbk == 1;
  // 16-B loads: every row of the non-unit dimension (and the batch step) keeps 8-element alignment
  auto al = [](const void* p, long long s1, long long s2) {
    return ((uintptr_t)p & 15) == 0 && s1 % 8 == 0 && s2 % 8 == 0;
  };
  a.va = al(A, akc ? sam : sak, saz) && (!A2 || al(A2, akc ? sam : sak, saz));
  a.vb = al(B, bkc ? sbn : sbk, sbz);
  a.vc = ((uintptr_t)C & 15) == 0 && ldc % 8 == 0 && scz % 8 == 0;
  const dim3 grid((N + BN - 1) / BN, (M + BM - 1) / BM, batch * splits);
  DNA_CHECK_ARG(grid.y <= 65535, "dna_gemm_bf16_strided: M too large");
  hipStream_t st = as_stream(stream);
#define DNA_SG_LAUNCH(AK, BK_, F)                                                                 \
  hipLaunchKernelGGL((sgemm_kernel<AK, BK_, F>), grid, dim3(NT), 0, st, a)
  if (out_f32) {
    if (akc && bkc) DNA_SG_LAUNCH(true, true, true);
    else if (akc) DNA_SG_LAUNCH(true, false, true);
    else if (bkc) DNA_SG_LAUNCH(false, true, true);
    else DNA_SG_LAUNCH(false, false, true);
  } else {
    if (akc && bkc) DNA_SG_LAUNCH(true, true, false);
    else if (akc) DNA_SG_LAUNCH(true, false, false);
    else if (bkc) DNA_SG_LAUNCH(false, true, false);
    else DNA_SG_LAUNCH(false, false, false);
  }
#undef DNA_SG_LAUNCH
  DNA_LAUNCH_CHECK("dna_gemm_bf16_strided");
  return DNA_OK;
}
