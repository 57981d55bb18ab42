// Dense projections of the DNABERT-2 encoder on MFMA (gfx950), with the GeGLU fused into the
// epilogues of the two GEMMs that touch the MLP intermediate.
//
// Replaces the nn.Linear calls of bert_layers.py (Wqkv :158, attention output dense :214,
// gated_layers :292 + GeGLU :293-296, wo :297, MLM transform :560) and their autograd backward:
//   fwd     y[M,N]  = x[M,K] . W[N,K]^T + b            (A K-major, B K-major)
//   dgrad   dx[M,K] = dy[M,N] . W[N,K]                 (A K-major, B stored [K][N])
//   wgrad   dW[N,K] = dy[M,N]^T . x[M,K]               (both stored [K][M]; split-K partials)
//   GeGLU   g = x . Wg^T + bg  and  a = dropout(gelu(g[:, :F]) * g[:, F:])   in one launch
//   GeGLU'  da = dy . Wo  and  dg = geglu_bwd(da, g)                           in one launch
//
// Tile 256x256x64, 512 threads = 8 waves as 2 (M) x 4 (N), each wave 128x64 outputs = 8x4
// 16x16 MFMA tiles (v_mfma_f32_16x16x32_bf16). The product is issued "swapped" (C^T = B . A^T)
// so a lane holds 4 CONSECUTIVE output columns of one row: 8-/16-byte stores, and the 4-element
// Philox dropout groups of common.h line up with one lane (fused and unfused GeGLU draw
// identical masks). Operands are staged global -> LDS with global_load_lds (16 B/lane, no VGPR
// round trip) into two LDS buffers; the LDS image is lane-linear, so the bank-conflict swizzle
// is applied to the per-lane SOURCE address and undone on the read:
//   K-major tile [256 rows][64 k] (128-B rows): 16-B chunk c of row r sits at c ^ ((r>>1)&7) --
//     a 16-lane ds_read_b128 group (16 consecutive rows, one chunk) hits 8 distinct chunk slots
//     of the two 128-B halves of a bank row: conflict-free.
//   [K][N] tile [64 k][256 cols] (512-B rows, all rows alias the same banks): chunk c of row r
//     sits at c ^ (((r&3)<<1) | (((r>>3)&1)<<3)) -- a 32-lane half of a ds_read_b64_tr_b16
//     (rows r0..r0+3 and r0+8..r0+11, 32 B each) covers all 16 chunk slots: conflict-free.
// Block order: bijective XCD remap (blocks sharing an L2 get consecutive tile ids), then
// groups of GM row-tiles swept column-fastest so a group's A panels stay L2-resident while the
// weight (<= 9.4 MB, MALL-resident) streams.
#include <stdlib.h>

#include "common.h"

namespace dna {
namespace gemm {

constexpr int BM = 256, BN = 256, BK = 64, NTHR = 512;
constexpr int HALF = 128 * BK * 2;      // bytes of one half-tile image (16 KB)
constexpr int LDS_BYTES = 8 * HALF;     // 2 buffers x {A0, A1, B0, B1} = 128 KB

enum Epi { EPI_BF16 = 0, EPI_F32 = 1, EPI_GEGLU = 2, EPI_GEGLU_BWD = 3 };

typedef __attribute__((address_space(3))) void lds_t;
typedef __attribute__((ext_vector_type(4))) short s16x4;

__device__ __forceinline__ int kswz(int r) { return (r >> 1) & 7; }
__device__ __forceinline__ int nswz(int r) { return ((r & 3) << 1) | (((r >> 3) & 1) << 3); }

__device__ __forceinline__ void glds16(const void* src, char* lds_base) {
  __builtin_amdgcn_global_load_lds(src, (lds_t*)lds_base, 16, 0, 0);
}

// Half-tiles. The wave grid is 2 (wr) x 4 (wc); a wave's 128x64 outputs are four quadrants
// (mq, nq) of 64x32 at tile rows mq*128 + wr*64 + [0,64) and tile columns nq*128 + wc*32 + [0,32).
// Half-tile A_mq is the contiguous row slab mq*128 + [0,128) (image row lr <-> tile row
// mq*128 + lr), B_nq the contiguous column slab nq*128 + [0,128): every staged piece is a whole
// 128-B (or 256-B) line segment, never half a line shared with the other half-tile.
__device__ __forceinline__ int a_row(int lr, int mq) { return mq * 128 + lr; }
__device__ __forceinline__ int b_col(int lr, int nq) { return nq * 128 + lr; }

// K-major half-tile (128 rows x 64 k, 128-B rows): 2 passes of 8 waves x 8 rows.
// grow_of(lr) gives the global row of image row lr.
template <typename RowOf>
__device__ __forceinline__ void stage_k(const bf16* __restrict__ P, int ld, int k0, char* img,
                                        int wave, int lane, RowOf grow_of) {
#pragma unroll
  for (int p = 0; p < 2; ++p) {
    const int lr = p * 64 + wave * 8 + (lane >> 3);
    const int c = (lane & 7) ^ kswz(lr);
    glds16(P + (size_t)grow_of(lr) * ld + k0 + c * 8, img + (p * 64 + wave * 8) * 128);
  }
}

// [K][N]-stored half-tile (64 k rows x 128 columns, 256-B rows): 2 passes of 8 waves x 4 rows.
// gcol_of(lc) gives the global column of image column lc (a multiple of 8).
template <typename ColOf>
__device__ __forceinline__ void stage_n(const bf16* __restrict__ P, int ld, int k0, char* img,
                                        int wave, int lane, ColOf gcol_of) {
#pragma unroll
  for (int p = 0; p < 2; ++p) {
    const int r = p * 32 + wave * 4 + (lane >> 4);
    const int c = (lane & 15) ^ nswz(r);
    glds16(P + (size_t)(k0 + r) * ld + gcol_of(c * 8), img + (p * 32 + wave * 4) * 256);
  }
}

__device__ __forceinline__ bf16x8 read_k(const char* img, int lr, int chunk) {
  return *reinterpret_cast<const bf16x8*>(img + lr * 128 + ((chunk ^ kswz(lr)) << 4));
}

__device__ __forceinline__ bf16x4 tr_read(const char* p) {
  s16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(p));
  return __builtin_bit_cast(bf16x4, v);
}

// MFMA operand (8 consecutive k of one column) from a [64 k][128] image: two transposed reads.
// lane l: image column c0 + (l&15), k = kbase + 8*(l>>4) + j
__device__ __forceinline__ bf16x8 read_n(const char* img, int kbase, int c0, int lane) {
  const int i = lane & 15, kq = lane >> 4;
  const int r = kbase + kq * 8 + (i >> 2);
  const int col = c0 + 4 * (i & 3);
  const int off = (((col >> 3) ^ nswz(r)) << 4) + (col & 7) * 2;  // nswz(r) == nswz(r+4)
  bf16x4 lo = tr_read(img + r * 256 + off);
  bf16x4 hi = tr_read(img + (r + 4) * 256 + off);
  return bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
}

__device__ __forceinline__ f32x4 mfma(bf16x8 a, bf16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

struct Args {
  const bf16* A; int lda;     // fwd/dgrad: [M][K]; wgrad: [K][M]
  const bf16* B; int ldb;     // fwd: [N][K]; dgrad/wgrad: [K][N]
  void* C; int ldc;           // output (bf16 or fp32 partial slices [split][M][ldc])
  const float* bias;          // [N] (fwd) / [2F] (GeGLU), may be null
  const bf16* g;              // GeGLU bwd: saved g [M][2F]
  bf16* aux;                  // GeGLU fwd: a [M][F];  GeGLU bwd: dg [M][2F]
  int M, N, K;                // N = output columns (GeGLU fwd: F)
  int ksplit;                 // k range per blockIdx.y
  int tilesM, tilesN, GM;
  int F;
  float p; uint32_t th; float ks; uint64_t seed, off;
};

__device__ __forceinline__ void tile_of(const Args& a, int& mt, int& nt) {
  const int nwg = gridDim.x, bid = blockIdx.x;
  const int xcd = bid & 7, q = nwg >> 3, rr = nwg & 7;
  const int L = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + (bid >> 3);
  const int width = a.GM * a.tilesN;
  const int grp = L / width, first = grp * a.GM;
  const int gsz = min(a.tilesM - first, a.GM);
  const int w = L - grp * width;
  mt = first + w % gsz;
  nt = w / gsz;
}

__device__ __forceinline__ void store_bf16x4(bf16* p, float v0, float v1, float v2, float v3) {
  *reinterpret_cast<bf16x4*>(p) = bf16x4{(bf16)v0, (bf16)v1, (bf16)v2, (bf16)v3};
}

#define DNA_BARRIER()                         \
  do {                                        \
    __builtin_amdgcn_sched_barrier(0);        \
    __builtin_amdgcn_s_barrier();             \
    asm volatile("" ::: "memory");            \
    __builtin_amdgcn_sched_barrier(0);        \
  } while (0)

// Main loop (per K-tile t, 4 phases; quadrant order (0,0) (0,1) (1,1) (1,0)):
//   phase  reads (LDS -> VGPR)        stages (global -> LDS)   wait
//   0      A_0(t), B_0(t)             B_1(t+1)                 vmcnt(8)
//   1      B_1(t)                     A_1(t+1)                 vmcnt(8)
//   2      A_1(t)                     A_0(t+2)                 vmcnt(8)
//   3      -- (B_0 still in VGPRs)    B_0(t+2)                 vmcnt(8)
// Each phase = [stage; wait; ds_reads; lgkmcnt(0); barrier] [16 MFMA; barrier]. Every half-tile
// is restaged >= 2 phases after its last read (WAR), and the vmcnt(8) of phase p (4 half-tiles
// = 8 glds/lane left in flight) retires the half-tile phase p+1 reads, behind at least one
// barrier for both wave groups (RAW). Waves 4-7 run one barrier behind waves 0-3, so on every
// SIMD one wave's MFMA cluster overlaps its partner's reads and DMA issue. Stages past the last
// K-tile re-load the last tile into a buffer nobody reads again (keeps vmcnt uniform).
template <bool AK, bool BKM, int EPI>
__global__ __launch_bounds__(NTHR) void gemm_kernel(Args a) {
  __shared__ __attribute__((aligned(1024))) char smem[LDS_BYTES];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 2, wc = wave & 3;
  int mt, nt;
  tile_of(a, mt, nt);
  const int m0 = mt * BM;
  const int n0 = (EPI == EPI_GEGLU ? nt * (BN / 2) : nt * BN);
  const int kbeg = blockIdx.y * a.ksplit;
  const int ntiles = a.ksplit / BK;

  // half-tile image h of buffer b: A_0, A_1, B_0, B_1
  auto img = [&](int b, int h) { return smem + (b * 4 + h) * HALF; };

  auto stageA = [&](int t, int mq) {
    const int k0 = kbeg + min(t, ntiles - 1) * BK;
    char* d = img(t & 1, mq);
    if constexpr (AK) {
      stage_k(a.A, a.lda, k0, d, wave, lane,
              [&](int lr) { return min(m0 + a_row(lr, mq), a.M - 1); });
    } else {
      stage_n(a.A, a.lda, k0, d, wave, lane,
              [&](int lc) { return min(m0 + a_row(lc, mq), a.M - 8); });
    }
  };
  auto stageB = [&](int t, int nq) {
    const int k0 = kbeg + min(t, ntiles - 1) * BK;
    char* d = img(t & 1, 2 + nq);
    if constexpr (BKM) {
      if constexpr (EPI == EPI_GEGLU)
        stage_k(a.B, a.ldb, k0, d, wave, lane, [&](int lr) { return nq * a.F + n0 + lr; });
      else
        stage_k(a.B, a.ldb, k0, d, wave, lane,
                [&](int lr) { return min(n0 + b_col(lr, nq), a.N - 1); });
    } else {
      stage_n(a.B, a.ldb, k0, d, wave, lane,
              [&](int lc) { return min(n0 + b_col(lc, nq), a.N - 8); });
    }
  };

  f32x4 acc[2][2][4][2];  // [mq][nq][i][j]
#pragma unroll
  for (int q = 0; q < 2; ++q)
#pragma unroll
    for (int r = 0; r < 2; ++r)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[q][r][i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  bf16x8 af[4][2], bf0[2][2], bf1[2][2];  // [subtile][k-step]

  auto readA = [&](int t, int mq) {
    const char* im = img(t & 1, mq);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        if constexpr (AK) af[i][kk] = read_k(im, wr * 64 + i * 16 + (lane & 15), kk * 4 + (lane >> 4));
        else af[i][kk] = read_n(im, kk * 32, wr * 64 + i * 16, lane);
      }
  };
  auto readB = [&](int t, int nq, bf16x8 (&bf)[2][2]) {
    const char* im = img(t & 1, 2 + nq);
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        if constexpr (BKM) bf[j][kk] = read_k(im, wc * 32 + j * 16 + (lane & 15), kk * 4 + (lane >> 4));
        else bf[j][kk] = read_n(im, kk * 32, wc * 32 + j * 16, lane);
      }
  };
  auto mma = [&](int mq, int nq, const bf16x8 (&bf)[2][2]) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[mq][nq][i][j] = mfma(bf[j][kk], af[i][kk], acc[mq][nq][i][j]);
    __builtin_amdgcn_s_setprio(0);
  };

  // prologue: slots of virtual tiles -2 and -1
  stageA(0, 0);
  stageB(0, 0);
  stageB(0, 1);
  stageA(0, 1);
  stageA(1, 0);
  stageB(1, 0);
  asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  DNA_BARRIER();
  if (wr == 1) DNA_BARRIER();  // stagger: waves 4-7 one barrier behind

  for (int t = 0; t < ntiles; ++t) {
    // phase 0: quadrant (0,0)
    stageB(t + 1, 1);
    asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    readA(t, 0);
    readB(t, 0, bf0);
    DNA_BARRIER();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    mma(0, 0, bf0);
    DNA_BARRIER();
    // phase 1: quadrant (0,1)
    stageA(t + 1, 1);
    asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    readB(t, 1, bf1);
    DNA_BARRIER();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    mma(0, 1, bf1);
    DNA_BARRIER();
    // phase 2: quadrant (1,1)
    stageA(t + 2, 0);
    asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    readA(t, 1);
    DNA_BARRIER();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    mma(1, 1, bf1);
    DNA_BARRIER();
    // phase 3: quadrant (1,0)
    stageB(t + 2, 0);
    asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    DNA_BARRIER();
    mma(1, 0, bf0);
    DNA_BARRIER();
  }
  if (wr == 0) DNA_BARRIER();  // re-align the two wave groups
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");

  // ------------------------------------------------------------------ epilogue
  // acc[mq][nq][i][j] lane holds C[m][n .. n+3]:
  //   m = m0 + mq*128 + wr*64 + i*16 + (lane&15),  n = n0 + nq*128 + wc*32 + j*16 + 4*(lane>>4)
  const int cq = 4 * (lane >> 4);
  if constexpr (EPI == EPI_BF16 || EPI == EPI_F32) {
#pragma unroll
    for (int mq = 0; mq < 2; ++mq)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int m = m0 + mq * 128 + wr * 64 + i * 16 + (lane & 15);
        if (m >= a.M) continue;
#pragma unroll
        for (int nq = 0; nq < 2; ++nq)
#pragma unroll
          for (int j = 0; j < 2; ++j) {
            const int n = n0 + nq * 128 + wc * 32 + j * 16 + cq;
            if (n >= a.N) continue;
            f32x4 v = acc[mq][nq][i][j];
            if (a.bias) v += *reinterpret_cast<const f32x4*>(a.bias + n);
            if constexpr (EPI == EPI_BF16) {
              store_bf16x4(reinterpret_cast<bf16*>(a.C) + (size_t)m * a.ldc + n, v[0], v[1], v[2], v[3]);
            } else {
              float* Cf = reinterpret_cast<float*>(a.C) + (size_t)blockIdx.y * a.M * a.ldc;
              *reinterpret_cast<f32x4*>(Cf + (size_t)m * a.ldc + n) = v;
            }
          }
      }
  } else if constexpr (EPI == EPI_GEGLU) {
    // quadrant column nq=0 holds g1 columns, nq=1 the matching g2 columns
    bf16* g = reinterpret_cast<bf16*>(a.C);
#pragma unroll
    for (int mq = 0; mq < 2; ++mq)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int m = m0 + mq * 128 + wr * 64 + i * 16 + (lane & 15);
        if (m >= a.M) continue;
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const int c = n0 + wc * 32 + j * 16 + cq;  // a column (0..F)
          f32x4 v1 = acc[mq][0][i][j], v2 = acc[mq][1][i][j];
          if (a.bias) {
            v1 += *reinterpret_cast<const f32x4*>(a.bias + c);
            v2 += *reinterpret_cast<const f32x4*>(a.bias + a.F + c);
          }
          const bf16x4 h1 = bf16x4{(bf16)v1[0], (bf16)v1[1], (bf16)v1[2], (bf16)v1[3]};
          const bf16x4 h2 = bf16x4{(bf16)v2[0], (bf16)v2[1], (bf16)v2[2], (bf16)v2[3]};
          *reinterpret_cast<bf16x4*>(g + (size_t)m * 2 * a.F + c) = h1;
          *reinterpret_cast<bf16x4*>(g + (size_t)m * 2 * a.F + a.F + c) = h2;
          const size_t e = (size_t)m * a.F + c;
          // c % 4 == 0: this lane's 4 columns are one half of a keep8 group
          const uint32_t keep = a.p > 0.f ? (dropout_keep8(a.seed, a.off, e >> 3, a.th) >> (e & 4)) & 0xFu : 0xFu;
          float o[4];
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const float x = gelu_erf((float)h1[q]) * (float)h2[q];
            o[q] = a.p > 0.f ? (((keep >> q) & 1) ? x * a.ks : 0.f) : x;
          }
          store_bf16x4(a.aux + e, o[0], o[1], o[2], o[3]);
        }
      }
  } else {  // EPI_GEGLU_BWD
    // da tile -> LDS (bf16, [256][256], 16-B chunks XOR-swizzled by row&15), then row-contiguous
    // 8-element chunks per thread: 16-B loads of g, 16-B stores of dg, one keep8 Philox draw.
    __syncthreads();
    char* T = smem;
#pragma unroll
    for (int mq = 0; mq < 2; ++mq)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int r = mq * 128 + wr * 64 + i * 16 + (lane & 15);
#pragma unroll
        for (int nq = 0; nq < 2; ++nq)
#pragma unroll
          for (int j = 0; j < 2; ++j) {
            const int col = nq * 128 + wc * 32 + j * 16 + cq;
            const f32x4 v = acc[mq][nq][i][j];
            *reinterpret_cast<bf16x4*>(T + r * 512 + (((col >> 3) ^ (r & 15)) << 4) + (col & 7) * 2) =
                bf16x4{(bf16)v[0], (bf16)v[1], (bf16)v[2], (bf16)v[3]};
          }
      }
    __syncthreads();
    for (int it = 0; it < 16; ++it) {
      const int idx = it * NTHR + tid;
      const int r = idx >> 5, c = idx & 31;
      const int m = m0 + r, n = n0 + c * 8;
      if (m >= a.M || n >= a.F) continue;
      const bf16x8 d = *reinterpret_cast<const bf16x8*>(T + r * 512 + ((c ^ (r & 15)) << 4));
      const bf16* grow = a.g + (size_t)m * 2 * a.F;
      const bf16x8 g1 = *reinterpret_cast<const bf16x8*>(grow + n);
      const bf16x8 g2 = *reinterpret_cast<const bf16x8*>(grow + a.F + n);
      const size_t e = (size_t)m * a.F + n;
      uint32_t keep = 0xFFu;
      if (a.p > 0.f) keep = dropout_keep8(a.seed, a.off, e >> 3, a.th);
      bf16x8 o1, o2;
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        float dd = (float)d[q];
        if (a.p > 0.f) dd = ((keep >> q) & 1) ? dd * a.ks : 0.f;
        const float x = (float)g1[q];
        float ge, dge;
        gelu_erf_and_grad(x, ge, dge);
        o1[q] = (bf16)(dd * (float)g2[q] * dge);
        o2[q] = (bf16)(dd * ge);
      }
      bf16* dg = a.aux + (size_t)m * 2 * a.F;
      *reinterpret_cast<bf16x8*>(dg + n) = o1;
      *reinterpret_cast<bf16x8*>(dg + a.F + n) = o2;
    }
  }
}

template <bool AK, bool BKM, int EPI>
int launch(Args& a, int splits, hipStream_t s, const char* name) {
  a.tilesM = (a.M + BM - 1) / BM;
  const int nper = (EPI == EPI_GEGLU ? BN / 2 : BN);
  a.tilesN = (a.N + nper - 1) / nper;
  if (const char* e = getenv("DNA_GEMM_GM")) a.GM = atoi(e);
  if (a.GM <= 0) a.GM = 4;
  dim3 grid(a.tilesM * a.tilesN, splits);
  hipLaunchKernelGGL((gemm_kernel<AK, BKM, EPI>), grid, dim3(NTHR), 0, s, a);
  DNA_LAUNCH_CHECK(name);
  return DNA_OK;
}

inline Args base_args() {
  Args a{};
  a.GM = 4;
  return a;
}

}  // namespace gemm
}  // namespace dna

using namespace dna;
using namespace dna::gemm;

extern "C" int dna_linear_fwd(const void* x, const void* w, const float* bias, int M, int N, int K,
                              void* y, void* stream) {
  DNA_CHECK_ARG(x && w && y, "dna_linear_fwd: null pointer");
  DNA_CHECK_ARG(M >= 0 && N > 0 && K > 0, "dna_linear_fwd: bad shape");
  DNA_CHECK_ARG(K % BK == 0 && N % 8 == 0, "dna_linear_fwd: K %% 64 and N %% 8 required (K=%d N=%d)", K, N);
  if (M == 0) return DNA_OK;
  Args a = base_args();
  a.A = (const bf16*)x; a.lda = K;
  a.B = (const bf16*)w; a.ldb = K;
  a.C = y; a.ldc = N; a.bias = bias;
  a.M = M; a.N = N; a.K = K; a.ksplit = K;
  return launch<true, true, EPI_BF16>(a, 1, as_stream(stream), "dna_linear_fwd");
}

extern "C" int dna_linear_dgrad(const void* dy, const void* w, int M, int N, int K, void* dx,
                                void* stream) {
  DNA_CHECK_ARG(dy && w && dx, "dna_linear_dgrad: null pointer");
  DNA_CHECK_ARG(M >= 0 && N > 0 && K > 0, "dna_linear_dgrad: bad shape");
  DNA_CHECK_ARG(N % BK == 0 && K % 8 == 0, "dna_linear_dgrad: N %% 64 and K %% 8 required (N=%d K=%d)", N, K);
  if (M == 0) return DNA_OK;
  Args a = base_args();
  a.A = (const bf16*)dy; a.lda = N;
  a.B = (const bf16*)w; a.ldb = K;
  a.C = dx; a.ldc = K;
  a.M = M; a.N = K; a.K = N; a.ksplit = N;
  return launch<true, false, EPI_BF16>(a, 1, as_stream(stream), "dna_linear_dgrad");
}

extern "C" int dna_linear_wgrad(const void* dy, const void* x, int M, int N, int K, int splits,
                                float* partials, void* stream) {
  DNA_CHECK_ARG(dy && x && partials, "dna_linear_wgrad: null pointer");
  DNA_CHECK_ARG(M > 0 && N > 0 && K > 0 && splits > 0, "dna_linear_wgrad: bad shape");
  DNA_CHECK_ARG(M % (splits * BK) == 0, "dna_linear_wgrad: rows %d not a multiple of 64*splits", M);
  DNA_CHECK_ARG(N % 8 == 0 && K % 8 == 0, "dna_linear_wgrad: N, K %% 8 required");
  Args a = base_args();
  a.A = (const bf16*)dy; a.lda = N;   // A[k=token][m=out feature]
  a.B = (const bf16*)x; a.ldb = K;    // B[k=token][n=in feature]
  a.C = partials; a.ldc = K;
  a.M = N; a.N = K; a.K = M; a.ksplit = M / splits;
  a.GM = 2;
  return launch<false, false, EPI_F32>(a, splits, as_stream(stream), "dna_linear_wgrad");
}

extern "C" int dna_geglu_linear_fwd(const void* x, const void* w, const float* bias, int M, int F,
                                    int K, float p_drop, uint64_t seed, uint64_t offset, void* g,
                                    void* out, void* stream) {
  DNA_CHECK_ARG(x && w && g && out, "dna_geglu_linear_fwd: null pointer");
  DNA_CHECK_ARG(M >= 0 && K % BK == 0 && F % (BN / 2) == 0,
                "dna_geglu_linear_fwd: K %% 64 and F %% 128 required (K=%d F=%d)", K, F);
  DNA_CHECK_ARG(p_drop >= 0.f && p_drop < 1.f, "dna_geglu_linear_fwd: bad p");
  if (M == 0) return DNA_OK;
  Args a = base_args();
  a.A = (const bf16*)x; a.lda = K;
  a.B = (const bf16*)w; a.ldb = K;
  a.C = g; a.ldc = 2 * F; a.bias = bias; a.aux = (bf16*)out;
  a.M = M; a.N = F; a.K = K; a.ksplit = K; a.F = F;
  a.p = p_drop; a.th = dropout_threshold16(p_drop); a.ks = 1.f / (1.f - p_drop);
  a.seed = seed; a.off = offset;
  return launch<true, true, EPI_GEGLU>(a, 1, as_stream(stream), "dna_geglu_linear_fwd");
}

extern "C" int dna_geglu_linear_dgrad(const void* dy, const void* w, const void* g, int M, int F,
                                      int N, float p_drop, uint64_t seed, uint64_t offset,
                                      void* dg, void* stream) {
  DNA_CHECK_ARG(dy && w && g && dg, "dna_geglu_linear_dgrad: null pointer");
  DNA_CHECK_ARG(M >= 0 && N % BK == 0 && F % 8 == 0,
                "dna_geglu_linear_dgrad: hidden %% 64 and F %% 8 required (N=%d F=%d)", N, F);
  if (M == 0) return DNA_OK;
  Args a = base_args();
  a.A = (const bf16*)dy; a.lda = N;
  a.B = (const bf16*)w; a.ldb = F;
  a.C = nullptr; a.ldc = F; a.g = (const bf16*)g; a.aux = (bf16*)dg;
  a.M = M; a.N = F; a.K = N; a.ksplit = N; a.F = F;
  a.p = p_drop; a.th = dropout_threshold16(p_drop); a.ks = 1.f / (1.f - p_drop);
  a.seed = seed; a.off = offset;
  return launch<true, false, EPI_GEGLU_BWD>(a, 1, as_stream(stream), "dna_geglu_linear_dgrad");
}
