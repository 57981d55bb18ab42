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

#include <type_traits>

#include "common.h"

namespace dna {
namespace gemm {

constexpr int BM = 256, BN = 256, BK = 64, NTHR = 512;
constexpr int HALF = 128 * BK * 2;      // bytes of one half-tile image (16 KB)
constexpr int LDS_BYTES = 8 * HALF;     // 2 buffers x {A0, A1, B0, B1} = 128 KB

// EPI_BF16_GELU: the bf16 output h plus a = gelu_tanh(h) into aux (the HyenaDNA Mlp's fc1 + act)
enum Epi { EPI_BF16 = 0, EPI_F32 = 1, EPI_GEGLU = 2, EPI_GEGLU_BWD = 3, EPI_GELU_BWD = 4,
           EPI_BF16_GELU = 5 };

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

// ds_read_b64_tr_b16 as inline asm: hipcc (ROCm 7.2) treats the builtin as a read that may alias
// any in-flight LDS-DMA stage and puts an `s_waitcnt vmcnt(0)` in front of it -- which drained
// the whole staging pipeline at every phase of the [K][N]-operand kernels (the token-major weight
// gradient waited on memory 77 % of its cycles). The asm form is invisible to that analysis; the
// kernels order it themselves: every read sits before the phase's barrier and its explicit
// `s_waitcnt lgkmcnt(0)` + sched_barrier, and the staged buffer it reads was retired by the
// counted vmcnt wait of an earlier phase.
__device__ __forceinline__ bf16x4 tr_read(const char* p) {
  s16x4 v;
  const uint32_t a = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char*)(p);
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(v) : "v"(a) : "memory");
  return __builtin_bit_cast(bf16x4, v);
}

// tr_read with the row offset as an instruction immediate: the address VGPR is per-lane and
// per-fragment (computed once per read group), the k-block / row-half steps are immediates
template <int OFF>
__device__ __forceinline__ bf16x4 tr_read_imm(uint32_t addr) {
  s16x4 v;
  asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(v) : "v"(addr), "i"(OFF) : "memory");
  return __builtin_bit_cast(bf16x4, v);
}
__device__ __forceinline__ uint32_t lds_addr(const char* p) {
  return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char*)(p);
}
// lane part of read_n's address for k-block 0, row half 0 of the fragment whose columns start
// at c0: rows k and k + 4 (the other row half) and k + 32 (k-block 1) share the chunk swizzle
__device__ __forceinline__ uint32_t read_n_lane_off(int c0, int lane) {
  const int i = lane & 15, kq = lane >> 4;
  const int r = kq * 8 + (i >> 2);
  const int col = c0 + 4 * (i & 3);
  return (uint32_t)(r * 256 + ((((col >> 3) ^ nswz(r)) << 4) + (col & 7) * 2));
}
// both k-blocks of one fragment: {kk = 0, kk = 1}
__device__ __forceinline__ void read_n2(uint32_t addr, bf16x8& k0, bf16x8& k1) {
  const bf16x4 a = tr_read_imm<0>(addr), b = tr_read_imm<1024>(addr);
  const bf16x4 c = tr_read_imm<8192>(addr), d = tr_read_imm<9216>(addr);
  k0 = bf16x8{a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
  k1 = bf16x8{c[0], c[1], c[2], c[3], d[0], d[1], d[2], d[3]};
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
  int rot;                    // persistent kernel: rotate each block's K order (store spreading)
  int dbg;                    // diagnostics (DNA_GEMM_DBG): 1 = stores dropped (OOB), 2 = no stores,
                              // 4 = output stores with the sc0 cache policy (A/B)
  int nt;                     // persistent kernel: non-temporal output stores (DNA_GEMM_NT, default 0)
  int order;                  // persistent kernel unit order: 0 = round-robin over the grid (XCD-
                              // remapped), 1 = XCD-major (each XCD sweeps one contiguous unit range)
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


// ---- branch-free epilogue I/O: raw buffer ops on a resource spanning one tile's rows
typedef __attribute__((ext_vector_type(2))) unsigned u32x2;
typedef __attribute__((ext_vector_type(4))) unsigned u32x4;
constexpr uint32_t kOOB = 0x7FFFFFF0u;  // past any tile resource: the access is dropped / reads 0

__device__ __forceinline__ __amdgpu_buffer_rsrc_t out_rsrc(const void* base, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)bytes, 0x00020000);
}
__device__ __forceinline__ void store_b64(__amdgpu_buffer_rsrc_t r, uint32_t off, f32x4 v) {
  const bf16x4 h = bf16x4{(bf16)v[0], (bf16)v[1], (bf16)v[2], (bf16)v[3]};
  __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, h), r, off, 0, 0);
}
__device__ __forceinline__ void store_b64h(__amdgpu_buffer_rsrc_t r, uint32_t off, bf16x4 h) {
  __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, h), r, off, 0, 0);
}
__device__ __forceinline__ void store_b128(__amdgpu_buffer_rsrc_t r, uint32_t off, f32x4 v) {
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), r, off, 0, 0);
}
__device__ __forceinline__ void store_b128h(__amdgpu_buffer_rsrc_t r, uint32_t off, bf16x8 h) {
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, h), r, off, 0, 0);
}
__device__ __forceinline__ bf16x8 load_b128h(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  return __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0));
}
__device__ float g_zero4[4];  // stands in for a missing bias (zero-initialised device memory)
// 4 bias columns starting at n (n % 4 == 0), zero past `limit` or without a bias; the load is
// unconditional (pointer select), so no branch holds a load
__device__ __forceinline__ f32x4 bias4(const float* bias, int n, int limit) {
  const float* p = (bias != nullptr && n < limit) ? bias + n : g_zero4;
  return *reinterpret_cast<const f32x4*>(p);
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
  // Epilogues: every store is a raw buffer store through a resource covering exactly this tile's
  // rows, and out-of-range lanes get an offset past its end (the hardware drops them), so no store
  // sits under a branch; every global load (bias columns, the saved GeGLU input) is issued
  // unconditionally ahead of the stores. A load under a divergent branch between two stores made
  // the compiler wait `vmcnt(0)` before every store (32 serial memory round trips per tile).
  const int cq = 4 * (lane >> 4);
  const int rows = min(a.M - m0, BM);
  if constexpr (EPI == EPI_BF16 || EPI == EPI_F32) {
    constexpr int ES = EPI == EPI_BF16 ? 2 : 4;
#pragma unroll
    for (int nq = 0; nq < 2; ++nq)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int n = n0 + nq * 128 + wc * 32 + j * 16 + cq;
        const f32x4 bv = bias4(a.bias, n, a.N);
#pragma unroll
        for (int mq = 0; mq < 2; ++mq)
#pragma unroll
          for (int i = 0; i < 4; ++i) acc[mq][nq][i][j] += bv;
      }
    char* base = reinterpret_cast<char*>(a.C) +
                 ((EPI == EPI_F32 ? (size_t)blockIdx.y * a.M * a.ldc : 0) + (size_t)m0 * a.ldc) * ES;
    const auto rs = out_rsrc(base, (uint32_t)((size_t)rows * a.ldc * ES));
#pragma unroll
    for (int mq = 0; mq < 2; ++mq)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int r = mq * 128 + wr * 64 + i * 16 + (lane & 15);
#pragma unroll
        for (int nq = 0; nq < 2; ++nq)
#pragma unroll
          for (int j = 0; j < 2; ++j) {
            const int n = n0 + nq * 128 + wc * 32 + j * 16 + cq;
            const uint32_t off = n < a.N ? (uint32_t)((r * a.ldc + n) * ES) : kOOB;
            const f32x4 v = acc[mq][nq][i][j];
            if constexpr (EPI == EPI_BF16) store_b64(rs, off, v);
            else store_b128(rs, off, v);
          }
      }
  } else if constexpr (EPI == EPI_GEGLU) {
    // quadrant column nq=0 holds g1 columns, nq=1 the matching g2 columns
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int c = n0 + wc * 32 + j * 16 + cq;
      const f32x4 b1 = bias4(a.bias, c, a.F), b2 = bias4(a.bias ? a.bias + a.F : nullptr, c, a.F);
#pragma unroll
      for (int mq = 0; mq < 2; ++mq)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          acc[mq][0][i][j] += b1;
          acc[mq][1][i][j] += b2;
        }
    }
    const auto rg = out_rsrc(reinterpret_cast<bf16*>(a.C) + (size_t)m0 * 2 * a.F,
                             (uint32_t)((size_t)rows * 2 * a.F * 2));
    const auto ra = out_rsrc(a.aux + (size_t)m0 * a.F, (uint32_t)((size_t)rows * a.F * 2));
#pragma unroll
    for (int mq = 0; mq < 2; ++mq)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int r = mq * 128 + wr * 64 + i * 16 + (lane & 15);
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const int c = n0 + wc * 32 + j * 16 + cq;  // a column (0..F)
          const f32x4 v1 = acc[mq][0][i][j], v2 = acc[mq][1][i][j];
          const bf16x4 h1 = bf16x4{(bf16)v1[0], (bf16)v1[1], (bf16)v1[2], (bf16)v1[3]};
          const bf16x4 h2 = bf16x4{(bf16)v2[0], (bf16)v2[1], (bf16)v2[2], (bf16)v2[3]};
          const uint32_t og = (uint32_t)((r * 2 * a.F + c) * 2);
          const size_t e = (size_t)(m0 + r) * a.F + c;
          // c % 4 == 0: this lane's 4 columns are one half of a keep8 group
          const uint32_t keep = a.p > 0.f ? (dropout_keep8(a.seed, a.off, e >> 3, a.th) >> (e & 4)) & 0xFu : 0xFu;
          f32x4 o, f1, f2;
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            float x, y1, y2;
            geglu_fwd_fac((float)h1[q], (float)h2[q], (keep >> q) & 1, a.ks, x, y1, y2);
            o[q] = x;
            f1[q] = y1;
            f2[q] = y2;
          }
          store_b64(rg, og, f1);  // the backward factors where g would go
          store_b64(rg, og + a.F * 2, f2);
          store_b64(ra, (uint32_t)((r * a.F + c) * 2), o);
        }
      }
  } else {  // EPI_GEGLU_BWD
    // da tile -> LDS (bf16, [256][256], 16-B chunks XOR-swizzled by row&15), then row-contiguous
    // 8-element chunks per thread: 16-B loads of the forward's factors fac, 16-B stores of
    // dg = bf16(da) * fac.
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
    const auto rgi = out_rsrc(const_cast<bf16*>(a.g) + (size_t)m0 * 2 * a.F,
                              (uint32_t)((size_t)rows * 2 * a.F * 2));
    const auto rdg = out_rsrc(a.aux + (size_t)m0 * 2 * a.F, (uint32_t)((size_t)rows * 2 * a.F * 2));
    constexpr int GB = 4;  // chunks whose g loads are in flight together
    for (int it0 = 0; it0 < 16; it0 += GB) {
      bf16x8 g1[GB], g2[GB];
      uint32_t offs[GB];
#pragma unroll
      for (int u = 0; u < GB; ++u) {
        const int idx = (it0 + u) * NTHR + tid;
        const int r = idx >> 5, n = n0 + (idx & 31) * 8;
        offs[u] = n < a.F ? (uint32_t)((r * 2 * a.F + n) * 2) : kOOB;
        g1[u] = load_b128h(rgi, offs[u]);
        g2[u] = load_b128h(rgi, offs[u] + a.F * 2);
      }
#pragma unroll
      for (int u = 0; u < GB; ++u) {
        const int idx = (it0 + u) * NTHR + tid;
        const int r = idx >> 5, c = idx & 31;
        const int m = m0 + r, n = n0 + c * 8;
        const bf16x8 d = *reinterpret_cast<const bf16x8*>(T + r * 512 + ((c ^ (r & 15)) << 4));
        (void)m;
        bf16x8 o1, o2;
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          o1[q] = (bf16)((float)d[q] * (float)g1[u][q]);
          o2[q] = (bf16)((float)d[q] * (float)g2[u][q]);
        }
        store_b128h(rdg, offs[u], o1);
        store_b128h(rdg, offs[u] + a.F * 2, o2);
      }
    }
  }
}

// ------------------------------------------------------------------ persistent K-major kernel
// y[M,N] = x[M,K] . W[N,K]^T (+ bias) with both operands K-major: the forward projections, and
// the data gradients through the transposed bf16 weight copy (dx = dy . W = dy . (W^T)^T).
// One 512-thread block per CU walks its units (256x256 output tiles) u = i*G + L(block) with the
// SAME 4-phase half-tile pipeline as gemm_kernel, but the K-steps of consecutive units form one
// continuous stream: the stages of unit i+1's first two K-steps are in flight while unit i ends,
// and unit i's outputs are stored (bias from LDS, branch-free 16-B buffer stores) piecewise in its
// last K-step, each quadrant / row half right after the MFMAs that finish it. The per-tile cost
// of the non-persistent kernel (pipeline fill from memory, block turnover, an 8-B store tail of
// 7 B/cycle/CU: ~13 us per tile at K = 768, i.e. 8 K-steps of work) drops to ~2-5 us.
// vmcnt accounting: stores issued in a unit's last K-step sit in the VMEM queue between LDS-DMA
// stages, so the waits of that step and of the next unit's first step leave them in flight
// (role-dependent immediates, see wait_vm); they retire with the waits of the step after.
constexpr int BIAS_LDS = 32 * 1024;  // bias row staged once per block (N <= 8192 floats)

__host__ __device__ constexpr int waitcnt_imm(int vm) {  // gfx9 s_waitcnt: vmcnt=vm, others no-wait
  return (vm & 0xF) | ((vm >> 4) << 14) | (0x7 << 4) | (0xF << 8);
}

// bijective blockIdx -> unit-order remap (blocks are dispatched to XCDs round-robin, b % 8): the
// blocks of one XCD get consecutive indices, for any grid size
__device__ __forceinline__ int xcd_remap(int b, int G) {
  const int xcd = b & 7, q = G >> 3, r = G & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (b >> 3);
}

template <int EPI>
__device__ __forceinline__ void unit_tile(const Args& a, int u, int& m0, int& n0) {
  const int width = a.GM * a.tilesN;
  const int grp = u / width, first = grp * a.GM;
  const int gsz = min(a.tilesM - first, a.GM);
  const int w = u - grp * width;
  m0 = (first + w % gsz) * BM;
  n0 = (w / gsz) * (EPI == EPI_GEGLU ? BN / 2 : BN);
}

// ABL (diagnostic ablations of the main loop, DNA_GEMM_ABL; results are garbage, timing only):
// 1 = no LDS-DMA staging, 2 = no LDS reads (MFMAs on stale fragments), 4 = no barriers,
// 8 = no B staging and no B reads, 16 = no B reads, 32 = no B staging
// SCH == 1 schedules: 16-B stores (per lane) issued after the stage of phase P-5 and before the
// wait of phase P, for a K-step of role r (see gemmp_kernel) and phase p. The previous unit's
// last K-step is phases -4..-1, the current unit's starts at lb. EPI_F32 = the weight-gradient
// kernel (8 fp32 stores per quadrant), EPI_BF16 4 per quadrant, EPI_GEGLU 12 after phases 1, 3.
template <int EPI>
__host__ __device__ constexpr int pend_stores(int r, int p) {
  const int P = r == 1 ? p : r == 3 ? 400 + p : 4 + p;
  const int lb = r == 3 ? 400 : r == 4 ? 4 : 1 << 20;
  int n = 0;
  for (int q = 0; q < 4; ++q) {
    const int st = EPI == EPI_F32 ? 8 : EPI == EPI_BF16 ? 4 : ((q & 1) ? 12 : 0);
    const int sp = q - 4, sc = lb + q;
    if (sp >= P - 5 && sp <= P - 1) n += st;
    if (sc >= P - 5 && sc <= P - 1) n += st;
  }
  return n;
}
static_assert(pend_stores<EPI_BF16>(1, 0) == 16 && pend_stores<EPI_BF16>(1, 3) == 8 &&
              pend_stores<EPI_BF16>(2, 0) == 4 && pend_stores<EPI_BF16>(2, 1) == 0 &&
              pend_stores<EPI_BF16>(3, 0) == 0 && pend_stores<EPI_BF16>(3, 3) == 12 &&
              pend_stores<EPI_BF16>(4, 0) == 4 && pend_stores<EPI_BF16>(4, 1) == 4 &&
              pend_stores<EPI_GEGLU>(1, 3) == 12 && pend_stores<EPI_GEGLU>(4, 2) == 12,
              "SCH 1 store counts");

// SCH selects the half-tile schedule: 0 = the original 4-phase order (reads 12/4/8/0 per phase),
// 1 = balanced reads (8/4/8/4: B_0 of the next K-step is read in phase 3) with 5 half-tiles in
// flight -- see the comment above the SCH == 1 branch
template <int EPI, int ABL = 0, int SCH = 0>
__global__ __launch_bounds__(NTHR) void gemmp_kernel(Args a) {
  static_assert(EPI == EPI_BF16 || EPI == EPI_GEGLU ||
                    (EPI == EPI_GEGLU_BWD && SCH == 2 && (ABL == 0 || ABL == 128)) ||
                    ((EPI == EPI_GELU_BWD || EPI == EPI_BF16_GELU) && SCH == 2 && ABL == 0),
                "persistent kernel: bf16 / GeGLU epilogues (GeGLU backward: lean body only)");
  __shared__ __attribute__((aligned(1024))) char smem[LDS_BYTES + BIAS_LDS];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 2, wc = wave & 3;
  const int G = gridDim.x, b = blockIdx.x;
  const int U = a.tilesM * a.tilesN;
  // this block's units: ubase + i * ustride, i < nb
  int ubase, ustride, nb;
  if (a.order == 1 && (G & 7) == 0) {
    // XCD-major: the blocks sharing an L2 (b % 8) sweep one contiguous eighth of the unit order,
    // so an A row panel is fetched into one L2 and used there for every column tile
    const int X = b & 7, j = b >> 3, GX = G >> 3;
    const int lo = (int)(((long long)U * X) >> 3), hi = (int)(((long long)U * (X + 1)) >> 3);
    ubase = lo + j;
    ustride = GX;
    nb = j < hi - lo ? (hi - lo - j + GX - 1) / GX : 0;
  } else {
    const int L = xcd_remap(b, G);  // blocks of one XCD: consecutive units
    ubase = L;
    ustride = G;
    nb = L < U ? (U - L + G - 1) / G : 0;
  }
  if (nb == 0) return;
  const int L = ubase;
  const int KT = a.K / BK;
  const int V = nb * KT;
  float* bias_lds = reinterpret_cast<float*>(smem + LDS_BYTES);
  const int nbias = EPI == EPI_GEGLU ? 2 * a.F : (EPI == EPI_GEGLU_BWD || EPI == EPI_GELU_BWD) ? 0 : a.N;
  for (int c = tid * 4; c < nbias; c += NTHR * 4)
    *reinterpret_cast<f32x4*>(bias_lds + c) =
        a.bias ? *reinterpret_cast<const f32x4*>(a.bias + c) : f32x4{0.f, 0.f, 0.f, 0.f};
  __syncthreads();

  // Operands through buffer resources over the whole matrices: per-lane offsets are fixed for the
  // kernel's life (2 VGPRs per operand), the wave-uniform tile / K position is added to voffset
  // (soffset is excluded from the range check), and rows past M read as zeros -- no per-lane
  // clamping, no 64-bit addresses.
  const int NB = EPI == EPI_GEGLU ? 2 * a.F : a.N;  // rows of the weight operand
  const auto rA = out_rsrc(a.A, (uint32_t)((size_t)a.M * a.lda * 2));
  const auto rB = out_rsrc(a.B, (uint32_t)((size_t)NB * a.ldb * 2));
  uint32_t voA[2], voB[2];
#pragma unroll
  for (int p = 0; p < 2; ++p) {
    const int lr = p * 64 + wave * 8 + (lane >> 3);
    const int ch = ((lane & 7) ^ kswz(lr)) << 4;
    voA[p] = (uint32_t)(lr * a.lda * 2 + ch);
    voB[p] = (uint32_t)(lr * a.ldb * 2 + ch);
  }

  // cursors over the virtual K-step stream: c0 = step being computed, c1/c2 = one / two ahead
  struct Cur { int i, kt, m0, n0; };
  auto cur_at = [&](int i) {
    Cur c;
    c.i = i;
    c.kt = 0;
    unit_tile<EPI>(a, ubase + min(i, nb - 1) * ustride, c.m0, c.n0);
    return c;
  };
  auto advance = [&](Cur& c) {
    if (++c.kt == KT) c = cur_at(c.i + 1);
  };
  auto img = [&](int v, int h) { return smem + ((v & 1) * 4 + h) * HALF; };
  // stage half-tile h of the K-step at cursor c (virtual step v); steps past the end re-load the
  // last unit's data into a buffer no one reads again (keeps every vmcnt count uniform)
  // K-step order within a unit is rotated per block (k = (kt + rot) mod KT): the blocks' store
  // bursts (one per unit) then fall on different steps instead of hitting memory all at once
  const int rot = a.rot ? (L * 5) % KT : 0;
  auto stage = [&](const Cur& c, int v, int h) {
    int kk = (c.i < nb ? c.kt : KT - 1) + rot;
    kk = kk >= KT ? kk - KT : kk;
    const int k0 = kk * BK;
    char* d = img(v, h);
    int row0;
    if (h < 2) row0 = c.m0 + h * 128;
    else if constexpr (EPI == EPI_GEGLU) row0 = (h - 2) * a.F + c.n0;
    else row0 = c.n0 + (h - 2) * 128;
    const int ld = h < 2 ? a.lda : a.ldb;
    // the tile offset goes into voffset, not soffset: the hardware range check covers
    // voffset + inst_offset only, so rows past M must be visible there to read as zeros
    const uint32_t toff = (uint32_t)__builtin_amdgcn_readfirstlane((row0 * ld + k0) * 2);
#pragma unroll
    for (int p = 0; p < 2; ++p)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(h < 2 ? rA : rB, (lds_t*)(d + (p * 64 + wave * 8) * 128),
                                               16, (h < 2 ? voA[p] : voB[p]) + toff, 0, 0, 0);
  };

  f32x4 acc[2][2][4][2];  // [mq][nq][i][j]
  auto zero_acc = [&]() {
#pragma unroll
    for (int q = 0; q < 2; ++q)
#pragma unroll
      for (int r = 0; r < 2; ++r)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j) acc[q][r][i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  };
  zero_acc();
  bf16x8 af[4][2], bf0[2][2], bf1[2][2];
  auto readA = [&](int v, int mq) {
    const char* im = img(v, mq);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) af[i][kk] = read_k(im, wr * 64 + i * 16 + (lane & 15), kk * 4 + (lane >> 4));
  };
  auto readB = [&](int v, int nq, bf16x8 (&bf)[2][2]) {
    const char* im = img(v, 2 + nq);
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) bf[j][kk] = read_k(im, wc * 32 + j * 16 + (lane & 15), kk * 4 + (lane >> 4));
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

  // epilogue stores: lane part of the offset fixed, tile row / column block added to it; rows
  // past M fall outside the resource and are dropped
  const int cq = 4 * (lane >> 4);
  const int ldo = EPI == EPI_GEGLU ? 2 * a.F : a.ldc;
  const auto rC = out_rsrc((EPI == EPI_GEGLU_BWD || EPI == EPI_GELU_BWD) ? (void*)a.aux : a.C,
                           (uint32_t)((size_t)a.M * ldo * 2));
  // EPI_BF16_GELU: gelu(h) beside h, same layout
  const auto rAct = out_rsrc(EPI == EPI_BF16_GELU ? (void*)a.aux : a.C, (uint32_t)((size_t)a.M * ldo * 2));
  const uint32_t voC = (uint32_t)(((wr * 64 + (lane & 15)) * ldo + wc * 32 + cq) * 2);
  // BF16: a quadrant (mq, nq) is final right after its MFMAs in a unit's last K-step, so it is
  // stored there (bias from LDS), overlapping the remaining phases. For each (row block i) the
  // lane's two 4-column groups j = 0 / 1 are exchanged with v_permlane16_swap so that every
  // lane holds 8 consecutive columns: one 16-B store instead of two 8-B ones (the store tail is
  // issue-bound per instruction). After the swap, column group cg = lane >> 4 holds columns
  // {0, 16, 8, 24}[cg] .. +7 of the wave's 32-column slab.
  const uint32_t voQ = (uint32_t)(((wr * 64 + (lane & 15)) * a.ldc + wc * 32 +
                                   (((lane >> 4) & 1) << 4) + (((lane >> 4) & 2) << 2)) * 2);
  auto store_quadrant = [&](const Cur& c, int mq, int nq) __attribute__((always_inline)) {
    const f32x4 bj0 = *reinterpret_cast<const f32x4*>(bias_lds + c.n0 + nq * 128 + wc * 32 + cq);
    const f32x4 bj1 = *reinterpret_cast<const f32x4*>(bias_lds + c.n0 + nq * 128 + wc * 32 + 16 + cq);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const f32x4 v0 = acc[mq][nq][i][0] + bj0, v1 = acc[mq][nq][i][1] + bj1;
      u32x2 h0 = __builtin_bit_cast(u32x2, bf16x4{(bf16)v0[0], (bf16)v0[1], (bf16)v0[2], (bf16)v0[3]});
      u32x2 h1 = __builtin_bit_cast(u32x2, bf16x4{(bf16)v1[0], (bf16)v1[1], (bf16)v1[2], (bf16)v1[3]});
      const auto sx = __builtin_amdgcn_permlane16_swap(h0[0], h1[0], false, false);
      const auto sy = __builtin_amdgcn_permlane16_swap(h0[1], h1[1], false, false);
      const u32x4 o = u32x4{sx[0], sy[0], sx[1], sy[1]};
      // row block in voffset (range-checked: rows past M are dropped), never in soffset
      const uint32_t off = voQ + (uint32_t)__builtin_amdgcn_readfirstlane(
                                     ((c.m0 + mq * 128 + i * 16) * a.ldc + c.n0 + nq * 128) * 2);
      // DNA_GEMM_NT=1 streams the output tiles with the non-temporal policy (aux 2): +2-9 % on
      // isolated K = 768 GEMMs, but -1 % on the training step (the next kernel reads them), so off
      if (a.dbg == 0) {
        if (a.nt) __builtin_amdgcn_raw_buffer_store_b128(o, rC, off, 0, 2);
        else __builtin_amdgcn_raw_buffer_store_b128(o, rC, off, 0, 0);
      } else if (a.dbg == 4) __builtin_amdgcn_raw_buffer_store_b128(o, rC, off, 0, 1);  // sc0
      else if (a.dbg == 1) __builtin_amdgcn_raw_buffer_store_b128(o, rC, kOOB, 0, 0);
      else asm volatile("" :: "v"(o));
      acc[mq][nq][i][0] = f32x4{0.f, 0.f, 0.f, 0.f};
      acc[mq][nq][i][1] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
  };

  // GeGLU: the rows of half mq are final once both column quadrants (mq, 0) = g1 and (mq, 1) = g2
  // are (phase 1 for mq = 0, phase 3 for mq = 1 of a unit's last K-step): bias, bf16 rounding of
  // g1 / g2, then a = dropout(gelu(g1) * g2) and the backward factors fac1 / fac2 (common.h
  // geglu_fwd_fac; stored where g would go) from the rounded values -- all three widened to 16-B
  // stores by the same permlane16 exchange; one Philox keep8 draw per 8 columns.
  const auto rAux = out_rsrc(a.aux, (uint32_t)((size_t)a.M * a.F * 2));
  const int colq = wc * 32 + (((lane >> 4) & 1) << 4) + (((lane >> 4) & 2) << 2);  // after the swap
  const uint32_t voG = (uint32_t)(((wr * 64 + (lane & 15)) * 2 * a.F + colq) * 2);
  const uint32_t voAx = (uint32_t)(((wr * 64 + (lane & 15)) * a.F + colq) * 2);
  auto swap8 = [&](f32x4 v0, f32x4 v1) __attribute__((always_inline)) {  // two 4-column groups -> this lane's 8 columns (bf16)
    u32x2 h0 = __builtin_bit_cast(u32x2, bf16x4{(bf16)v0[0], (bf16)v0[1], (bf16)v0[2], (bf16)v0[3]});
    u32x2 h1 = __builtin_bit_cast(u32x2, bf16x4{(bf16)v1[0], (bf16)v1[1], (bf16)v1[2], (bf16)v1[3]});
    const auto sx = __builtin_amdgcn_permlane16_swap(h0[0], h1[0], false, false);
    const auto sy = __builtin_amdgcn_permlane16_swap(h0[1], h1[1], false, false);
    return u32x4{sx[0], sy[0], sx[1], sy[1]};
  };
  auto store_geglu_half = [&](const auto& c, int mq) __attribute__((always_inline)) {
    const f32x4 b10 = *reinterpret_cast<const f32x4*>(bias_lds + c.n0 + wc * 32 + cq);
    const f32x4 b11 = *reinterpret_cast<const f32x4*>(bias_lds + c.n0 + wc * 32 + 16 + cq);
    const f32x4 b20 = *reinterpret_cast<const f32x4*>(bias_lds + a.F + c.n0 + wc * 32 + cq);
    const f32x4 b21 = *reinterpret_cast<const f32x4*>(bias_lds + a.F + c.n0 + wc * 32 + 16 + cq);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const u32x4 g1 = swap8(acc[mq][0][i][0] + b10, acc[mq][0][i][1] + b11);
      const u32x4 g2 = swap8(acc[mq][1][i][0] + b20, acc[mq][1][i][1] + b21);
      const int row = c.m0 + mq * 128 + i * 16;
      // row-block offsets added per lane (soffset 0): keeps this epilogue's scalar footprint small
      const uint32_t og = voG + (uint32_t)((row * 2 * a.F + c.n0) * 2);
      const uint32_t oa = voAx + (uint32_t)((row * a.F + c.n0) * 2);
      const bf16x8 h1 = __builtin_bit_cast(bf16x8, g1), h2 = __builtin_bit_cast(bf16x8, g2);
      const size_t e = (size_t)(row + wr * 64 + (lane & 15)) * a.F + c.n0 + colq;  // e % 8 == 0
      // the keep decision per element straight from its 16-bit half of the draw (a compare +
      // select each; packing the 8 bits into a mask and unpacking them cost ~4 VALU more apiece)
      const uint4 r = a.p > 0.f ? dropout_draw8(a.seed, a.off, e >> 3) : make_uint4(~0u, ~0u, ~0u, ~0u);
      bf16x8 o, f1, f2;
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        float x, y1, y2;
        geglu_fwd_fac((float)h1[q], (float)h2[q], dropout_kept8(r, q, a.th), a.ks, x, y1, y2);
        o[q] = (bf16)x;
        f1[q] = (bf16)y1;
        f2[q] = (bf16)y2;
      }
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, f1), rC, og, 0, 0);
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, f2), rC, og + a.F * 2, 0, 0);
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, o), rAux, oa, 0, 0);
#pragma unroll
      for (int nq = 0; nq < 2; ++nq)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[mq][nq][i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
  };

  constexpr int QS = 4;  // 16-B stores per quadrant and lane (BF16)
  constexpr int GS = 12;  // GeGLU: 16-B stores per half (g1, g2, a x 4 row blocks)
  Cur c0 = cur_at(0), c1 = c0, c2 = c0;
  advance(c1);
  advance(c2);
  advance(c2);
  if constexpr (SCH == 0) {
  // prologue: all four halves of step 0, the A_0 / B_0 halves of step 1
  stage(c0, 0, 0);
  stage(c0, 0, 2);
  stage(c0, 0, 3);
  stage(c0, 0, 1);
  stage(c1, 1, 0);
  stage(c1, 1, 2);
  __builtin_amdgcn_s_waitcnt(waitcnt_imm(8));
  DNA_BARRIER();
  if (wr == 1) DNA_BARRIER();  // stagger: waves 4-7 one barrier behind

  // One copy of the K-step body; the wait immediates depend on the step's role (a scalar branch
  // around each s_waitcnt, so the MFMA code and its accumulator registers are shared):
  //   role 0  ordinary step: vmcnt(8) (4 half-tiles = 8 LDS-DMA pieces stay in flight)
  //   role 1  a unit's last step (BF16): quadrant q's QS stores are issued after phase q's MFMAs,
  //           so phase p's wait also leaves the p * QS stores issued since phase 0 in flight
  //   role 2  a unit's first step after an epilogue: the stores issued behind the half-tiles it
  //           waits for stay in flight -- BF16 (4 - p) * QS, GeGLU (epilogue after the last step) S
  auto wait_vm = [&](auto phase, int role) {
    constexpr int p = decltype(phase)::value;
    // GeGLU: half 0 stored after phase 1's MFMAs, half 1 after phase 3's
    constexpr int w1 = EPI == EPI_BF16 ? 8 + p * QS : 8 + (p >= 2 ? GS : 0);
    constexpr int w2 = EPI == EPI_BF16 ? 8 + (4 - p) * QS : 8 + (p < 2 ? 2 * GS : GS);
    if (role == 0) __builtin_amdgcn_s_waitcnt(waitcnt_imm(8));
    else if (role == 1) __builtin_amdgcn_s_waitcnt(waitcnt_imm(w1));
    else __builtin_amdgcn_s_waitcnt(waitcnt_imm(w2));
  };
  using P0 = std::integral_constant<int, 0>;
  using P1 = std::integral_constant<int, 1>;
  using P2 = std::integral_constant<int, 2>;
  using P3 = std::integral_constant<int, 3>;
  auto kstep = [&](int v, int role) {
    auto stg = [&](const Cur& c, int vv, int h) {
      if constexpr (!(ABL & 1)) {
        if (!(ABL & 40) || h < 2) stage(c, vv, h);
      }
    };
    auto rdA = [&](int vv, int mq) { if constexpr (!(ABL & 2)) readA(vv, mq); };
    auto rdB = [&](int vv, int nq, bf16x8 (&bf)[2][2]) {
      if constexpr (!(ABL & 2) && !(ABL & 24)) readB(vv, nq, bf);
    };
    auto bar = [&]() { if constexpr (!(ABL & 4)) { DNA_BARRIER(); } else { __builtin_amdgcn_sched_barrier(0); } };
    const bool st = EPI == EPI_BF16 && role == 1;
    const bool sg = EPI == EPI_GEGLU && role == 1;
    // phase 0: quadrant (0,0)
    stg(c1, v + 1, 3);
    wait_vm(P0{}, role);
    rdA(v, 0);
    rdB(v, 0, bf0);
    bar();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    mma(0, 0, bf0);
    if (st) store_quadrant(c0, 0, 0);
    bar();
    // phase 1: quadrant (0,1)
    stg(c1, v + 1, 1);
    wait_vm(P1{}, role);
    rdB(v, 1, bf1);
    bar();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    mma(0, 1, bf1);
    if (st) store_quadrant(c0, 0, 1);
    if (sg) store_geglu_half(c0, 0);
    bar();
    // phase 2: quadrant (1,1)
    stg(c2, v + 2, 0);
    wait_vm(P2{}, role);
    rdA(v, 1);
    bar();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    mma(1, 1, bf1);
    if (st) store_quadrant(c0, 1, 1);
    bar();
    // phase 3: quadrant (1,0)
    stg(c2, v + 2, 2);
    wait_vm(P3{}, role);
    bar();
    mma(1, 0, bf0);
    if (st) store_quadrant(c0, 1, 0);
    if (sg) store_geglu_half(c0, 1);
    bar();
  };

  int v = 0;
  for (int i = 0; i < nb; ++i) {
    for (int kt = 0; kt < KT; ++kt, ++v) {
      const int role = kt == KT - 1 ? 1 : (kt == 0 && i > 0) ? 2 : 0;
      kstep(v, role);
      advance(c1);
      advance(c2);
    }
    c0 = cur_at(i + 1);
  }
  } else if constexpr (SCH == 1) {
    // SCH == 1. Per K-step v (quadrant order (0,0) (0,1) (1,1) (1,0)):
    //   phase  reads        stages         MFMAs with
    //   0      A_0(v)       S(v+1, A_1)    A_0, B_0(v) (read in phase 3 of step v-1)
    //   1      B_1(v)       S(v+2, B_0)    A_0, B_1
    //   2      A_1(v)       S(v+2, A_0)    A_1, B_1
    //   3      B_0(v+1)     S(v+2, B_1)    A_1, B_0(v)
    // Every phase reads at most 8 fragments per wave (the SCH 0 order reads 12 in phase 0, whose
    // LDS time plus the DMA writes then outlasts the partner wave's 16-MFMA cluster). The two B
    // register sets swap roles every K-step. WAR: every half is restaged 2 phases after its last
    // read (the other wave group's reads of the phase before may still be in flight). RAW: a
    // half read in phase P was staged in phase P-6 or earlier and is retired by the wait of phase
    // P-1 (then a barrier), which leaves the 5 youngest half-tiles (10 LDS-DMA pieces per lane) in
    // flight plus every epilogue store issued after the retiring stage -- the stores of a unit's
    // last K-step sit in the same in-order VMEM count.
    constexpr int hA0 = 0, hA1 = 1, hB0 = 2, hB1 = 3;
    // step roles: 0 = no store pending in any wait window, 1 = a unit's first K-step after an
    // epilogue, 2 = its second, 3 = a unit's last K-step (KT > 2, or the block's first unit),
    // 4 = second and last at once (KT == 2 after an epilogue). pend_stores<EPI>(role, p) is the
    // number of 16-B stores issued after the stage of phase P-5 and before the wait of phase P.
    auto wait_p = [&](auto phase, int role) {
      constexpr int p = decltype(phase)::value;
      if (role == 0) __builtin_amdgcn_s_waitcnt(waitcnt_imm(10));
      else if (role == 1) __builtin_amdgcn_s_waitcnt(waitcnt_imm(10 + pend_stores<EPI>(1, p)));
      else if (role == 2) __builtin_amdgcn_s_waitcnt(waitcnt_imm(10 + pend_stores<EPI>(2, p)));
      else if (role == 3) __builtin_amdgcn_s_waitcnt(waitcnt_imm(10 + pend_stores<EPI>(3, p)));
      else __builtin_amdgcn_s_waitcnt(waitcnt_imm(10 + pend_stores<EPI>(4, p)));
    };
    auto lgkm0 = [&]() {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
    };
    auto step = [&](int v, int kt, bool prev, bf16x8 (&bB0)[2][2], bf16x8 (&bB1)[2][2]) {
      const bool last = kt == KT - 1;
      const int role = __builtin_amdgcn_readfirstlane(
          last ? (prev && kt == 1 ? 4 : 3) : prev && kt == 0 ? 1 : prev && kt == 1 ? 2 : 0);
      const bool st = EPI == EPI_BF16 && last;
      const bool sg = EPI == EPI_GEGLU && last;
      // phase 0: quadrant (0,0)
      stage(c1, v + 1, hA1);
      wait_p(std::integral_constant<int, 0>{}, role);
      readA(v, 0);
      DNA_BARRIER();
      lgkm0();
      mma(0, 0, bB0);
      if (st) store_quadrant(c0, 0, 0);
      DNA_BARRIER();
      // phase 1: quadrant (0,1)
      stage(c2, v + 2, hB0);
      wait_p(std::integral_constant<int, 1>{}, role);
      readB(v, 1, bB1);
      DNA_BARRIER();
      lgkm0();
      mma(0, 1, bB1);
      if (st) store_quadrant(c0, 0, 1);
      if (sg) store_geglu_half(c0, 0);
      DNA_BARRIER();
      // phase 2: quadrant (1,1)
      stage(c2, v + 2, hA0);
      wait_p(std::integral_constant<int, 2>{}, role);
      readA(v, 1);
      DNA_BARRIER();
      lgkm0();
      mma(1, 1, bB1);
      if (st) store_quadrant(c0, 1, 1);
      DNA_BARRIER();
      // phase 3: quadrant (1,0); B_0 of the next K-step into the set B_1 just left
      stage(c2, v + 2, hB1);
      wait_p(std::integral_constant<int, 3>{}, role);
      readB(v + 1, 0, bB1);
      DNA_BARRIER();
      lgkm0();
      mma(1, 0, bB0);
      if (st) store_quadrant(c0, 1, 0);
      if (sg) store_geglu_half(c0, 1);
      DNA_BARRIER();
    };
    // prologue = the stages of the virtual steps -2 and -1: S(0,B0) S(0,A0) S(0,B1) S(0,A1)
    // S(1,B0) S(1,A0) S(1,B1); the wait retires the two oldest, then B_0(0) is read ("phase 3
    // of step -1")
    stage(c0, 0, hB0);
    stage(c0, 0, hA0);
    stage(c0, 0, hB1);
    stage(c0, 0, hA1);
    stage(c1, 1, hB0);
    stage(c1, 1, hA0);
    stage(c1, 1, hB1);
    __builtin_amdgcn_s_waitcnt(waitcnt_imm(10));
    DNA_BARRIER();
    readB(0, 0, bf0);
    if (wr == 1) DNA_BARRIER();  // stagger: waves 4-7 one barrier behind
    int kt = 0, i = 0;
    auto next = [&]() {
      advance(c1);
      advance(c2);
      if (++kt == KT) {
        kt = 0;
        ++i;
        c0 = cur_at(i);
      }
    };
    for (int v = 0; v < V; v += 2) {
      step(v, kt, i > 0, bf0, bf1);
      next();
      if (v + 1 < V) {
        step(v + 1, kt, i > 0, bf1, bf0);
        next();
      }
    }
  } else {
    // SCH == 2: the SCH 0 schedule with the per-phase instruction overhead taken out of the
    // load half-phases (the half-phase in which a wave stages, waits and reads while its SIMD
    // partner runs its MFMA cluster): K-steps unrolled by two so the LDS buffer parity is a
    // compile-time constant, every fragment read is one ds_read_b128 off one of 8 per-lane base
    // registers with an immediate offset (no address VALU), the stage offsets of a unit are
    // computed once when a cursor enters it (one scalar add per stage), the wait role is one
    // scalar per K-step, and the epilogue stores carry no diagnostic branches.
    const int l16 = lane & 15, lq = lane >> 4, sw = kswz(l16);  // kswz(row) == kswz(row & 15)
    const uint32_t sbase = lds_addr(smem);
    uint32_t rbA[2][2], rbB[2][2];  // [parity][k half]
#pragma unroll
    for (int par = 0; par < 2; ++par)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        const uint32_t ch = (uint32_t)((((kk * 4 + lq) ^ sw)) << 4);
        rbA[par][kk] = sbase + par * 4 * HALF + (wr * 64 + l16) * 128 + ch;
        rbB[par][kk] = sbase + par * 4 * HALF + 2 * HALF + (wc * 32 + l16) * 128 + ch;
      }
    // a unit's tile and the byte offsets of its four half-tile row blocks
    struct LCur { int o0, o1, o2, o3, m0, n0; };
    auto lcur_at = [&](int i) {
      LCur c;
      unit_tile<EPI>(a, ubase + i * ustride, c.m0, c.n0);
      c.o0 = __builtin_amdgcn_readfirstlane(c.m0 * a.lda * 2);
      c.o1 = __builtin_amdgcn_readfirstlane((c.m0 + 128) * a.lda * 2);
      // weight rows of the two B halves: n0 + [0, 128) and n0 + [128, 256); GeGLU: the g1 rows
      // n0 + [0, 128) and the g2 rows F + n0 + [0, 128)
      c.o2 = __builtin_amdgcn_readfirstlane(c.n0 * a.ldb * 2);
      c.o3 = __builtin_amdgcn_readfirstlane((c.n0 + (EPI == EPI_GEGLU ? a.F : 128)) * a.ldb * 2);
      return c;
    };
    // stage half h of K-step k of the current unit (k >= KT: step k - KT of the next unit; past
    // the block's last unit "next" is the last unit again, re-staged into buffers nobody reads)
    auto lstage = [&](const LCur& cur, const LCur& nxt, int k, auto par_c, auto h_c) {
      constexpr int par = decltype(par_c)::value, h = decltype(h_c)::value;
      const int oc = h == 0 ? cur.o0 : h == 1 ? cur.o1 : h == 2 ? cur.o2 : cur.o3;
      const int on = h == 0 ? nxt.o0 : h == 1 ? nxt.o1 : h == 2 ? nxt.o2 : nxt.o3;
      const uint32_t toff = (uint32_t)(k < KT ? oc + k * (BK * 2) : on + (k - KT) * (BK * 2));
      char* d = smem + (par * 4 + h) * HALF;
#pragma unroll
      for (int p = 0; p < 2; ++p)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(h < 2 ? rA : rB, (lds_t*)(d + (p * 64 + wave * 8) * 128),
                                                 16, (h < 2 ? voA[p] : voB[p]) + toff, 0, 0, 0);
    };
    auto rd16 = [](uint32_t addr, auto off_c) {
      constexpr int off = decltype(off_c)::value;
      u32x4 r;
      asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(r) : "v"(addr), "i"(off) : "memory");
      return __builtin_bit_cast(bf16x8, r);
    };
    using I0 = std::integral_constant<int, 0>;
    using I1 = std::integral_constant<int, 1>;
    using I2 = std::integral_constant<int, 2>;
    using I3 = std::integral_constant<int, 3>;
    auto lreadA = [&](auto par_c, auto mq_c) {
      constexpr int par = decltype(par_c)::value, mq = decltype(mq_c)::value;
      af[0][0] = rd16(rbA[par][0], std::integral_constant<int, mq * HALF>{});
      af[0][1] = rd16(rbA[par][1], std::integral_constant<int, mq * HALF>{});
      af[1][0] = rd16(rbA[par][0], std::integral_constant<int, mq * HALF + 2048>{});
      af[1][1] = rd16(rbA[par][1], std::integral_constant<int, mq * HALF + 2048>{});
      af[2][0] = rd16(rbA[par][0], std::integral_constant<int, mq * HALF + 4096>{});
      af[2][1] = rd16(rbA[par][1], std::integral_constant<int, mq * HALF + 4096>{});
      af[3][0] = rd16(rbA[par][0], std::integral_constant<int, mq * HALF + 6144>{});
      af[3][1] = rd16(rbA[par][1], std::integral_constant<int, mq * HALF + 6144>{});
    };
    auto lreadB = [&](auto par_c, auto nq_c, bf16x8 (&bf)[2][2]) {
      constexpr int par = decltype(par_c)::value, nq = decltype(nq_c)::value;
      bf[0][0] = rd16(rbB[par][0], std::integral_constant<int, nq * HALF>{});
      bf[0][1] = rd16(rbB[par][1], std::integral_constant<int, nq * HALF>{});
      bf[1][0] = rd16(rbB[par][0], std::integral_constant<int, nq * HALF + 2048>{});
      bf[1][1] = rd16(rbB[par][1], std::integral_constant<int, nq * HALF + 2048>{});
    };
    // the bias of quadrant column block nq, read in the load half-phase (beside the fragment
    // reads, retired by the same lgkmcnt wait) so the epilogue never waits on LDS
    auto lbias = [&](const LCur& c, int nq, f32x4& bj0, f32x4& bj1) {
      bj0 = *reinterpret_cast<const f32x4*>(bias_lds + c.n0 + nq * 128 + wc * 32 + cq);
      bj1 = *reinterpret_cast<const f32x4*>(bias_lds + c.n0 + nq * 128 + wc * 32 + 16 + cq);
    };
    // stores quadrant (mq, nq) of the unit's tile; the accumulators are not re-zeroed: the next
    // unit's first K-step starts its MFMA chains from a zero C operand (mmaz)
    auto lstore = [&](const LCur& c, int mq, int nq, f32x4 bj0, f32x4 bj1) __attribute__((always_inline)) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const f32x4 v0 = acc[mq][nq][i][0] + bj0, v1 = acc[mq][nq][i][1] + bj1;
        u32x2 h0 = __builtin_bit_cast(u32x2, bf16x4{(bf16)v0[0], (bf16)v0[1], (bf16)v0[2], (bf16)v0[3]});
        u32x2 h1 = __builtin_bit_cast(u32x2, bf16x4{(bf16)v1[0], (bf16)v1[1], (bf16)v1[2], (bf16)v1[3]});
        const auto sx = __builtin_amdgcn_permlane16_swap(h0[0], h1[0], false, false);
        const auto sy = __builtin_amdgcn_permlane16_swap(h0[1], h1[1], false, false);
        const u32x4 o = u32x4{sx[0], sy[0], sx[1], sy[1]};
        uint32_t off = voQ + (uint32_t)__builtin_amdgcn_readfirstlane(
                                 ((c.m0 + mq * 128 + i * 16) * a.ldc + c.n0 + nq * 128) * 2);
        off = a.dbg == 1 ? kOOB : off;  // diagnostics: stores dropped by the range check
        if constexpr (EPI == EPI_BF16_GELU) {
          // a = bf16(gelu_tanh(h)) of the bf16-rounded h, as torch's GELU reads h
          const bf16x4 e0 = __builtin_bit_cast(bf16x4, h0), e1 = __builtin_bit_cast(bf16x4, h1);
          bf16x4 g0, g1;
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            g0[q] = (bf16)gelu_tanh((float)e0[q]);
            g1[q] = (bf16)gelu_tanh((float)e1[q]);
          }
          const u32x2 k0 = __builtin_bit_cast(u32x2, g0), k1 = __builtin_bit_cast(u32x2, g1);
          const auto gx = __builtin_amdgcn_permlane16_swap(k0[0], k1[0], false, false);
          const auto gy = __builtin_amdgcn_permlane16_swap(k0[1], k1[1], false, false);
          __builtin_amdgcn_raw_buffer_store_b128(u32x4{gx[0], gy[0], gx[1], gy[1]}, rAct, off, 0, 0);
        }
        // DNA_GEMM_NT=1 (A/B): non-temporal stores. Measured (profiles/r03b): nt, sc1 and sc0 sc1
        // stores and whole-line store patterns are all slower or equal; dropping the stores
        // (DNA_GEMM_DBG=1) saves ~3.5 us per unit at every K: the in-order vmcnt makes the
        // stages issued after a unit's stores wait for them
        if (a.nt) __builtin_amdgcn_raw_buffer_store_b128(o, rC, off, 0, 2);
        else __builtin_amdgcn_raw_buffer_store_b128(o, rC, off, 0, 0);
      }
    };
    // GeGLU backward (dg = geglu_bwd(da, g) with da = this GEMM's output, never stored): quadrant
    // (mq, nq)'s saved g1 / g2 (8 columns per lane and row block, the layout after the permlane16
    // exchange) are loaded in the phase's load half-phase, beside the fragment reads, and used
    // after its MFMAs -- the compiler's own vmcnt waits count them against the LDS-DMA stages
    // issued before; da is rounded to bf16 first, as the separate pass reads it
    // GeGLU backward: g / dg rows are 2F wide; GELU backward (EPI_GELU_BWD): h / dh rows F wide
    // -- either way = a.ldc (launcher), so the lane offset is voQ's (no extra VGPR)
    constexpr bool GELU = EPI == EPI_GELU_BWD;
    const int gld = GELU ? a.F : 2 * a.F;
    const auto rGi = out_rsrc(a.g, (uint32_t)((size_t)a.M * gld * 2));
    const uint32_t voGB = voQ;
    auto lgload = [&](const LCur& c, int mq, int nq, bf16x8 (&gv)[4][2]) __attribute__((always_inline)) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const uint32_t off = voGB + (uint32_t)__builtin_amdgcn_readfirstlane(
                                        ((c.m0 + mq * 128 + i * 16) * gld + c.n0 + nq * 128) * 2);
        gv[i][0] = load_b128h(rGi, (ABL & 128) ? kOOB : off);
      }
      if constexpr (GELU) return;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const uint32_t off = voGB + (uint32_t)__builtin_amdgcn_readfirstlane(
                                        ((c.m0 + mq * 128 + i * 16) * 2 * a.F + c.n0 + nq * 128) * 2);
        gv[i][1] = load_b128h(rGi, (ABL & 128) ? kOOB : off + a.F * 2);
      }
    };
    auto lgstore = [&](const LCur& c, int mq, int nq, const bf16x8 (&gv)[4][2]) __attribute__((always_inline)) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const bf16x8 d = __builtin_bit_cast(bf16x8, swap8(acc[mq][nq][i][0], acc[mq][nq][i][1]));
        const int row = c.m0 + mq * 128 + i * 16;
        if constexpr (GELU) {
          // dh = bf16(da) * gelu_tanh'(h), da rounded to bf16 first as torch's separate
          // GeluBackward reads it (the MLP fc2 data gradient, HyenaDNA Mlp)
          bf16x8 o;
#pragma unroll
          for (int q = 0; q < 8; ++q) o[q] = (bf16)((float)d[q] * gelu_tanh_grad((float)gv[i][0][q]));
          const uint32_t off = voGB + (uint32_t)__builtin_amdgcn_readfirstlane(
                                          (row * a.F + c.n0 + nq * 128) * 2);
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, o), rC, off, 0, 0);
          continue;
        }
        // dg = bf16(da) * fac (the forward's factors: GELU derivative, g2, keep bit and 1/(1-p)
        // folded in, common.h geglu_fwd_fac)
        bf16x8 o1, o2;
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          o1[q] = (bf16)((float)d[q] * (float)gv[i][0][q]);
          o2[q] = (bf16)((float)d[q] * (float)gv[i][1][q]);
        }
        const uint32_t off = voGB + (uint32_t)__builtin_amdgcn_readfirstlane(
                                        (row * 2 * a.F + c.n0 + nq * 128) * 2);
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, o1), rC, off, 0, 0);
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, o2), rC, off + a.F * 2, 0, 0);
      }
    };
    auto mmaz = [&](int mq, int nq, const bf16x8 (&bf)[2][2]) {
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[mq][nq][i][j] = mfma(bf[j][0], af[i][0], f32x4{0.f, 0.f, 0.f, 0.f});
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[mq][nq][i][j] = mfma(bf[j][1], af[i][1], acc[mq][nq][i][j]);
      __builtin_amdgcn_s_setprio(0);
    };
    // roles (compile-time, one step body per role): 0 ordinary, 1 a unit's last K-step (its
    // quadrant stores sit between the stages), 2 the first K-step after an epilogue
    auto lwait = [&](auto phase_c, auto role_c) {
      constexpr int p = decltype(phase_c)::value, role = decltype(role_c)::value;
      // BF16: QS stores after every phase of a unit's last step; GeGLU: GS after phases 1 and 3
      // GeGLU backward: each phase of the last step issues its quadrant's 8 g loads before its
      // stage (they stay in flight through the wait: + 8) and 8 stores after its MFMAs, each
      // group after an epilogue wait that retired everything older than its g loads
      // (GELU backward: 4 h loads and 4 dh stores per quadrant)
      constexpr int QB = EPI == EPI_GELU_BWD ? 4 : 8;
      constexpr int QE = EPI == EPI_BF16_GELU ? 2 * QS : QS;  // + the a stores
      constexpr int n = (EPI == EPI_BF16 || EPI == EPI_BF16_GELU)
                            ? (role == 0 ? 8 : role == 1 ? 8 + p * QE : 8 + (4 - p) * QE)
                            : (EPI == EPI_GEGLU_BWD || EPI == EPI_GELU_BWD)
                            ? (role == 0 ? 8 : role == 1 ? 8 + QB + p * QB : 8 + (4 - p) * QB)
                            : (role == 0 ? 8 : role == 1 ? 8 + (p >= 2 ? GS : 0) : 8 + (p < 2 ? 2 * GS : GS));
      __builtin_amdgcn_s_waitcnt(waitcnt_imm(n));
    };
    auto lgkm0 = [&]() {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
    };
    constexpr bool SB = EPI == EPI_BF16 || EPI == EPI_BF16_GELU;  // per-quadrant stores (else GeGLU halves)
    constexpr bool GB = EPI == EPI_GEGLU_BWD || EPI == EPI_GELU_BWD;  // per-quadrant backward epilogue
    // one K-step k of the current unit in buffer parity par; ZI: the unit's first K-step (MFMA
    // chains start from zero)
    auto lstep = [&](auto par_c, auto role_c, auto zi_c, int k, const LCur& cur, const LCur& nxt) {
      constexpr int par = decltype(par_c)::value, role = decltype(role_c)::value;
      constexpr bool ZI = decltype(zi_c)::value;
      using Pc = std::integral_constant<int, par>;
      using Qc = std::integral_constant<int, par ^ 1>;
      auto mm = [&](int mq, int nq, const bf16x8 (&bf)[2][2]) {
        if constexpr (ZI) mmaz(mq, nq, bf);
        else mma(mq, nq, bf);
      };
      f32x4 bj0, bj1;
      bf16x8 gv[4][2];
      // phase 0: quadrant (0,0)
      if constexpr (GB && role == 1) lgload(cur, 0, 0, gv);
      lstage(cur, nxt, k + 1, Qc{}, I3{});
      lwait(I0{}, role_c);
      lreadA(Pc{}, I0{});
      lreadB(Pc{}, I0{}, bf0);
      if constexpr (SB && role == 1) lbias(cur, 0, bj0, bj1);
      DNA_BARRIER();
      lgkm0();
      mm(0, 0, bf0);
      if constexpr (SB && role == 1) lstore(cur, 0, 0, bj0, bj1);
      if constexpr (GB && role == 1) lgstore(cur, 0, 0, gv);
      DNA_BARRIER();
      // phase 1: quadrant (0,1)
      if constexpr (GB && role == 1) lgload(cur, 0, 1, gv);
      lstage(cur, nxt, k + 1, Qc{}, I1{});
      lwait(I1{}, role_c);
      lreadB(Pc{}, I1{}, bf1);
      if constexpr (SB && role == 1) lbias(cur, 1, bj0, bj1);
      DNA_BARRIER();
      lgkm0();
      mm(0, 1, bf1);
      if constexpr (SB && role == 1) lstore(cur, 0, 1, bj0, bj1);
      if constexpr (GB && role == 1) lgstore(cur, 0, 1, gv);
      if constexpr (!SB && !GB && role == 1) store_geglu_half(cur, 0);
      DNA_BARRIER();
      // phase 2: quadrant (1,1)
      if constexpr (GB && role == 1) lgload(cur, 1, 1, gv);
      lstage(cur, nxt, k + 2, Pc{}, I0{});
      lwait(I2{}, role_c);
      lreadA(Pc{}, I1{});
      DNA_BARRIER();
      lgkm0();
      mm(1, 1, bf1);
      if constexpr (SB && role == 1) lstore(cur, 1, 1, bj0, bj1);
      if constexpr (GB && role == 1) lgstore(cur, 1, 1, gv);
      DNA_BARRIER();
      // phase 3: quadrant (1,0)
      if constexpr (GB && role == 1) lgload(cur, 1, 0, gv);
      lstage(cur, nxt, k + 2, Pc{}, I2{});
      lwait(I3{}, role_c);
      if constexpr (SB && role == 1) lbias(cur, 0, bj0, bj1);
      DNA_BARRIER();
      if constexpr (SB && role == 1) lgkm0();
      mm(1, 0, bf0);
      if constexpr (SB && role == 1) lstore(cur, 1, 0, bj0, bj1);
      if constexpr (GB && role == 1) lgstore(cur, 1, 0, gv);
      if constexpr (!SB && !GB && role == 1) store_geglu_half(cur, 1);
      DNA_BARRIER();
    };
    using ZN = std::false_type;
    using ZY = std::true_type;
    using R0 = std::integral_constant<int, 0>;
    using RL = std::integral_constant<int, 1>;
    using RF = std::integral_constant<int, 2>;
    // KT is even (launcher), so every unit starts on buffer parity 0
    LCur cur = lcur_at(0), nxt = lcur_at(nb > 1 ? 1 : 0);
    // prologue (as SCH 0): all four halves of step 0, A_0 / B_0 of step 1
    lstage(cur, nxt, 0, I0{}, I0{});
    lstage(cur, nxt, 0, I0{}, I2{});
    lstage(cur, nxt, 0, I0{}, I3{});
    lstage(cur, nxt, 0, I0{}, I1{});
    lstage(cur, nxt, 1, I1{}, I0{});
    lstage(cur, nxt, 1, I1{}, I2{});
    __builtin_amdgcn_s_waitcnt(waitcnt_imm(8));
    DNA_BARRIER();
    if (wr == 1) DNA_BARRIER();  // stagger: waves 4-7 one barrier behind
    lstep(I0{}, R0{}, ZY{}, 0, cur, nxt);
    for (int i = 0;;) {
      for (int k = 1; k < KT - 1; k += 2) {
        lstep(I1{}, R0{}, ZN{}, k, cur, nxt);
        lstep(I0{}, R0{}, ZN{}, k + 1, cur, nxt);
      }
      lstep(I1{}, RL{}, ZN{}, KT - 1, cur, nxt);
      if (++i == nb) break;
      cur = nxt;
      nxt = lcur_at(i + 1 < nb ? i + 1 : i);
      lstep(I0{}, RF{}, ZY{}, 0, cur, nxt);
    }
  }
  if (wr == 0) DNA_BARRIER();  // re-align the two wave groups
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no LDS-DMA outlives the block
}

// ------------------------------------------------------------------ persistent weight gradient
// dW[Nw][Kw] partial slices: part[c][n][k] = sum_{t in chunk c} dy[t][n] x[t][k], both operands
// token-major ([T][*], as the forward left them: no transposed activation copies). A unit is
// (chunk c, 256x256 tile); units are ordered chunk-major so the blocks of one XCD work on the same
// token chunk at once (dy / x panels shared through L2), and the chunk count s is chosen on the
// host so that the unit count fills the grid evenly. Operands are staged like the [K][N] halves
// of gemm_kernel (64 token rows x 128 columns, 256-B rows, LDS-DMA through buffer resources;
// rows past T read as zeros) and read with ds_read_b64_tr_b16 (read_n). The same 4-phase
// pipeline and role-dependent waits as gemmp_kernel; a quadrant's fp32 partial (QS = 8 16-B
// stores per lane) is written right after its MFMAs in the unit's last K-step. The s slices are
// folded into the fp32 gradient by dna_sum_slices_accum (deterministic order).
struct WArgs {
  const bf16* dy; int ldy;  // [T][Nw]
  const bf16* x; int ldx;   // [T][Kw]
  float* part;              // [s][Nw][Kw]
  int T, Nw, Kw, tilesM, tilesN, s, KTtot;
};

template <bool IMM, int SCH = 0>
__global__ __launch_bounds__(NTHR) void wgradp_kernel(WArgs a) {
  constexpr int QS = 8;
  __shared__ __attribute__((aligned(1024))) char smem[LDS_BYTES];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 2, wc = wave & 3;
  const int G = gridDim.x, b = blockIdx.x;
  const int L = xcd_remap(b, G);  // blocks of one XCD: consecutive units
  const int tiles = a.tilesM * a.tilesN;
  const int U = tiles * a.s;
  const int nb = L < U ? (U - L + G - 1) / G : 0;
  if (nb == 0) return;

  uint32_t voA[2], voB[2];
#pragma unroll
  for (int p = 0; p < 2; ++p) {
    const int r = p * 32 + wave * 4 + (lane >> 4);
    const int ch = ((lane & 15) ^ nswz(r)) * 16;
    voA[p] = (uint32_t)(r * a.ldy * 2 + ch);
    voB[p] = (uint32_t)(r * a.ldx * 2 + ch);
  }

  struct Cur { int i, kt, len, t0, m0, n0, c; };  // kt within the unit, t0 its first K-step
  auto cur_at = [&](int i) {
    Cur c;
    c.i = i;
    c.kt = 0;
    const int u = min(i, nb - 1) * G + L;
    c.c = u / tiles;
    const int tl = u - c.c * tiles;
    c.m0 = (tl / a.tilesN) * BM;
    c.n0 = (tl % a.tilesN) * BN;
    const int s0 = (int)((long long)c.c * a.KTtot / a.s), s1 = (int)((long long)(c.c + 1) * a.KTtot / a.s);
    c.t0 = s0;
    c.len = s1 - s0;
    return c;
  };
  auto advance = [&](Cur& c) {
    if (++c.kt == c.len) c = cur_at(c.i + 1);
  };
  auto img = [&](int v, int h) { return smem + ((v & 1) * 4 + h) * HALF; };
  // one buffer resource per (chunk, operand): base at the chunk's first token row, records up to
  // its last row (or T), so offsets stay 32-bit for any T and rows past T read as zeros
  auto stage = [&](const Cur& c, int v, int h) {
    const int kt = c.i < nb ? c.kt : c.len - 1;
    char* d = img(v, h);
    const bool isA = h < 2;
    const int col0 = isA ? c.m0 + h * 128 : c.n0 + (h - 2) * 128;
    const int ld = isA ? a.ldy : a.ldx;
    const long long r0 = (long long)c.t0 * BK;
    const int rows = min((long long)a.T, (long long)(c.t0 + c.len) * BK) - r0;
    const bf16* base = (isA ? a.dy : a.x) + r0 * ld;
    const auto rs = out_rsrc(base, (uint32_t)((size_t)rows * ld * 2));
    const uint32_t toff = (uint32_t)__builtin_amdgcn_readfirstlane((kt * BK * ld + col0) * 2);
#pragma unroll
    for (int p = 0; p < 2; ++p)  // offset in voffset: token rows past the chunk fail the range check
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_t*)(d + (p * 32 + wave * 4) * 256), 16,
                                               (isA ? voA[p] : voB[p]) + toff, 0, 0, 0);
  };

  f32x4 acc[2][2][4][2];
#pragma unroll
  for (int q = 0; q < 2; ++q)
#pragma unroll
    for (int r = 0; r < 2; ++r)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[q][r][i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  bf16x8 af[4][2], bf0[2][2], bf1[2][2];
  // IMM: per-lane fragment addresses computed once; k-block / row-half steps are instruction
  // immediates (4 address VALU per read group instead of 16)
  uint32_t loA[4], loB[2];
#pragma unroll
  for (int i = 0; i < 4; ++i) loA[i] = read_n_lane_off(wr * 64 + i * 16, lane);
#pragma unroll
  for (int j = 0; j < 2; ++j) loB[j] = read_n_lane_off(wc * 32 + j * 16, lane);
  auto readA = [&](int v, int mq) {
    const char* im = img(v, mq);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      if constexpr (IMM) {
        read_n2(lds_addr(im) + loA[i], af[i][0], af[i][1]);
      } else {
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) af[i][kk] = read_n(im, kk * 32, wr * 64 + i * 16, lane);
      }
    }
  };
  auto readB = [&](int v, int nq, bf16x8 (&bf)[2][2]) {
    const char* im = img(v, 2 + nq);
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      if constexpr (IMM) {
        read_n2(lds_addr(im) + loB[j], bf[j][0], bf[j][1]);
      } else {
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) bf[j][kk] = read_n(im, kk * 32, wc * 32 + j * 16, lane);
      }
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

  const int cq = 4 * (lane >> 4);
  const auto rC = out_rsrc(a.part, (uint32_t)min((size_t)a.s * a.Nw * a.Kw * 4, (size_t)0xFFFFFFF0u));
  const uint32_t voC = (uint32_t)(((wr * 64 + (lane & 15)) * a.Kw + wc * 32 + cq) * 4);
  auto store_quadrant = [&](const Cur& c, int mq, int nq) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const uint32_t toff = (uint32_t)__builtin_amdgcn_readfirstlane(
          (int)((((size_t)c.c * a.Nw + c.m0 + mq * 128 + i * 16) * a.Kw + c.n0 + nq * 128) * 4));
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, acc[mq][nq][i][j]), rC,
                                               voC + toff + j * 64, 0, 0);
        acc[mq][nq][i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
      }
    }
  };

  Cur c0 = cur_at(0), c1 = c0, c2 = c0;
  advance(c1);
  advance(c2);
  advance(c2);
  if constexpr (SCH == 0) {
  stage(c0, 0, 0);
  stage(c0, 0, 2);
  stage(c0, 0, 3);
  stage(c0, 0, 1);
  stage(c1, 1, 0);
  stage(c1, 1, 2);
  __builtin_amdgcn_s_waitcnt(waitcnt_imm(8));
  DNA_BARRIER();
  if (wr == 1) DNA_BARRIER();

  auto wait_vm = [&](auto phase, int role) {
    constexpr int p = decltype(phase)::value;
    if (role == 0) __builtin_amdgcn_s_waitcnt(waitcnt_imm(8));
    else if (role == 1) __builtin_amdgcn_s_waitcnt(waitcnt_imm(8 + p * QS));
    else __builtin_amdgcn_s_waitcnt(waitcnt_imm(8 + (4 - p) * QS));
  };
  using P0 = std::integral_constant<int, 0>;
  using P1 = std::integral_constant<int, 1>;
  using P2 = std::integral_constant<int, 2>;
  using P3 = std::integral_constant<int, 3>;
  auto kstep = [&](int v, int role) {
    const bool st = role == 1;
    stage(c1, v + 1, 3);
    wait_vm(P0{}, role);
    readA(v, 0);
    readB(v, 0, bf0);
    DNA_BARRIER();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    mma(0, 0, bf0);
    if (st) store_quadrant(c0, 0, 0);
    DNA_BARRIER();
    stage(c1, v + 1, 1);
    wait_vm(P1{}, role);
    readB(v, 1, bf1);
    DNA_BARRIER();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    mma(0, 1, bf1);
    if (st) store_quadrant(c0, 0, 1);
    DNA_BARRIER();
    stage(c2, v + 2, 0);
    wait_vm(P2{}, role);
    readA(v, 1);
    DNA_BARRIER();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    mma(1, 1, bf1);
    if (st) store_quadrant(c0, 1, 1);
    DNA_BARRIER();
    stage(c2, v + 2, 2);
    wait_vm(P3{}, role);
    DNA_BARRIER();
    mma(1, 0, bf0);
    if (st) store_quadrant(c0, 1, 0);
    DNA_BARRIER();
  };

  int v = 0;
  for (int i = 0; i < nb; ++i) {
    for (int kt = 0; kt < c0.len; ++kt, ++v) {
      const int role = kt == c0.len - 1 ? 1 : (kt == 0 && i > 0) ? 2 : 0;
      kstep(v, role);
      advance(c1);
      advance(c2);
    }
    c0 = cur_at(i + 1);
  }
  } else if constexpr (SCH == 1) {
    // SCH == 1: gemmp_kernel's balanced-read schedule (reads A_0 / B_1 / A_1 / B_0(next) per
    // phase, 5 half-tiles in flight; see there). Units have per-chunk lengths, so the current
    // unit's last K-step starts at phase 4 * (len - 1).
    constexpr int hA0 = 0, hA1 = 1, hB0 = 2, hB1 = 3;
    auto wait_p = [&](auto phase, int role) {
      constexpr int p = decltype(phase)::value;
      if (role == 0) __builtin_amdgcn_s_waitcnt(waitcnt_imm(10));
      else if (role == 1) __builtin_amdgcn_s_waitcnt(waitcnt_imm(10 + pend_stores<EPI_F32>(1, p)));
      else if (role == 2) __builtin_amdgcn_s_waitcnt(waitcnt_imm(10 + pend_stores<EPI_F32>(2, p)));
      else if (role == 3) __builtin_amdgcn_s_waitcnt(waitcnt_imm(10 + pend_stores<EPI_F32>(3, p)));
      else __builtin_amdgcn_s_waitcnt(waitcnt_imm(10 + pend_stores<EPI_F32>(4, p)));
    };
    auto lgkm0 = [&]() {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
    };
    auto step = [&](int v, int kt, bool prev, bf16x8 (&bB0)[2][2], bf16x8 (&bB1)[2][2]) {
      const bool st = kt == c0.len - 1;
      const int role = __builtin_amdgcn_readfirstlane(
          st ? (prev && kt == 1 ? 4 : 3) : prev && kt == 0 ? 1 : prev && kt == 1 ? 2 : 0);
      stage(c1, v + 1, hA1);
      wait_p(std::integral_constant<int, 0>{}, role);
      readA(v, 0);
      DNA_BARRIER();
      lgkm0();
      mma(0, 0, bB0);
      if (st) store_quadrant(c0, 0, 0);
      DNA_BARRIER();
      stage(c2, v + 2, hB0);
      wait_p(std::integral_constant<int, 1>{}, role);
      readB(v, 1, bB1);
      DNA_BARRIER();
      lgkm0();
      mma(0, 1, bB1);
      if (st) store_quadrant(c0, 0, 1);
      DNA_BARRIER();
      stage(c2, v + 2, hA0);
      wait_p(std::integral_constant<int, 2>{}, role);
      readA(v, 1);
      DNA_BARRIER();
      lgkm0();
      mma(1, 1, bB1);
      if (st) store_quadrant(c0, 1, 1);
      DNA_BARRIER();
      stage(c2, v + 2, hB1);
      wait_p(std::integral_constant<int, 3>{}, role);
      readB(v + 1, 0, bB1);
      DNA_BARRIER();
      lgkm0();
      mma(1, 0, bB0);
      if (st) store_quadrant(c0, 1, 0);
      DNA_BARRIER();
    };
    stage(c0, 0, hB0);
    stage(c0, 0, hA0);
    stage(c0, 0, hB1);
    stage(c0, 0, hA1);
    stage(c1, 1, hB0);
    stage(c1, 1, hA0);
    stage(c1, 1, hB1);
    __builtin_amdgcn_s_waitcnt(waitcnt_imm(10));
    DNA_BARRIER();
    readB(0, 0, bf0);
    if (wr == 1) DNA_BARRIER();
    int kt = 0, i = 0;
    const int V = [&]() {  // K-steps of this block's units
      int n = 0;
      for (int j = 0; j < nb; ++j) n += cur_at(j).len;
      return n;
    }();
    auto next = [&]() {
      advance(c1);
      advance(c2);
      if (++kt == c0.len) {
        kt = 0;
        ++i;
        c0 = cur_at(i);
      }
    };
    for (int v = 0; v < V; v += 2) {
      step(v, kt, i > 0, bf0, bf1);
      next();
      if (v + 1 < V) {
        step(v + 1, kt, i > 0, bf1, bf0);
        next();
      }
    }
  } else {
    // SCH == 2: the lean form of the SCH 0 schedule (see gemmp_kernel's SCH == 2): K-steps
    // unrolled by two with compile-time buffer parity, fragment reads off per-lane base
    // registers with immediate offsets, per-unit stage offsets and buffer resources computed once
    // per unit, compile-time wait roles. Chunks are whole K-step pairs (WArgs.pairs), so every
    // unit starts on parity 0.
    uint32_t bA[2][4], bB[2][2];
    const uint32_t sbase = lds_addr(smem);
#pragma unroll
    for (int par = 0; par < 2; ++par) {
#pragma unroll
      for (int i = 0; i < 4; ++i) bA[par][i] = sbase + par * 4 * HALF + loA[i];
#pragma unroll
      for (int j = 0; j < 2; ++j) bB[par][j] = sbase + par * 4 * HALF + 2 * HALF + loB[j];
    }
    struct WCur { const bf16 *pA, *pB; uint32_t nA, nB; int len, m0, n0, c; };
    auto wcur_at = [&](int i) {
      WCur w;
      const int u = i * G + L;
      w.c = u / tiles;
      const int tl = u - w.c * tiles;
      w.m0 = (tl / a.tilesN) * BM;
      w.n0 = (tl % a.tilesN) * BN;
      const int KP = a.KTtot >> 1;
      const int s0 = 2 * (int)((long long)w.c * KP / a.s), s1 = 2 * (int)((long long)(w.c + 1) * KP / a.s);
      w.len = s1 - s0;
      const long long r0 = (long long)s0 * BK;
      const int rows = (int)(min((long long)a.T, (long long)s1 * BK) - r0);
      w.pA = a.dy + r0 * a.ldy;
      w.pB = a.x + r0 * a.ldx;
      w.nA = (uint32_t)((size_t)rows * a.ldy * 2);
      w.nB = (uint32_t)((size_t)rows * a.ldx * 2);
      return w;
    };
    // stage half h of K-step k of the current unit (k >= len: step k - len of the next unit)
    auto wstage = [&](const WCur& cur, const WCur& nxt, int k, auto par_c, auto h_c) {
      constexpr int par = decltype(par_c)::value, h = decltype(h_c)::value;
      constexpr bool isA = h < 2;
      const bool in = k < cur.len;
      const int kk = in ? k : k - cur.len;
      const int col0 = isA ? (in ? cur.m0 : nxt.m0) + h * 128 : (in ? cur.n0 : nxt.n0) + (h - 2) * 128;
      const int ld = isA ? a.ldy : a.ldx;
      const bf16* base = isA ? (in ? cur.pA : nxt.pA) : (in ? cur.pB : nxt.pB);
      const uint32_t bytes = isA ? (in ? cur.nA : nxt.nA) : (in ? cur.nB : nxt.nB);
      const uint32_t toff = (uint32_t)__builtin_amdgcn_readfirstlane((kk * BK * ld + col0) * 2);
      char* d = smem + (par * 4 + h) * HALF;
#pragma unroll
      for (int p = 0; p < 2; ++p)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(out_rsrc(base, bytes), (lds_t*)(d + (p * 32 + wave * 4) * 256),
                                                 16, (isA ? voA[p] : voB[p]) + toff, 0, 0, 0);
    };
    auto rd2 = [](uint32_t addr, auto off_c, bf16x8& k0, bf16x8& k1) {
      constexpr int off = decltype(off_c)::value;
      const bf16x4 x0 = tr_read_imm<off>(addr), x1 = tr_read_imm<off + 1024>(addr);
      const bf16x4 x2 = tr_read_imm<off + 8192>(addr), x3 = tr_read_imm<off + 9216>(addr);
      k0 = bf16x8{x0[0], x0[1], x0[2], x0[3], x1[0], x1[1], x1[2], x1[3]};
      k1 = bf16x8{x2[0], x2[1], x2[2], x2[3], x3[0], x3[1], x3[2], x3[3]};
    };
    auto wreadA = [&](auto par_c, auto mq_c) {
      constexpr int par = decltype(par_c)::value, mq = decltype(mq_c)::value;
      using O = std::integral_constant<int, mq * HALF>;
      rd2(bA[par][0], O{}, af[0][0], af[0][1]);
      rd2(bA[par][1], O{}, af[1][0], af[1][1]);
      rd2(bA[par][2], O{}, af[2][0], af[2][1]);
      rd2(bA[par][3], O{}, af[3][0], af[3][1]);
    };
    auto wreadB = [&](auto par_c, auto nq_c, bf16x8 (&bf)[2][2]) {
      constexpr int par = decltype(par_c)::value, nq = decltype(nq_c)::value;
      using O = std::integral_constant<int, nq * HALF>;
      rd2(bB[par][0], O{}, bf[0][0], bf[0][1]);
      rd2(bB[par][1], O{}, bf[1][0], bf[1][1]);
    };
    auto wstore = [&](const WCur& w, int mq, int nq) __attribute__((always_inline)) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const uint32_t toff = (uint32_t)__builtin_amdgcn_readfirstlane(
            (int)((((size_t)w.c * a.Nw + w.m0 + mq * 128 + i * 16) * a.Kw + w.n0 + nq * 128) * 4));
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, acc[mq][nq][i][j]), rC,
                                                 voC + toff + j * 64, 0, 0);
        }
      }
    };
    auto& mma_acc = mma;
    auto mmaz = [&](int mq, int nq, const bf16x8 (&bf)[2][2]) {
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[mq][nq][i][j] = mfma(bf[j][0], af[i][0], f32x4{0.f, 0.f, 0.f, 0.f});
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[mq][nq][i][j] = mfma(bf[j][1], af[i][1], acc[mq][nq][i][j]);
      __builtin_amdgcn_s_setprio(0);
    };
    auto wwait = [&](auto phase_c, auto role_c) {
      constexpr int p = decltype(phase_c)::value, role = decltype(role_c)::value;
      constexpr int n = role == 0 ? 8 : role == 1 ? 8 + p * QS : 8 + (4 - p) * QS;
      __builtin_amdgcn_s_waitcnt(waitcnt_imm(n));
    };
    auto lgkm0 = [&]() {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
    };
    using I0 = std::integral_constant<int, 0>;
    using I1 = std::integral_constant<int, 1>;
    using I2 = std::integral_constant<int, 2>;
    using I3 = std::integral_constant<int, 3>;
    auto wstep = [&](auto par_c, auto role_c, auto zi_c, int k, const WCur& cur, const WCur& nxt) {
      constexpr int par = decltype(par_c)::value, role = decltype(role_c)::value;
      constexpr bool ZI = decltype(zi_c)::value;
      using Pc = std::integral_constant<int, par>;
      using Qc = std::integral_constant<int, par ^ 1>;
      auto mma = [&](int mq, int nq, const bf16x8 (&bf)[2][2]) {
        if constexpr (ZI) mmaz(mq, nq, bf);
        else mma_acc(mq, nq, bf);
      };
      wstage(cur, nxt, k + 1, Qc{}, I3{});
      wwait(I0{}, role_c);
      wreadA(Pc{}, I0{});
      wreadB(Pc{}, I0{}, bf0);
      DNA_BARRIER();
      lgkm0();
      mma(0, 0, bf0);
      if constexpr (role == 1) wstore(cur, 0, 0);
      DNA_BARRIER();
      wstage(cur, nxt, k + 1, Qc{}, I1{});
      wwait(I1{}, role_c);
      wreadB(Pc{}, I1{}, bf1);
      DNA_BARRIER();
      lgkm0();
      mma(0, 1, bf1);
      if constexpr (role == 1) wstore(cur, 0, 1);
      DNA_BARRIER();
      wstage(cur, nxt, k + 2, Pc{}, I0{});
      wwait(I2{}, role_c);
      wreadA(Pc{}, I1{});
      DNA_BARRIER();
      lgkm0();
      mma(1, 1, bf1);
      if constexpr (role == 1) wstore(cur, 1, 1);
      DNA_BARRIER();
      wstage(cur, nxt, k + 2, Pc{}, I2{});
      wwait(I3{}, role_c);
      DNA_BARRIER();
      mma(1, 0, bf0);
      if constexpr (role == 1) wstore(cur, 1, 0);
      DNA_BARRIER();
    };
    using R0 = std::integral_constant<int, 0>;
    using RL = std::integral_constant<int, 1>;
    using RF = std::integral_constant<int, 2>;
    WCur cur = wcur_at(0), nxt = wcur_at(nb > 1 ? 1 : 0);
    wstage(cur, nxt, 0, I0{}, I0{});
    wstage(cur, nxt, 0, I0{}, I2{});
    wstage(cur, nxt, 0, I0{}, I3{});
    wstage(cur, nxt, 0, I0{}, I1{});
    wstage(cur, nxt, 1, I1{}, I0{});
    wstage(cur, nxt, 1, I1{}, I2{});
    __builtin_amdgcn_s_waitcnt(waitcnt_imm(8));
    DNA_BARRIER();
    if (wr == 1) DNA_BARRIER();
    using ZN = std::false_type;
    using ZY = std::true_type;
    wstep(I0{}, R0{}, ZY{}, 0, cur, nxt);
    for (int i = 0;;) {
      for (int k = 1; k < cur.len - 1; k += 2) {
        wstep(I1{}, R0{}, ZN{}, k, cur, nxt);
        wstep(I0{}, R0{}, ZN{}, k + 1, cur, nxt);
      }
      wstep(I1{}, RL{}, ZN{}, cur.len - 1, cur, nxt);
      if (++i == nb) break;
      cur = nxt;
      nxt = wcur_at(i + 1 < nb ? i + 1 : i);
      wstep(I0{}, RF{}, ZY{}, 0, cur, nxt);
    }
  }
  if (wr == 0) DNA_BARRIER();
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
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


inline int num_cus() {
  static int n = 0;
  if (n == 0) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
      n = 256;
  }
  return n;
}

inline bool persistent_enabled() {
  static int on = -1;
  if (on < 0) {
    const char* e = getenv("DNA_GEMM_P");
    on = (e && e[0] == '0') ? 0 : 1;
  }
  return on == 1;
}

// persistent-kernel half-tile schedule (DNA_GEMM_SCHED, read per call for in-process A/B):
// 2 (default) = the lean K-step body, 0 = the original one, 1 = balanced reads (slower)
inline int gemm_sched() {
  const char* e = getenv("DNA_GEMM_SCHED");
  return e ? atoi(e) : 2;
}

template <int EPI>
int launchp(Args& a, hipStream_t s, const char* name) {
  a.tilesM = (a.M + BM - 1) / BM;
  const int nper = (EPI == EPI_GEGLU ? BN / 2 : BN);
  a.tilesN = (a.N + nper - 1) / nper;
  if (const char* e = getenv("DNA_GEMM_GM")) a.GM = atoi(e);
  if (a.GM <= 0) a.GM = 8;
  const int U = a.tilesM * a.tilesN;
  int G = num_cus();
  if (const char* e = getenv("DNA_GEMM_GRID")) G = atoi(e);
  G = U < G ? U : (G & ~7);
  a.rot = 0;
  if (const char* e = getenv("DNA_GEMM_ROT")) a.rot = atoi(e);
  a.dbg = 0;
  if (const char* e = getenv("DNA_GEMM_DBG")) a.dbg = atoi(e);
  a.nt = 0;
  if (const char* e = getenv("DNA_GEMM_NT")) a.nt = atoi(e);
  a.order = 0;
  if (const char* e = getenv("DNA_GEMM_ORDER")) a.order = atoi(e);
  if constexpr (EPI == EPI_BF16_GELU) {  // lean body only (K / BK even: the launcher checks)
    hipLaunchKernelGGL((gemmp_kernel<EPI, 0, 2>), dim3(G), dim3(NTHR), 0, s, a);
  } else {
    const char* ab = getenv("DNA_GEMM_ABL");
    const int abl = ab ? atoi(ab) : 0;
    if (abl == 0 && gemm_sched() == 1) hipLaunchKernelGGL((gemmp_kernel<EPI, 0, 1>), dim3(G), dim3(NTHR), 0, s, a);
    else if (abl == 0 && gemm_sched() == 2 && (a.K / BK) % 2 == 0)
      hipLaunchKernelGGL((gemmp_kernel<EPI, 0, 2>), dim3(G), dim3(NTHR), 0, s, a);
    else if (abl == 1) hipLaunchKernelGGL((gemmp_kernel<EPI, 1>), dim3(G), dim3(NTHR), 0, s, a);
    else if (abl == 2) hipLaunchKernelGGL((gemmp_kernel<EPI, 2>), dim3(G), dim3(NTHR), 0, s, a);
    else if (abl == 3) hipLaunchKernelGGL((gemmp_kernel<EPI, 3>), dim3(G), dim3(NTHR), 0, s, a);
    else if (abl == 7) hipLaunchKernelGGL((gemmp_kernel<EPI, 7>), dim3(G), dim3(NTHR), 0, s, a);
    else if (abl == 8) hipLaunchKernelGGL((gemmp_kernel<EPI, 8>), dim3(G), dim3(NTHR), 0, s, a);
    else if (abl == 16) hipLaunchKernelGGL((gemmp_kernel<EPI, 16>), dim3(G), dim3(NTHR), 0, s, a);
    else if (abl == 32) hipLaunchKernelGGL((gemmp_kernel<EPI, 32>), dim3(G), dim3(NTHR), 0, s, a);
    else hipLaunchKernelGGL((gemmp_kernel<EPI>), dim3(G), dim3(NTHR), 0, s, a);
  }
  DNA_LAUNCH_CHECK(name);
  return DNA_OK;
}


// chunk count for dna_linear_wgrad_p: minimise the modelled time in K-step units --
//   ceil(tiles*s / G) rounds x (KTtot/s steps + ~3 steps of per-unit store tail)
//   + the fp32 partial round trip of the slice sum (s*N*K*8 bytes at ~6 TB/s, ~1.6 us a step)
// with each chunk >= 4 K-steps and s <= 64
inline int wgrad_chunks(int tiles, int KTtot, int G, double nk) {
  int best = 1;
  double best_cost = 1e30;
  for (int s = 1; s <= 64 && KTtot / s >= 4; ++s) {
    const int rounds = (tiles * s + G - 1) / G;
    const double cost = rounds * ((double)KTtot / s + 3.0) + s * nk * 8.0 / (6e12 * 1.6e-6);
    if (cost < best_cost - 1e-9) { best_cost = cost; best = s; }
  }
  return best;
}

// Row-block size for an operand past 32-bit byte offsets: the fewest blocks of at most `cap` rows
// (cap a multiple of the 256-row tile), split as evenly as the tile allows -- so every launch
// gets about the same unit count (a max-size-first split left the K = 6144 data gradient's second
// launch 4.01 rounds of units: a fifth round with 2 units, ~0.1 ms of idle chip per call)
inline int row_block(int M, int cap) {
  const int nblk = (M + cap - 1) / cap;
  const int per = (M + nblk - 1) / nblk;
  return (per + BM - 1) / BM * BM;
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
  if (persistent_enabled() && N <= BIAS_LDS / 4 && N % BN == 0 && K >= 2 * BK &&
      (size_t)N * K * 2 < (1ull << 31)) {
    // the persistent kernel addresses an operand with 32-bit byte offsets: row blocks of at most
    // mc rows (a multiple of the 256-row tile) per launch, so e.g. T = 262,144 tokens (b = 512)
    // at N = 6144 runs as two launches of the b = 256 shape instead of the non-persistent kernel
    const size_t wide = (size_t)(K > N ? K : N) * 2;
    const int cap = (int)(((1ull << 31) - 1) / wide / BM * BM);
    if (cap >= BM) {
      const int mc = row_block(M, cap);
      for (int r0 = 0; r0 < M; r0 += mc) {
        Args c = a;
        c.A = a.A + (size_t)r0 * K;
        c.C = (bf16*)a.C + (size_t)r0 * N;
        c.M = M - r0 < mc ? M - r0 : mc;
        const int st = launchp<EPI_BF16>(c, as_stream(stream), "dna_linear_fwd");
        if (st != DNA_OK) return st;
      }
      return DNA_OK;
    }
  }
  return launch<true, true, EPI_BF16>(a, 1, as_stream(stream), "dna_linear_fwd");
}

extern "C" int dna_linear_gelu_fwd(const void* x, const void* w, const float* bias, int M, int N,
                                   int K, void* h, void* act, void* stream) {
  DNA_CHECK_ARG(x && w && h && act, "dna_linear_gelu_fwd: null pointer");
  DNA_CHECK_ARG(M >= 0 && N > 0 && K > 0, "dna_linear_gelu_fwd: bad shape");
  // the persistent kernel's lean body only: N a multiple of the 256-column tile with its bias in
  // LDS, an even number of 64-deep K-steps, the weight under 2 GB (32-bit offsets)
  DNA_CHECK_ARG(N % BN == 0 && N <= BIAS_LDS / 4 && K % (2 * BK) == 0 &&
                    (size_t)N * K * 2 < (1ull << 31),
                "dna_linear_gelu_fwd: N %% 256 (<= %d) and K %% 128 required (N=%d K=%d)",
                BIAS_LDS / 4, N, K);
  if (M == 0) return DNA_OK;
  Args a = base_args();
  a.A = (const bf16*)x; a.lda = K;
  a.B = (const bf16*)w; a.ldb = K;
  a.C = h; a.ldc = N; a.bias = bias; a.aux = (bf16*)act;
  a.M = M; a.N = N; a.K = K; a.ksplit = K;
  const size_t wide = (size_t)(K > N ? K : N) * 2;
  const int cap = (int)(((1ull << 31) - 1) / wide / BM * BM);
  const int mc = row_block(M, cap);
  for (int r0 = 0; r0 < M; r0 += mc) {
    Args c = a;
    c.A = a.A + (size_t)r0 * K;
    c.C = (bf16*)a.C + (size_t)r0 * N;
    c.aux = a.aux + (size_t)r0 * N;
    c.M = M - r0 < mc ? M - r0 : mc;
    const int st = launchp<EPI_BF16_GELU>(c, as_stream(stream), "dna_linear_gelu_fwd");
    if (st != DNA_OK) return st;
  }
  return DNA_OK;
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
                                    int K, float p_drop, uint64_t seed, uint64_t offset, void* fac,
                                    void* out, void* stream) {
  DNA_CHECK_ARG(x && w && fac && out, "dna_geglu_linear_fwd: null pointer");
  void* g = fac;  // the backward factors take g's place (same layout, [M][2F])
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
  if (persistent_enabled() && 2 * F <= BIAS_LDS / 4 && K >= 2 * BK && (size_t)2 * F * K * 2 < (1ull << 31)) {
    // 32-bit byte offsets: row blocks of at most mc rows per launch (see dna_linear_fwd)
    const size_t wide = (size_t)(K > 2 * F ? K : 2 * F) * 2;
    const int cap = (int)(((1ull << 31) - 1) / wide / BM * BM);
    if (cap >= BM) {
      const int mc = row_block(M, cap);
      for (int r0 = 0; r0 < M; r0 += mc) {
        Args c = a;
        c.A = a.A + (size_t)r0 * K;
        c.C = (bf16*)a.C + (size_t)r0 * 2 * F;
        c.aux = a.aux + (size_t)r0 * F;
        c.M = M - r0 < mc ? M - r0 : mc;
        c.off = a.off + (uint64_t)r0 * F / 8;  // dropout groups of 8 elements, row-major
        const int st = launchp<EPI_GEGLU>(c, as_stream(stream), "dna_geglu_linear_fwd");
        if (st != DNA_OK) return st;
      }
      return DNA_OK;
    }
  }
  return launch<true, true, EPI_GEGLU>(a, 1, as_stream(stream), "dna_geglu_linear_fwd");
}

extern "C" int dna_geglu_linear_dgrad(const void* dy, const void* w, const void* fac, int M, int F,
                                      int N, void* dg, void* stream) {
  DNA_CHECK_ARG(dy && w && fac && dg, "dna_geglu_linear_dgrad: null pointer");
  const void* g = fac;
  DNA_CHECK_ARG(M >= 0 && N % BK == 0 && F % 8 == 0,
                "dna_geglu_linear_dgrad: hidden %% 64 and F %% 8 required (N=%d F=%d)", N, F);
  if (M == 0) return DNA_OK;
  Args a = base_args();
  a.A = (const bf16*)dy; a.lda = N;
  a.B = (const bf16*)w; a.ldb = F;
  a.C = nullptr; a.ldc = F; a.g = (const bf16*)g; a.aux = (bf16*)dg;
  a.M = M; a.N = F; a.K = N; a.ksplit = N; a.F = F;
  return launch<true, false, EPI_GEGLU_BWD>(a, 1, as_stream(stream), "dna_geglu_linear_dgrad");
}

// dg[M, 2F] = bf16(dy[M, N] . Wt[F, N]^T) * fac on the persistent kernel: the data gradient of
// `wo` through its transposed bf16 copy (both operands K-major, as dna_linear_fwd's dgrad use),
// with the GeGLU backward of bert_layers.py:292-296 in the epilogue (fac = the forward's
// factors, dropout folded in); da never reaches memory. Row blocks past 2^31-byte operands as
// dna_geglu_linear_fwd.
extern "C" int dna_geglu_linear_dgrad_p(const void* dy, const void* wt, const void* fac, int M,
                                        int F, int N, void* dg, void* stream) {
  DNA_CHECK_ARG(dy && wt && fac && dg, "dna_geglu_linear_dgrad_p: null pointer");
  DNA_CHECK_ARG(M >= 0 && N % BK == 0 && (N / BK) % 2 == 0 && N >= 2 * BK && F % BN == 0,
                "dna_geglu_linear_dgrad_p: hidden %% 128 and F %% 256 required (N=%d F=%d)", N, F);
  const void* g = fac;
  DNA_CHECK_ARG((size_t)F * N * 2 < (1ull << 31), "dna_geglu_linear_dgrad_p: weight too large");
  if (M == 0) return DNA_OK;
  Args a = base_args();
  a.A = (const bf16*)dy; a.lda = N;
  a.B = (const bf16*)wt; a.ldb = N;
  a.C = nullptr; a.ldc = 2 * F; a.g = (const bf16*)g; a.aux = (bf16*)dg;
  a.N = F; a.K = N; a.ksplit = N; a.F = F;
  // DNA_GEMM_ABL=128 (timing-only diagnostic, results invalid): the epilogue without the
  // factor loads
  const char* ab = getenv("DNA_GEMM_ABL");
  const int abl = ab ? atoi(ab) : 0;
  a.tilesN = F / BN;
  a.GM = 8;
  if (const char* e = getenv("DNA_GEMM_GM")) a.GM = atoi(e);
  const size_t wide = (size_t)(N > 2 * F ? N : 2 * F) * 2;
  const int cap = (int)(((1ull << 31) - 1) / wide / BM * BM);
  DNA_CHECK_ARG(cap >= BM, "dna_geglu_linear_dgrad_p: rows of %zu bytes exceed 32-bit offsets", wide);
  const int mc = row_block(M, cap);
  for (int r0 = 0; r0 < M; r0 += mc) {
    Args c = a;
    c.A = a.A + (size_t)r0 * N;
    c.g = a.g + (size_t)r0 * 2 * F;
    c.aux = a.aux + (size_t)r0 * 2 * F;
    c.M = M - r0 < mc ? M - r0 : mc;
    c.tilesM = (c.M + BM - 1) / BM;
    const int U = c.tilesM * c.tilesN;
    int G = num_cus();
    G = U < G ? U : (G & ~7);
    if (abl == 128) hipLaunchKernelGGL((gemmp_kernel<EPI_GEGLU_BWD, 128, 2>), dim3(G), dim3(NTHR), 0, as_stream(stream), c);
    else hipLaunchKernelGGL((gemmp_kernel<EPI_GEGLU_BWD, 0, 2>), dim3(G), dim3(NTHR), 0, as_stream(stream), c);
    DNA_LAUNCH_CHECK("dna_geglu_linear_dgrad_p");
  }
  return DNA_OK;
}

// dh = gelu_tanh'(h) * (dy . W) for the Mlp's fc2 (HyenaDNA Block, flash_attn Mlp with
// activation gelu approximate="tanh"): the data gradient of fc2 through the transposed weight
// copy wt [F][N] with the GELU backward in the epilogue (da never stored). dy [M][N], h / dh [M][F].
extern "C" int dna_gelu_linear_dgrad_p(const void* dy, const void* wt, const void* h, int M, int F,
                                       int N, void* dh, void* stream) {
  DNA_CHECK_ARG(dy && wt && h && dh, "dna_gelu_linear_dgrad_p: null pointer");
  DNA_CHECK_ARG(M >= 0 && N % BK == 0 && (N / BK) % 2 == 0 && N >= 2 * BK && F % BN == 0,
                "dna_gelu_linear_dgrad_p: N %% 128 and F %% 256 required (N=%d F=%d)", N, F);
  DNA_CHECK_ARG((size_t)F * N * 2 < (1ull << 31), "dna_gelu_linear_dgrad_p: weight too large");
  if (M == 0) return DNA_OK;
  Args a = base_args();
  a.A = (const bf16*)dy; a.lda = N;
  a.B = (const bf16*)wt; a.ldb = N;
  a.C = nullptr; a.ldc = F; a.g = (const bf16*)h; a.aux = (bf16*)dh;
  a.N = F; a.K = N; a.ksplit = N; a.F = F;
  a.p = 0.f;
  a.tilesN = F / BN;
  a.GM = 8;
  if (const char* e = getenv("DNA_GEMM_GM")) a.GM = atoi(e);
  const size_t wide = (size_t)(N > F ? N : F) * 2;
  const int cap = (int)(((1ull << 31) - 1) / wide / BM * BM);
  DNA_CHECK_ARG(cap >= BM, "dna_gelu_linear_dgrad_p: rows of %zu bytes exceed 32-bit offsets", wide);
  const int mc = row_block(M, cap);
  for (int r0 = 0; r0 < M; r0 += mc) {
    Args c = a;
    c.A = a.A + (size_t)r0 * N;
    c.g = a.g + (size_t)r0 * F;
    c.aux = a.aux + (size_t)r0 * F;
    c.M = M - r0 < mc ? M - r0 : mc;
    c.tilesM = (c.M + BM - 1) / BM;
    const int U = c.tilesM * c.tilesN;
    int G = num_cus();
    G = U < G ? U : (G & ~7);
    hipLaunchKernelGGL((gemmp_kernel<EPI_GELU_BWD, 0, 2>), dim3(G), dim3(NTHR), 0, as_stream(stream), c);
    DNA_LAUNCH_CHECK("dna_gelu_linear_dgrad_p");
  }
  return DNA_OK;
}

extern "C" int dna_linear_wgrad_p_splits(int M, int N, int K) {
  if (M <= 0 || N % BM || K % BN) return 1;
  return wgrad_chunks((N / BM) * (K / BN), (M + BK - 1) / BK, num_cus() & ~7, (double)N * K);
}

extern "C" int dna_linear_wgrad_p(const void* dy, const void* x, int M, int N, int K, int splits,
                                  float* partials, void* stream) {
  DNA_CHECK_ARG(dy && x && partials, "dna_linear_wgrad_p: null pointer");
  DNA_CHECK_ARG(M > 0 && N % BM == 0 && K % BN == 0,
                "dna_linear_wgrad_p: N, K %% 256 required (N=%d K=%d)", N, K);
  const int KTtot = (M + BK - 1) / BK;
  DNA_CHECK_ARG(splits >= 1 && KTtot / splits >= 2, "dna_linear_wgrad_p: bad splits %d", splits);
  DNA_CHECK_ARG((size_t)((KTtot + splits - 1) / splits) * BK * (N > K ? N : K) * 2 < (1ull << 31) &&
                    (size_t)splits * N * K * 4 < (1ull << 32),
                "dna_linear_wgrad_p: chunks / partials too large for 32-bit buffer offsets");
  WArgs a{};
  a.dy = (const bf16*)dy; a.ldy = N;
  a.x = (const bf16*)x; a.ldx = K;
  a.part = partials;
  a.T = M; a.Nw = N; a.Kw = K;
  a.tilesM = N / BM; a.tilesN = K / BN; a.s = splits; a.KTtot = KTtot;
  const int U = a.tilesM * a.tilesN * splits;
  int G = num_cus() & ~7;
  G = U < G ? U : G;
  const char* ie = getenv("DNA_WGRAD_IMM");  // A/B: 0 = per-read address VALU
  // the lean kernel works in K-step pairs: an odd step count (e.g. the MLM head's masked rows)
  // gets one more step past T, which reads zeros (rows past T lie outside the chunk resources)
  const int KTe = KTtot + (KTtot & 1);
  const bool pairs_ok = KTe / 2 / splits >= 1 &&
                        (size_t)((KTe / 2 + splits - 1) / splits) * 2 * BK * (N > K ? N : K) * 2 < (1ull << 31);
  if (gemm_sched() == 2 && pairs_ok && (!ie || atoi(ie) != 0)) {
    a.KTtot = KTe;
    hipLaunchKernelGGL((wgradp_kernel<true, 2>), dim3(G), dim3(NTHR), 0, as_stream(stream), a);
  }
  else if (gemm_sched() == 1 && (!ie || atoi(ie) != 0))
    hipLaunchKernelGGL((wgradp_kernel<true, 1>), dim3(G), dim3(NTHR), 0, as_stream(stream), a);
  else if (!ie || atoi(ie) != 0)
    hipLaunchKernelGGL(wgradp_kernel<true>, dim3(G), dim3(NTHR), 0, as_stream(stream), a);
  else
    hipLaunchKernelGGL(wgradp_kernel<false>, dim3(G), dim3(NTHR), 0, as_stream(stream), a);
  DNA_LAUNCH_CHECK("dna_linear_wgrad_p");
  return DNA_OK;
}
