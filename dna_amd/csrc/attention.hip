// Fused ALiBi + key-pad attention for DNABERT-2 (MosaicBERT), forward and backward, gfx950.
//
// Replaces bert_layers.py:160-196 (PyTorch attention with an fp32 [b,H,S,S] bias built at
// :421-448) and the disabled Triton slot flash_attn_triton.py:1077-1130. Scores never leave the
// CU: S = Q K^T * scale + bias with bias[h,i,j] = -slope_h*|i-j| + (key j is pad ? -10000 : 0)
// computed in registers, online softmax in log2 domain, P V on MFMA.
//
// bf16 path (head_dim 64): MFMA v_mfma_f32_32x32x16_bf16. A workgroup = 4 waves = 128 queries
// of one (batch, head); each wave owns 32 queries and sweeps the keys in tiles of 64 staged in
// LDS (K XOR-swizzled for conflict-free ds_read_b128 row reads; V read transposed with
// ds_read_b64_tr_b16). The "swapped" products keep the query on the MFMA lane:
//   S^T[key][q] = K . Q^T       (A = K rows from LDS, B = Q held in registers)
//   O^T[d][q]  += V^T . P^T     (A = V^T via tr reads, B = P^T straight from the accumulator)
// so the softmax statistics of a query live in one lane pair (lane, lane^32).
// Backward: dQ kernel (queries on lanes, like forward) and dK/dV kernel (keys on lanes, sweeping
// query tiles), both recomputing P from the forward LSE -- no atomics, deterministic.
//
// fp32 path: exact-arithmetic reference-grade kernels (one thread per query / key) used for the
// 1e-3 fp32 parity mode; not a throughput path.
#include <stdlib.h>

#include <algorithm>
#include <type_traits>

#include "common.h"

namespace dna {
namespace attn {

constexpr int D = 64;       // head dim
constexpr int BQ = 128;     // queries per workgroup (4 waves x 32)
constexpr int BK = 64;      // keys per LDS tile
constexpr float LOG2E = 1.4426950408889634f;
constexpr float LN2 = 0.6931471805599453f;
constexpr float PAD_BIAS = -10000.0f;  // bert_layers.py:424

typedef __attribute__((address_space(3))) bf16x4 lds_bf16x4;
typedef __attribute__((ext_vector_type(4))) short s16x4;

// element offset of (row, col) in a [64][64] bf16 tile (128-B rows) with 16-byte chunks
// XOR-swizzled by row. Rows r, r+1 share a 256-B bank row, so the key depends on r>>1:
//  * row reads (ds_read_b128, 16 lanes = 16 consecutive rows, one chunk): any bijection of
//    (r>>1)&7 spreads the 8 row pairs over 8 chunk slots -> conflict-free;
//  * transposed reads (ds_read_b64_tr_b16, a 32-lane half reads rows r0..r0+3, 4 chunks): rows r0
//    and r0+2 must land in different chunk halves, i.e. their keys differ in bit 2 -- so the key
//    is the bit-reversal of (r>>1)&7.
__device__ __forceinline__ int swz_key(int r) {
  const int k = (r >> 1) & 7;
  return ((k & 1) << 2) | (k & 2) | ((k >> 2) & 1);
}
__device__ __forceinline__ int swz(int r, int c) {
  return r * D + ((((c >> 3) ^ swz_key(r)) & 7) << 3) + (c & 7);
}

__device__ __forceinline__ bf16x4 tr_read(const bf16* lds_elem_ptr) {
  s16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (__attribute__((address_space(3))) s16x4*)(lds_elem_ptr));
  return __builtin_bit_cast(bf16x4, v);
}

__device__ __forceinline__ bf16x8 cat(bf16x4 a, bf16x4 b) {
  return bf16x8{a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
}

__device__ __forceinline__ f32x16 mfma(bf16x8 a, bf16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

// key index (within a 32-row block) held by accumulator register r of lane half hh
__device__ __forceinline__ int acc_row(int r, int hh) { return (r & 3) + 8 * (r >> 2) + 4 * hh; }

// raw v_exp_f32 (2^x): arguments here are <= ~0 (scores minus their running max / LSE), where
// the denormal-range fixups of exp2f() are not needed.
__device__ __forceinline__ float ex2(float x) { return __builtin_amdgcn_exp2f(x); }

// ALiBi distance term of accumulator register r (key offset within a 64-key tile, lane half hh)
// in log2 units: slope2 * ((r&3) + 8*(r>>2) + 32*kh) + slope2*4*hh  -- one FMA.
template <int KH, int R>
__device__ __forceinline__ float alibi_b(float slope2, float h4) {
  return fmaf(slope2, (float)(KH * 32 + (R & 3) + 8 * (R >> 2)), h4);
}


// Block -> (tile, head, batch). Blocks are dealt round-robin over the 8 XCDs (each with its own
// L2); all tiles of one (batch, head) read the same K/V (or Q/dO) rows, so map them to blocks with
// equal blockIdx % 8 (speed only -- placement is not guaranteed; any mapping is correct).
__device__ __forceinline__ void decode_block(int ntile, int H, int& tile, int& h, int& b) {
  const int L = blockIdx.x;
  const int nbh = gridDim.x / ntile;
  int bh;
  if ((nbh & 7) == 0) {
    const int r = L >> 3;
    tile = r % ntile;
    bh = (r / ntile) * 8 + (L & 7);
  } else {
    tile = L % ntile;
    bh = L / ntile;
  }
  h = bh % H;
  b = bh / H;
}

// ----------------------------------------------------------------------------- bf16 forward
struct TileRegs {
  bf16x8 k[2], v[2];
};

__global__ __launch_bounds__(256) void fwd_bf16_kernel(const bf16* __restrict__ qkv,
                                                        const uint8_t* __restrict__ key_valid,
                                                        const float* __restrict__ slopes, int S,
                                                        int H, float scale_log2,
                                                        bf16* __restrict__ out,
                                                        float* __restrict__ lse) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  bf16* Ks = reinterpret_cast<bf16*>(smem);            // [2][64*64] swizzled
  bf16* Vs = Ks + 2 * BK * D;                           // [2][64*64] swizzled
  float* kb = reinterpret_cast<float*>(Vs + 2 * BK * D);  // [2][64] pad bias (log2 units)

  int qblk, h, b;
  decode_block((S + BQ - 1) / BQ, H, qblk, h, b);
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int ql = lane & 31, hh = lane >> 5;
  const int ld = 3 * H * D;
  const bf16* base = qkv + (size_t)b * S * ld;
  const int q0 = qblk * BQ + wave * 32;
  const int qi = q0 + ql;
  const int qrow = min(qi, S - 1);
  const float slope2 = slopes[h] * LOG2E;

  bf16x8 qf[4];
#pragma unroll
  for (int s = 0; s < 4; ++s)
    qf[s] = *reinterpret_cast<const bf16x8*>(base + (size_t)qrow * ld + h * D + 16 * s + 8 * hh);

  // staging assignment: 512 16-byte chunks per K (and V) tile, 2 per thread
  auto load_tile = [&](int kt, TileRegs& t, float& bias) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      int c = tid + i * 256, r = c >> 3, ch = c & 7;
      const bf16* src = base + (size_t)(kt * BK + r) * ld + h * D + ch * 8;
      t.k[i] = *reinterpret_cast<const bf16x8*>(src + H * D);
      t.v[i] = *reinterpret_cast<const bf16x8*>(src + 2 * H * D);
    }
    bias = 0.f;
    if (tid < BK && key_valid) bias = key_valid[(size_t)b * S + kt * BK + tid] ? 0.f : PAD_BIAS * LOG2E;
  };
  auto store_tile = [&](int buf, const TileRegs& t, float bias) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      int c = tid + i * 256, r = c >> 3, ch = c & 7;
      *reinterpret_cast<bf16x8*>(Ks + buf * BK * D + swz(r, ch * 8)) = t.k[i];
      *reinterpret_cast<bf16x8*>(Vs + buf * BK * D + swz(r, ch * 8)) = t.v[i];
    }
    if (tid < BK) kb[buf * BK + tid] = bias;
  };

  f32x16 oacc[2];
#pragma unroll
  for (int i = 0; i < 16; ++i) { oacc[0][i] = 0.f; oacc[1][i] = 0.f; }
  float m = -INFINITY, l = 0.f;

  const int nt = S / BK;
  const int kt0 = (qblk * BQ / BK) % nt;  // diagonal tiles first: the max settles early
  {
    TileRegs t; float bias;
    load_tile(kt0, t, bias);
    store_tile(0, t, bias);
  }
  __syncthreads();

  const float h4 = slope2 * 4.f * hh;
  for (int it = 0; it < nt; ++it) {
    const int kt = (kt0 + it) % nt;
    const int buf = it & 1;
    TileRegs nx; float nbias = 0.f;
    if (it + 1 < nt) load_tile((kt0 + it + 1) % nt, nx, nbias);

    const bf16* K = Ks + buf * BK * D;
    const bf16* V = Vs + buf * BK * D;
    const float* kbias = kb + buf * BK;

    // S^T = K Q^T for the two 32-key halves
    f32x16 sacc[2];
#pragma unroll
    for (int kh = 0; kh < 2; ++kh) {
#pragma unroll
      for (int i = 0; i < 16; ++i) sacc[kh][i] = 0.f;
      const int r = kh * 32 + ql;
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        bf16x8 a = *reinterpret_cast<const bf16x8*>(K + swz(r, 16 * s + 8 * hh));
        sacc[kh] = mfma(a, qf[s], sacc[kh]);
      }
    }
    // scores in log2 units: x = s*scale*log2e + bias2. For a tile wholly left (right) of this
    // wave's 32 queries and without pads, bias2 = +-slope2*(key offset) + u with a per-lane u:
    // x~ = fma(s, c, +-b_r) and u folds into the running max (2 VALU per score instead of 5).
    float tmax = -INFINITY, u = 0.f;
    const int kbase = kt * BK;
    const bool haspad = key_valid && __any(kbias[lane] != 0.f);
    const bool left = !haspad && kbase + BK - 1 < q0;
    const bool right = !haspad && kbase > q0 + 31;
    if (left || right) {
      u = left ? slope2 * (float)(kbase - qi) : slope2 * (float)(qi - kbase);
#define DNA_SEP(KH, R, SG)                                                   \
  {                                                                         \
    float x = fmaf(sacc[KH][R], scale_log2, SG alibi_b<KH, R>(slope2, h4));  \
    sacc[KH][R] = x;                                                        \
    tmax = fmaxf(tmax, x);                                                  \
  }
#define DNA_SEP16(KH, SG)                                                                     \
  DNA_SEP(KH, 0, SG) DNA_SEP(KH, 1, SG) DNA_SEP(KH, 2, SG) DNA_SEP(KH, 3, SG)                 \
  DNA_SEP(KH, 4, SG) DNA_SEP(KH, 5, SG) DNA_SEP(KH, 6, SG) DNA_SEP(KH, 7, SG)                 \
  DNA_SEP(KH, 8, SG) DNA_SEP(KH, 9, SG) DNA_SEP(KH, 10, SG) DNA_SEP(KH, 11, SG)               \
  DNA_SEP(KH, 12, SG) DNA_SEP(KH, 13, SG) DNA_SEP(KH, 14, SG) DNA_SEP(KH, 15, SG)
      if (left) {
        DNA_SEP16(0, +)
        DNA_SEP16(1, +)
      } else {
        DNA_SEP16(0, -)
        DNA_SEP16(1, -)
      }
#undef DNA_SEP16
#undef DNA_SEP
    } else {
#pragma unroll
      for (int kh = 0; kh < 2; ++kh) {
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int kr = kh * 32 + 8 * g + 4 * hh;  // first of 4 consecutive keys
          const f32x4 pb = *reinterpret_cast<const f32x4*>(kbias + kr);
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int r = 4 * g + e;
            const float rel = fabsf((float)(qi - (kbase + kr + e)));
            float x = fmaf(sacc[kh][r], scale_log2, fmaf(-slope2, rel, pb[e]));
            sacc[kh][r] = x;
            tmax = fmaxf(tmax, x);
          }
        }
      }
    }
    tmax = fmaxf(tmax, __shfl_xor(tmax, 32, 64)) + u;
    const float mnew = fmaxf(m, tmax);
    const float alpha = ex2(m - mnew);
    m = mnew;
    const float mu = mnew - u;
    float psum = 0.f;
#pragma unroll
    for (int kh = 0; kh < 2; ++kh)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        float p = ex2(sacc[kh][r] - mu);
        sacc[kh][r] = p;
        psum += p;
      }
    l = l * alpha + psum;
    if (__any(alpha != 1.f)) {  // wave-uniform: skipped once the running max has settled
#pragma unroll
      for (int i = 0; i < 16; ++i) { oacc[0][i] *= alpha; oacc[1][i] *= alpha; }
    }
    // O^T += V^T P^T
    const int g16 = lane >> 4, i16 = lane & 15;
#pragma unroll
    for (int kh = 0; kh < 2; ++kh) {
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        bf16x8 pbf;
#pragma unroll
        for (int j = 0; j < 8; ++j) pbf[j] = (bf16)sacc[kh][8 * s + j];
        const int krow = kh * 32 + 16 * s + 4 * (g16 >> 1) + (i16 >> 2);
#pragma unroll
        for (int dt = 0; dt < 2; ++dt) {
          const int dcol = 32 * dt + 16 * (g16 & 1) + 4 * (i16 & 3);
          bf16x8 a = cat(tr_read(V + swz(krow, dcol)), tr_read(V + swz(krow + 8, dcol)));
          oacc[dt] = mfma(a, pbf, oacc[dt]);
        }
      }
    }
    if (it + 1 < nt) store_tile(buf ^ 1, nx, nbias);
    __syncthreads();
  }

  const float ltot = l + __shfl_xor(l, 32, 64);
  const float inv = 1.f / ltot;
  if (qi < S) {
    bf16* orow = out + ((size_t)b * S + qi) * (H * D) + h * D;
#pragma unroll
    for (int dt = 0; dt < 2; ++dt)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        bf16x4 v;
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = (bf16)(oacc[dt][4 * g + e] * inv);
        *reinterpret_cast<bf16x4*>(orow + 32 * dt + 8 * g + 4 * hh) = v;
      }
    if (hh == 0) lse[((size_t)b * H + h) * S + qi] = (m + __log2f(ltot)) * LN2;
  }
}

// ----------------------------------------------------------------------------- bf16 forward, v2
// Same math as fwd_bf16_kernel, reorganised for issue rate (the v1 loop was VALU-issue bound on
// per-score bias arithmetic and per-tile address recomputation):
//  * a wave owns 64 queries = two 32-query blocks, so every K row read and V transposed read
//    from LDS feeds two MFMAs; a workgroup (4 waves) owns 256 queries of one (batch, head);
//  * ALiBi enters the MFMA as the initial accumulator: for a 32-key half that lies wholly left
//    (right) of a 32-query block the bias is slope*(key offset) + a per-lane constant U, and the
//    key-offset part is a loop-invariant vector (+/- slope/scale * a_r) passed as the C operand.
//    A score then costs max3/2 + one FMA + v_exp + one add + cvt/2; only the diagonal half and
//    halves containing pad keys take the explicit per-score bias path;
//  * deferred rescaling: the running max m only moves when a half-tile's max exceeds it by more
//    than DEFER log2 units (P values stay <= 2^DEFER, exact in bf16/fp32 range);
//  * the cross-lane-half max/sum is one v_permlane32_swap; LDS addresses are per-lane constants
//    plus immediates.
constexpr int BQ2 = 256;          // queries per workgroup (4 waves x 64)
constexpr float DEFER = 8.0f;     // log2 units

__device__ __forceinline__ float pair_max(float x) {
  auto r = __builtin_amdgcn_permlane32_swap(__builtin_bit_cast(unsigned, x),
                                            __builtin_bit_cast(unsigned, x), false, false);
  return fmaxf(__builtin_bit_cast(float, (unsigned)r[0]), __builtin_bit_cast(float, (unsigned)r[1]));
}
__device__ __forceinline__ float pair_sum(float x) {
  auto r = __builtin_amdgcn_permlane32_swap(__builtin_bit_cast(unsigned, x),
                                            __builtin_bit_cast(unsigned, x), false, false);
  return __builtin_bit_cast(float, (unsigned)r[0]) + __builtin_bit_cast(float, (unsigned)r[1]);
}
// fmaxf of three. This file is compiled with -fno-honor-nans (dna_amd/build.py): scores are never
// NaN, and without it the compiler puts an IEEE-mode canonicalising v_max before every fmaxf of
// an MFMA result. (Inline asm is no way round that: the hazard recognizer does not see an asm
// statement reading an MFMA result, so it would read stale accumulators.)
__device__ __forceinline__ float max3(float a, float b, float c) { return fmaxf(fmaxf(a, b), c); }
__device__ __forceinline__ bool wave_any(bool p) { return __builtin_amdgcn_ballot_w64(p) != 0; }

// key offset (within a 32-key half, lane half hh excluded) of accumulator register r
__device__ __forceinline__ constexpr int aoff(int r) { return (r & 3) + 8 * (r >> 2); }

// NW waves per workgroup: 4 (two workgroups per CU) or 8 (one workgroup covers 512 queries, so
// at S = 512 each (b, h)'s K/V tiles stream from HBM once instead of once per 256 queries)
// DMA (NW = 4 only): the K / V tiles go global -> LDS by LDS-DMA (buffer_load ... lds) into a
// ring of NST tile buffers, two tiles ahead of the one computed -- no staging registers, no LDS
// writes by the waves, and a tile's HBM latency has two iterations to land; the pad bias of the
// whole key row is staged in LDS once. LDS image as before (the swizzle is applied by choosing
// which 16-B chunk of its row each lane fetches).
constexpr int NST = 3;
constexpr size_t fwd_dma_lds(int S) { return (size_t)NST * 2 * BK * D * 2 + (size_t)S * 4; }

template <int NQB, int NW = 4, bool DMA = false>
__global__ __launch_bounds__(64 * NW, NQB == 1 ? 3 : (NQB == 2 ? 2 : 1)) void fwd2_bf16_kernel(const bf16* __restrict__ qkv,
                                                           const uint8_t* __restrict__ key_valid,
                                                           const float* __restrict__ slopes,
                                                           int S, int H, float c,
                                                           bf16* __restrict__ out,
                                                           float* __restrict__ lse) {
  static_assert(!DMA || NW == 4, "DMA staging: 4 waves");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  bf16* Ks = reinterpret_cast<bf16*>(smem);               // [2][64*64] swizzled
  bf16* Vs = Ks + 2 * BK * D;                             // [2][64*64] swizzled
  float* kb = reinterpret_cast<float*>(Vs + 2 * BK * D);  // [2][64] pad bias (log2 units)
  // DMA: tile buffer t = K [64*64] then V [64*64] at smem + t * 16 KB; pad bias [S] after them
  float* kball = reinterpret_cast<float*>(smem + (size_t)NST * 2 * BK * D * 2);

  int qblk, h, b;
  constexpr int QPB = NW * 32 * NQB;  // queries per workgroup
  constexpr int NTH = 64 * NW, TPI = 512 / NTH;  // threads; 16-B tile chunks per thread
  decode_block((S + QPB - 1) / QPB, H, qblk, h, b);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // scalar: branches stay uniform
  const int ql = lane & 31, hh = lane >> 5;
  const int ld = 3 * H * D;
  const bf16* base = qkv + (size_t)b * S * ld;
  const int q0 = qblk * QPB + wave * 32 * NQB;
  const float slope2 = slopes[h] * LOG2E;
  const float sl_t = slope2 / c;  // ALiBi slope in raw-score units
  const float invc = 1.f / c;

  bf16x8 qf[NQB][4];
#pragma unroll
  for (int j = 0; j < NQB; ++j) {
    const int qrow = min(q0 + 32 * j + ql, S - 1);
#pragma unroll
    for (int s = 0; s < 4; ++s)
      qf[j][s] = *reinterpret_cast<const bf16x8*>(base + (size_t)qrow * ld + h * D + 16 * s + 8 * hh);
  }
  // DMA: per-lane byte offsets of piece p (rows (p*4 + wave)*8 + lane/8 of a tile, the 16-B chunk
  // that lands in slot lane%8 of the swizzled row); the tile's row offset is added per issue
  const auto rq = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16*>(base), (short)0,
                                                    (int)((size_t)S * ld * 2), 0x00020000);
  uint32_t vk[2];
#pragma unroll
  for (int p = 0; p < 2; ++p) {
    const int rr = (p * 4 + wave) * 8 + (lane >> 3);
    const int cc = (lane & 7) ^ swz_key(rr);
    vk[p] = (uint32_t)((rr * ld + H * D + h * D + cc * 8) * 2);
  }
  auto issue = [&](int kt, int buf) __attribute__((always_inline)) {
    typedef __attribute__((address_space(3))) void lds_v;
    const uint32_t toff = (uint32_t)(kt * BK * ld * 2);
    char* dk = smem + (size_t)buf * 2 * BK * D * 2;
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      char* dst = dk + (p * 4 + wave) * 8 * 128;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rq, (lds_v*)dst, 16, vk[p] + toff, 0, 0, 0);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rq, (lds_v*)(dst + BK * D * 2), 16,
                                               vk[p] + (uint32_t)(H * D * 2) + toff, 0, 0, 0);
    }
  };
  // per-lane integer part of the key - query distance, as float (exact): dqk = kb2 + lq[j]
  float lq[NQB];
#pragma unroll
  for (int j = 0; j < NQB; ++j) lq[j] = (float)(4 * hh - (q0 + 32 * j + ql));
  f32x16 initL, initR;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    initL[r] = sl_t * (float)aoff(r);
    initR[r] = -initL[r];
  }

  // per-lane LDS element offsets (tile buffer, kh and s add immediates)
  int so[TPI];
#pragma unroll
  for (int i = 0; i < TPI; ++i) {
    const int cidx = tid + i * NTH;
    so[i] = swz(cidx >> 3, (cidx & 7) * 8);
  }
  int kro[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) kro[s] = swz(ql, 16 * s + 8 * hh);
  const int g16 = lane >> 4, i16 = lane & 15;
  const int vr0 = 4 * (g16 >> 1) + (i16 >> 2);
  int vro[2][2];
#pragma unroll
  for (int dt = 0; dt < 2; ++dt) {
    const int dcol = 32 * dt + 16 * (g16 & 1) + 4 * (i16 & 3);
    vro[dt][0] = swz(vr0, dcol);
    vro[dt][1] = swz(vr0 + 8, dcol);
  }

  auto load_tile = [&](int kt, TileRegs& t, float& bias) {
#pragma unroll
    for (int i = 0; i < TPI; ++i) {
      const int cidx = tid + i * NTH;
      const bf16* src = base + (size_t)(kt * BK + (cidx >> 3)) * ld + h * D + (cidx & 7) * 8;
      t.k[i] = *reinterpret_cast<const bf16x8*>(src + H * D);
      t.v[i] = *reinterpret_cast<const bf16x8*>(src + 2 * H * D);
    }
    bias = 0.f;
    if (tid < BK && key_valid) bias = key_valid[(size_t)b * S + kt * BK + tid] ? 0.f : PAD_BIAS * LOG2E;
  };
  auto store_tile = [&](int buf, const TileRegs& t, float bias) {
#pragma unroll
    for (int i = 0; i < TPI; ++i) {
      *reinterpret_cast<bf16x8*>(Ks + buf * BK * D + so[i]) = t.k[i];
      *reinterpret_cast<bf16x8*>(Vs + buf * BK * D + so[i]) = t.v[i];
    }
    if (tid < BK) kb[buf * BK + tid] = bias;
  };

  f32x16 o[NQB][2];
#pragma unroll
  for (int j = 0; j < NQB; ++j)
#pragma unroll
    for (int i = 0; i < 16; ++i) { o[j][0][i] = 0.f; o[j][1][i] = 0.f; }
  float m[NQB], l[NQB];
#pragma unroll
  for (int j = 0; j < NQB; ++j) { m[j] = -INFINITY; l[j] = 0.f; }

  const int nt = S / BK;
  const int kt0 = (qblk * (QPB / BK) + (NQB == 1 ? 0 : 1)) % nt;  // near-diagonal tiles first
  auto tile_at = [&](int i) { const int t = kt0 + i % nt; return t >= nt ? t - nt : t; };
  if constexpr (DMA) {
    // the Q and key_valid loads are older than the tile pieces, so the first wait retires them
    for (int j = tid; j < S; j += 64 * NW)
      kball[j] = key_valid && !key_valid[(size_t)b * S + j] ? PAD_BIAS * LOG2E : 0.f;
    issue(tile_at(0), 0);
    issue(tile_at(1), 1);
  } else {
    TileRegs t; float bias;
    load_tile(kt0, t, bias);
    store_tile(0, t, bias);
    __syncthreads();
  }

  // one key tile; bufc is the tile's buffer -- a compile-time constant in the DMA ring (the loop
  // below is unrolled by NST), so every LDS address is a per-lane base plus an immediate
  auto iter = [&](const int it, const auto bufc) __attribute__((always_inline)) {
    int kt = kt0 + it;
    if (kt >= nt) kt -= nt;
    const int buf = bufc;
    TileRegs nx; float nbias = 0.f;
    if constexpr (DMA) {
      // this tile's pieces landed (the 4 of the next tile may still be in flight), everyone's
      // pieces too and every wave is past the tile it - 1, whose buffer the issue below refills
      // (past the end: a tile nobody reads, so every wait keeps the same count)
      __builtin_amdgcn_s_waitcnt((4 & 0xF) | (0x7 << 4) | (0xF << 8));
      __syncthreads();
      issue(tile_at(it + 2), (buf + 2) % NST);
    } else {
      if (it + 1 < nt) load_tile(kt + 1 < nt ? kt + 1 : kt + 1 - nt, nx, nbias);
    }

    const bf16* K = DMA ? reinterpret_cast<const bf16*>(smem) + (size_t)buf * 2 * BK * D : Ks + buf * BK * D;
    const bf16* V = DMA ? K + BK * D : Vs + buf * BK * D;
    const float* kbias = DMA ? kball + kt * BK : kb + buf * BK;
    const bool haspad = key_valid && wave_any(kbias[lane] != 0.f);

#pragma unroll
    for (int kh = 0; kh < 2; ++kh) {
      const int kb2 = kt * BK + 32 * kh;  // first key of this half
      const float kb2f = (float)kb2;
      bf16x8 kf[4];
#pragma unroll
      for (int s = 0; s < 4; ++s)
        kf[s] = *reinterpret_cast<const bf16x8*>(K + kh * 32 * D + kro[s]);
      bf16x8 pbf[NQB][2];
#pragma unroll
      for (int j = 0; j < NQB; ++j) {
        const int qf0 = q0 + 32 * j;  // wave-uniform
        const bool generic = haspad || kb2 == qf0;
        const bool left = kb2 < qf0;
        // every path leaves true score (log2 units) = sacc * c + U, U a per-lane constant, so
        // the max / exp tail below is one code path (no per-path vector phis)
        f32x16 sacc;
        float U = 0.f;
        if (!generic) {
          if (left) sacc = mfma(kf[0], qf[j][0], initL);
          else sacc = mfma(kf[0], qf[j][0], initR);
#pragma unroll
          for (int s = 1; s < 4; ++s) sacc = mfma(kf[s], qf[j][s], sacc);
          const float dqk = kb2f + lq[j];
          U = left ? slope2 * dqk : -slope2 * dqk;
        } else {
          f32x16 zero;
#pragma unroll
          for (int r = 0; r < 16; ++r) zero[r] = 0.f;
          sacc = mfma(kf[0], qf[j][0], zero);
#pragma unroll
          for (int s = 1; s < 4; ++s) sacc = mfma(kf[s], qf[j][s], sacc);
          const float dqk = kb2f + lq[j];
#pragma unroll
          for (int g = 0; g < 4; ++g) {
            const f32x4 pb = *reinterpret_cast<const f32x4*>(kbias + 32 * kh + 8 * g + 4 * hh);
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              const int r = 4 * g + e;
              sacc[r] = fmaf(fmaf(-slope2, fabsf(dqk + (float)aoff(r)), pb[e]), invc, sacc[r]);
            }
          }
        }
        float mx = max3(sacc[0], sacc[1], sacc[2]);
#pragma unroll
        for (int r = 3; r < 15; r += 2) mx = max3(mx, sacc[r], sacc[r + 1]);
        float tm = pair_max(fmaf(fmaxf(mx, sacc[15]), c, U));
        if (wave_any(tm > m[j] + DEFER)) {
          const float mn = fmaxf(m[j], tm);
          const float alpha = ex2(m[j] - mn);
          m[j] = mn;
          l[j] *= alpha;
#pragma unroll
          for (int i = 0; i < 16; ++i) { o[j][0][i] *= alpha; o[j][1][i] *= alpha; }
        }
        float ps = 0.f;
        const float off = U - m[j];
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const float p = ex2(fmaf(sacc[r], c, off));
          sacc[r] = p;
          ps += p;
        }
        l[j] += ps;
#pragma unroll
        for (int s = 0; s < 2; ++s)
#pragma unroll
          for (int e = 0; e < 8; ++e) pbf[j][s][e] = (bf16)sacc[8 * s + e];
      }
      // O^T += V^T P^T over the 32 keys of this half (2 k-steps of 16), V reads shared by j
#pragma unroll
      for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int dt = 0; dt < 2; ++dt) {
          const bf16* vb = V + (kh * 32 + 16 * s) * D;
          const bf16x8 a = cat(tr_read(vb + vro[dt][0]), tr_read(vb + vro[dt][1]));
#pragma unroll
          for (int j = 0; j < NQB; ++j) o[j][dt] = mfma(a, pbf[j][s], o[j][dt]);
        }
    }
    if constexpr (!DMA) {
      if (it + 1 < nt) store_tile(buf ^ 1, nx, nbias);
      __syncthreads();
    }
  };
  if constexpr (DMA) {
    using B0 = std::integral_constant<int, 0>;
    using B1 = std::integral_constant<int, 1>;
    using B2 = std::integral_constant<int, 2>;
    static_assert(NST == 3, "ring unrolled by 3");
    int it = 0;
    for (; it + NST <= nt; it += NST) {
      iter(it, B0{});
      iter(it + 1, B1{});
      iter(it + 2, B2{});
    }
    if (it < nt) iter(it, B0{});
    if (it + 1 < nt) iter(it + 1, B1{});
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no LDS-DMA outlives the block
  } else {
    for (int it = 0; it < nt; ++it) iter(it, it & 1);
  }

#pragma unroll
  for (int j = 0; j < NQB; ++j) {
    const int qi = q0 + 32 * j + ql;
    const float ltot = pair_sum(l[j]);
    const float inv = 1.f / ltot;
    if (qi < S) {
      bf16* orow = out + ((size_t)b * S + qi) * (H * D) + h * D;
#pragma unroll
      for (int dt = 0; dt < 2; ++dt)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          bf16x4 v;
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] = (bf16)(o[j][dt][4 * g + e] * inv);
          *reinterpret_cast<bf16x4*>(orow + 32 * dt + 8 * g + 4 * hh) = v;
        }
      if (hh == 0) lse[((size_t)b * H + h) * S + qi] = (m[j] + __log2f(ltot)) * LN2;
    }
  }
}

// ----------------------------------------------------------------------------- delta = rowsum(dO*O)
template <typename T>
__global__ void delta_kernel(const T* __restrict__ out, const T* __restrict__ dout, int T_rows,
                             int H, int S, float* __restrict__ delta) {
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;  // (row, head)
  if (idx >= T_rows * H) return;
  const int row = idx / H, h = idx % H;
  const T* o = out + (size_t)row * H * D + h * D;
  const T* g = dout + (size_t)row * H * D + h * D;
  float acc = 0.f;
#pragma unroll 8
  for (int d = 0; d < D; ++d) acc = fmaf(to_f32(o[d]), to_f32(g[d]), acc);
  const int b = row / S, s = row % S;
  delta[((size_t)b * H + h) * S + s] = acc;
}

// ----------------------------------------------------------------------------- bf16 dQ
// Queries on lanes (as forward). Per 64-key tile: S^T (8 MFMA), dP^T = V dO^T (8), dQ^T += K^T dS^T (8).
// Column sums over a block's 128 rows of a [128 x 64] fp32 tile held as two 32x32 MFMA
// accumulators (lane (wave, ql, hh): row wave*32+ql, columns 32dt + 8g + 4hh + e of acc[dt][4g+e]),
// times `mul`; rows with !valid count as zero. `red` is >= 32 KiB of free LDS (16-B chunks
// XOR-swizzled by row). Writes 64 floats to out. Fuses the packed-QKV projection's bias gradient
// (column sums of dqkv) into the attention backward: one partial row per 128-row block.
// Generalisation to NW waves (NW/4 groups of 4 waves = 128 rows): group g writes its 64 sums to
// out + g * row_stride, so the partial-row layout stays one row per 128 rows whatever the block.
// `red` needs NW * 32 * 64 floats.
template <int NW>
__device__ void block_colsum64_nw(float* red, const f32x16 (&acc)[2], float mul, bool valid,
                                  float* __restrict__ out, size_t row_stride) {
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, ql = lane & 31, hh = lane >> 5;
  const int r = wave * 32 + ql;
#pragma unroll
  for (int dt = 0; dt < 2; ++dt)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      f32x4 v;
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = valid ? acc[dt][4 * g + e] * mul : 0.f;
      const int chunk = 8 * dt + 2 * g + hh;  // 16-B chunk of the 64-column row
      *reinterpret_cast<f32x4*>(red + r * 64 + ((chunk ^ (r & 15)) << 2)) = v;
    }
  __syncthreads();
  const int c = tid & 63, qr = tid >> 6;
  float s = 0.f;
#pragma unroll 8
  for (int i = 0; i < 32; ++i) {
    const int rr = qr * 32 + i;
    s += red[rr * 64 + ((((c >> 2) ^ (rr & 15)) << 2) | (c & 3))];
  }
  __syncthreads();
  red[qr * 64 + c] = s;
  __syncthreads();
  if ((tid & 255) < 64) {
    const float* rg = red + (tid >> 8) * 256;
    out[(tid >> 8) * row_stride + c] = (rg[c] + rg[64 + c]) + (rg[128 + c] + rg[192 + c]);
  }
  __syncthreads();
}

__device__ void block_colsum64(float* red, const f32x16 (&acc)[2], float mul, bool valid,
                               float* __restrict__ out) {
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, ql = lane & 31, hh = lane >> 5;
  const int r = wave * 32 + ql;
#pragma unroll
  for (int dt = 0; dt < 2; ++dt)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      f32x4 v;
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = valid ? acc[dt][4 * g + e] * mul : 0.f;
      const int chunk = 8 * dt + 2 * g + hh;  // 16-B chunk of the 64-column row
      *reinterpret_cast<f32x4*>(red + r * 64 + ((chunk ^ (r & 15)) << 2)) = v;
    }
  __syncthreads();
  const int c = tid & 63, qr = tid >> 6;
  float s = 0.f;
#pragma unroll 8
  for (int i = 0; i < 32; ++i) {
    const int rr = qr * 32 + i;
    s += red[rr * 64 + ((((c >> 2) ^ (rr & 15)) << 2) | (c & 3))];
  }
  __syncthreads();
  red[qr * 64 + c] = s;
  __syncthreads();
  if (tid < 64) out[c] = (red[c] + red[64 + c]) + (red[128 + c] + red[192 + c]);
  __syncthreads();
}

__global__ __launch_bounds__(256) void dq_bf16_kernel(
    const bf16* __restrict__ qkv, const bf16* __restrict__ out, const bf16* __restrict__ dout,
    const float* __restrict__ lse, float* __restrict__ delta,
    const uint8_t* __restrict__ key_valid, const float* __restrict__ slopes, int S, int H,
    float scale_log2, float scale, bf16* __restrict__ dqkv, float* __restrict__ dbias_part) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  bf16* Ks = reinterpret_cast<bf16*>(smem);     // [2][64*64] swizzled
  bf16* Vs = Ks + 2 * BK * D;                    // [2][64*64] swizzled
  float* kb = reinterpret_cast<float*>(Vs + 2 * BK * D);

  int qblk, h, b;
  decode_block((S + BQ - 1) / BQ, H, qblk, h, b);
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int ql = lane & 31, hh = lane >> 5;
  const int ld = 3 * H * D;
  const bf16* base = qkv + (size_t)b * S * ld;
  const int qi = qblk * BQ + wave * 32 + ql;
  const int qrow = min(qi, S - 1);
  const float slope2 = slopes[h] * LOG2E;
  const float lse2 = lse[((size_t)b * H + h) * S + qrow] * LOG2E;

  bf16x8 qf[4], df[4];
  const size_t orow_off = ((size_t)b * S + qrow) * (H * D) + h * D;
  float dl = 0.f;  // delta = rowsum(dO * O): this lane holds half the row, lane^32 the other
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    qf[s] = *reinterpret_cast<const bf16x8*>(base + (size_t)qrow * ld + h * D + 16 * s + 8 * hh);
    df[s] = *reinterpret_cast<const bf16x8*>(dout + orow_off + 16 * s + 8 * hh);
    const bf16x8 o8 = *reinterpret_cast<const bf16x8*>(out + orow_off + 16 * s + 8 * hh);
#pragma unroll
    for (int j = 0; j < 8; ++j) dl = fmaf((float)df[s][j], (float)o8[j], dl);
  }
  dl += __shfl_xor(dl, 32, 64);
  if (hh == 0 && qi < S) delta[((size_t)b * H + h) * S + qi] = dl;

  auto load_tile = [&](int kt, TileRegs& t, float& bias) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      int c = tid + i * 256, r = c >> 3, ch = c & 7;
      const bf16* src = base + (size_t)(kt * BK + r) * ld + h * D + ch * 8;
      t.k[i] = *reinterpret_cast<const bf16x8*>(src + H * D);
      t.v[i] = *reinterpret_cast<const bf16x8*>(src + 2 * H * D);
    }
    bias = 0.f;
    if (tid < BK && key_valid) bias = key_valid[(size_t)b * S + kt * BK + tid] ? 0.f : PAD_BIAS * LOG2E;
  };
  auto store_tile = [&](int buf, const TileRegs& t, float bias) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      int c = tid + i * 256, r = c >> 3, ch = c & 7;
      *reinterpret_cast<bf16x8*>(Ks + buf * BK * D + swz(r, ch * 8)) = t.k[i];
      *reinterpret_cast<bf16x8*>(Vs + buf * BK * D + swz(r, ch * 8)) = t.v[i];
    }
    if (tid < BK) kb[buf * BK + tid] = bias;
  };

  f32x16 dq[2];
#pragma unroll
  for (int i = 0; i < 16; ++i) { dq[0][i] = 0.f; dq[1][i] = 0.f; }

  const int nt = S / BK;
  {
    TileRegs t; float bias;
    load_tile(0, t, bias);
    store_tile(0, t, bias);
  }
  __syncthreads();
  const int g16 = lane >> 4, i16 = lane & 15;

  const int q0 = qblk * BQ + wave * 32;
  const float h4 = slope2 * 4.f * hh;
  for (int kt = 0; kt < nt; ++kt) {
    const int buf = kt & 1;
    TileRegs nx; float nbias = 0.f;
    if (kt + 1 < nt) load_tile(kt + 1, nx, nbias);
    const bf16* K = Ks + buf * BK * D;
    const bf16* V = Vs + buf * BK * D;
    const float* kbias = kb + buf * BK;
    const int kbase = kt * BK;
    // separable ALiBi (see the forward): tiles wholly left/right of this wave's queries, no pads
    const bool haspad = key_valid && __any(kbias[lane] != 0.f);
    const bool left = !haspad && kbase + BK - 1 < q0;
    const bool right = !haspad && kbase > q0 + 31;
    const float lu = lse2 - (left ? slope2 * (float)(kbase - qi) : slope2 * (float)(qi - kbase));

#pragma unroll
    for (int kh = 0; kh < 2; ++kh) {
      f32x16 sa, pa;
#pragma unroll
      for (int i = 0; i < 16; ++i) { sa[i] = 0.f; pa[i] = 0.f; }
      const int r = kh * 32 + ql;
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        bf16x8 ak = *reinterpret_cast<const bf16x8*>(K + swz(r, 16 * s + 8 * hh));
        bf16x8 av = *reinterpret_cast<const bf16x8*>(V + swz(r, 16 * s + 8 * hh));
        sa = mfma(ak, qf[s], sa);
        pa = mfma(av, df[s], pa);
      }
      // dS^T = P^T (dP^T - delta), P^T = exp2(S c + bias - lse2)
      if (left || right) {
#pragma unroll
        for (int rr = 0; rr < 16; ++rr) {
          const float br = fmaf(slope2, (float)(kh * 32 + (rr & 3) + 8 * (rr >> 2)), h4);
          const float x = fmaf(sa[rr], scale_log2, left ? br : -br);
          sa[rr] = ex2(x - lu) * (pa[rr] - dl);
        }
      } else {
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int kr = kh * 32 + 8 * g + 4 * hh;
          const f32x4 pb = *reinterpret_cast<const f32x4*>(kbias + kr);
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int rr = 4 * g + e;
            const float rel = fabsf((float)(qi - (kbase + kr + e)));
            float x = fmaf(sa[rr], scale_log2, fmaf(-slope2, rel, pb[e]));
            float p = ex2(x - lse2);
            sa[rr] = p * (pa[rr] - dl);
          }
        }
      }
      // dQ^T[d][q] += K^T[d][key] dS^T[key][q]   (k-steps over 16 keys)
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        bf16x8 db;
#pragma unroll
        for (int j = 0; j < 8; ++j) db[j] = (bf16)sa[8 * s + j];
        const int krow = kh * 32 + 16 * s + 4 * (g16 >> 1) + (i16 >> 2);
#pragma unroll
        for (int dt = 0; dt < 2; ++dt) {
          const int dcol = 32 * dt + 16 * (g16 & 1) + 4 * (i16 & 3);
          bf16x8 a = cat(tr_read(K + swz(krow, dcol)), tr_read(K + swz(krow + 8, dcol)));
          dq[dt] = mfma(a, db, dq[dt]);
        }
      }
    }
    if (kt + 1 < nt) store_tile(buf ^ 1, nx, nbias);
    __syncthreads();
  }
  if (qi < S) {
    bf16* row = dqkv + ((size_t)b * S + qi) * ld + h * D;
#pragma unroll
    for (int dt = 0; dt < 2; ++dt)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        bf16x4 v;
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = (bf16)(dq[dt][4 * g + e] * scale);
        *reinterpret_cast<bf16x4*>(row + 32 * dt + 8 * g + 4 * hh) = v;
      }
  }  if (dbias_part) {
    const int nq = (S + BQ - 1) / BQ;
    block_colsum64(reinterpret_cast<float*>(smem), dq, scale, qi < S,
                   dbias_part + ((size_t)b * nq + qblk) * ld + h * D);
  }
}

// ----------------------------------------------------------------------------- bf16 dK / dV
// Keys on lanes: a workgroup = 4 waves x 32 keys; sweeps query tiles of 64 (two 32-halves).
// Per 32-query half: S (4 MFMA), dP = dO V^T (4), dV^T += dO^T P (4), dK^T += Q^T dS (4).
constexpr int BKW = 128;  // keys per workgroup
constexpr int BQT = 64;   // queries per LDS tile

__global__ __launch_bounds__(256) void dkdv_bf16_kernel(
    const bf16* __restrict__ qkv, const bf16* __restrict__ dout, const float* __restrict__ lse,
    const float* __restrict__ delta, const uint8_t* __restrict__ key_valid,
    const float* __restrict__ slopes, int S, int H, float scale_log2, float scale,
    bf16* __restrict__ dqkv, float* __restrict__ dbias_part) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  bf16* Qs = reinterpret_cast<bf16*>(smem);      // [2][64*64] swizzled
  bf16* Os = Qs + 2 * BQT * D;                    // [2][64*64] dO, swizzled
  float* ls = reinterpret_cast<float*>(Os + 2 * BQT * D);  // [2][64] lse (log2)
  float* ds = ls + 2 * BQT;                                 // [2][64] delta

  int kblk, h, b;
  decode_block((S + BKW - 1) / BKW, H, kblk, h, b);
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int kl = lane & 31, hh = lane >> 5;
  const int ld = 3 * H * D;
  const bf16* base = qkv + (size_t)b * S * ld;
  const bf16* obase = dout + (size_t)b * S * (H * D);
  const int kj = kblk * BKW + wave * 32 + kl;
  const int krow = min(kj, S - 1);
  const float slope2 = slopes[h] * LOG2E;
  const float kbias = (key_valid && !key_valid[(size_t)b * S + krow]) ? PAD_BIAS * LOG2E : 0.f;
  const float h4kv = slope2 * 4.f * hh;
  const float* lse_bh = lse + ((size_t)b * H + h) * S;
  const float* dl_bh = delta + ((size_t)b * H + h) * S;

  bf16x8 kf[4], vf[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    kf[s] = *reinterpret_cast<const bf16x8*>(base + (size_t)krow * ld + H * D + h * D + 16 * s + 8 * hh);
    vf[s] = *reinterpret_cast<const bf16x8*>(base + (size_t)krow * ld + 2 * H * D + h * D + 16 * s + 8 * hh);
  }

  struct QRegs { bf16x8 q[2], o[2]; float l, d; };
  auto load_tile = [&](int qt, QRegs& t) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      int c = tid + i * 256, r = c >> 3, ch = c & 7;
      const size_t row = (size_t)(qt * BQT + r);
      t.q[i] = *reinterpret_cast<const bf16x8*>(base + row * ld + h * D + ch * 8);
      t.o[i] = *reinterpret_cast<const bf16x8*>(obase + row * (H * D) + h * D + ch * 8);
    }
    if (tid < BQT) { t.l = lse_bh[qt * BQT + tid] * LOG2E; t.d = dl_bh[qt * BQT + tid]; }
  };
  auto store_tile = [&](int buf, const QRegs& t) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      int c = tid + i * 256, r = c >> 3, ch = c & 7;
      *reinterpret_cast<bf16x8*>(Qs + buf * BQT * D + swz(r, ch * 8)) = t.q[i];
      *reinterpret_cast<bf16x8*>(Os + buf * BQT * D + swz(r, ch * 8)) = t.o[i];
    }
    if (tid < BQT) { ls[buf * BQT + tid] = t.l; ds[buf * BQT + tid] = t.d; }
  };

  f32x16 dk[2], dv[2];
#pragma unroll
  for (int i = 0; i < 16; ++i) { dk[0][i] = dk[1][i] = dv[0][i] = dv[1][i] = 0.f; }

  const int nt = S / BQT;
  {
    QRegs t;
    load_tile(0, t);
    store_tile(0, t);
  }
  __syncthreads();
  const int g16 = lane >> 4, i16 = lane & 15;

  for (int qt = 0; qt < nt; ++qt) {
    const int buf = qt & 1;
    QRegs nx;
    if (qt + 1 < nt) load_tile(qt + 1, nx);
    const bf16* Q = Qs + buf * BQT * D;
    const bf16* O = Os + buf * BQT * D;
    const float* L = ls + buf * BQT;
    const float* DL = ds + buf * BQT;
    const int qbase = qt * BQT;
    const int kw0 = kblk * BKW + wave * 32;
#pragma unroll
    for (int qh = 0; qh < 2; ++qh) {
      const int qb = qbase + qh * 32;
      const bool after = qb > kw0 + 31;   // every query of this half is right of every key
      const bool before = qb + 31 < kw0;  // every query is left of every key
      f32x16 sa, pa;
#pragma unroll
      for (int i = 0; i < 16; ++i) { sa[i] = 0.f; pa[i] = 0.f; }
      const int r = qh * 32 + kl;  // A-operand row = query
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        bf16x8 aq = *reinterpret_cast<const bf16x8*>(Q + swz(r, 16 * s + 8 * hh));
        bf16x8 ao = *reinterpret_cast<const bf16x8*>(O + swz(r, 16 * s + 8 * hh));
        sa = mfma(aq, kf[s], sa);  // S[q][key]
        pa = mfma(ao, vf[s], pa);  // dP[q][key]
      }
      f32x16 pp;
      // after: bias2 = -slope2*(q - k) = -(slope2*c_r + h4 - u); before: +(slope2*c_r + h4 + u)
      const float hu = after ? h4kv - slope2 * (float)(kj - qb) - kbias
                             : h4kv + slope2 * (float)(qb - kj) + kbias;
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int qr = qh * 32 + 8 * g + 4 * hh;
        const f32x4 lq = *reinterpret_cast<const f32x4*>(L + qr);
        const f32x4 dq4 = *reinterpret_cast<const f32x4*>(DL + qr);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int rr = 4 * g + e;
          float x;
          if (after || before) {
            const float br = fmaf(slope2, (float)(8 * g + e), hu);
            x = fmaf(sa[rr], scale_log2, after ? -br : br);
          } else {
            const float rel = fabsf((float)(qbase + qr + e - kj));
            x = fmaf(sa[rr], scale_log2, fmaf(-slope2, rel, kbias));
          }
          float p = ex2(x - lq[e]);
          pp[rr] = p;
          sa[rr] = p * (pa[rr] - dq4[e]);  // dS
        }
      }
      // dV^T[d][key] += dO^T[d][q] P[q][key];  dK^T[d][key] += Q^T[d][q] dS[q][key]
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        bf16x8 pb, sb;
#pragma unroll
        for (int j = 0; j < 8; ++j) { pb[j] = (bf16)pp[8 * s + j]; sb[j] = (bf16)sa[8 * s + j]; }
        const int qrow = qh * 32 + 16 * s + 4 * (g16 >> 1) + (i16 >> 2);
#pragma unroll
        for (int dt = 0; dt < 2; ++dt) {
          const int dcol = 32 * dt + 16 * (g16 & 1) + 4 * (i16 & 3);
          bf16x8 ao = cat(tr_read(O + swz(qrow, dcol)), tr_read(O + swz(qrow + 8, dcol)));
          bf16x8 aq = cat(tr_read(Q + swz(qrow, dcol)), tr_read(Q + swz(qrow + 8, dcol)));
          dv[dt] = mfma(ao, pb, dv[dt]);
          dk[dt] = mfma(aq, sb, dk[dt]);
        }
      }
    }
    if (qt + 1 < nt) store_tile(buf ^ 1, nx);
    __syncthreads();
  }
  if (kj < S) {
    bf16* row = dqkv + ((size_t)b * S + kj) * ld + h * D;
#pragma unroll
    for (int dt = 0; dt < 2; ++dt)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        bf16x4 vk, vv;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          vk[e] = (bf16)(dk[dt][4 * g + e] * scale);
          vv[e] = (bf16)dv[dt][4 * g + e];
        }
        *reinterpret_cast<bf16x4*>(row + H * D + 32 * dt + 8 * g + 4 * hh) = vk;
        *reinterpret_cast<bf16x4*>(row + 2 * H * D + 32 * dt + 8 * g + 4 * hh) = vv;
      }
  }  if (dbias_part) {
    const int nk = (S + BKW - 1) / BKW;
    float* prow = dbias_part + ((size_t)b * nk + kblk) * ld + h * D;
    block_colsum64(reinterpret_cast<float*>(smem), dk, scale, kj < S, prow + H * D);
    block_colsum64(reinterpret_cast<float*>(smem), dv, 1.f, kj < S, prow + 2 * H * D);
  }
}

// ----------------------------------------------------------------------------- bf16 backward, v2
// Same decomposition as dq_bf16_kernel / dkdv_bf16_kernel (no atomics, deterministic) with the
// per-score VALU work cut the way fwd2_bf16_kernel does it:
//  * row constants enter the MFMAs as initial accumulators. dK/dV kernel (queries on rows):
//    S starts from (-LSE2 -+ slope2*q)/c, so with the per-lane (key) constant U = +-slope2*k +
//    pad(k), P = exp2(S*c + U) is one FMA + v_exp; dP starts from -delta, so dS = P * dP.
//    dQ kernel (queries on lanes): S^T starts from the +-slope/scale*offset vector of a
//    separable block, dP^T from -delta;
//  * blocks are classified per 32x32 (before / after / diagonal) with scalar branches; only
//    diagonal blocks (and, in the dQ kernel, key tiles with pad keys) compute |q - k| per score.
template <int NW>
__global__ __launch_bounds__(NW * 64, 8 / NW) void dkdv2_bf16_kernel(
    const bf16* __restrict__ qkv, const bf16* __restrict__ dout, const float* __restrict__ lse,
    const float* __restrict__ delta, const uint8_t* __restrict__ key_valid,
    const float* __restrict__ slopes, int S, int H, float c, float scale,
    bf16* __restrict__ dqkv, float* __restrict__ dbias_part) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  bf16* Qs = reinterpret_cast<bf16*>(smem);                // [2][64*64] swizzled
  bf16* Os = Qs + 2 * BQT * D;                              // [2][64*64] dO, swizzled
  float* rc = reinterpret_cast<float*>(Os + 2 * BQT * D);   // [2][4][64] row constants:
  // [0] (-LSE2 - slope2*q)/c  (query after the key), [1] (-LSE2 + slope2*q)/c  (before),
  // [2] -LSE2/c  (diagonal blocks), [3] -delta

  constexpr int NTHR = NW * 64, KPB = NW * 32;  // threads, keys per workgroup
  constexpr int NSTG = 512 / NTHR;               // 16-B staging chunks per thread per tensor
  int kblk, h, b;
  decode_block((S + KPB - 1) / KPB, H, kblk, h, b);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int kl = lane & 31, hh = lane >> 5;
  const int ld = 3 * H * D;
  const bf16* base = qkv + (size_t)b * S * ld;
  const bf16* obase = dout + (size_t)b * S * (H * D);
  const int kw0 = kblk * KPB + wave * 32;  // this wave's first key (uniform)
  const int kj = kw0 + kl;
  const int krow = min(kj, S - 1);
  const float slope2 = slopes[h] * LOG2E;
  const float invc = 1.f / c;
  const float sl_t = slope2 * invc;
  const float kbias = (key_valid && !key_valid[(size_t)b * S + krow]) ? PAD_BIAS * LOG2E : 0.f;
  const float* lse_bh = lse + ((size_t)b * H + h) * S;
  const float* dl_bh = delta + ((size_t)b * H + h) * S;

  bf16x8 kf[4], vf[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    kf[s] = *reinterpret_cast<const bf16x8*>(base + (size_t)krow * ld + H * D + h * D + 16 * s + 8 * hh);
    vf[s] = *reinterpret_cast<const bf16x8*>(base + (size_t)krow * ld + 2 * H * D + h * D + 16 * s + 8 * hh);
  }

  struct QRegs { bf16x8 q[NSTG], o[NSTG]; float l, d; };
  auto load_tile = [&](int qt, QRegs& t) {
#pragma unroll
    for (int i = 0; i < NSTG; ++i) {
      int cc = tid + i * NTHR, r = cc >> 3, ch = cc & 7;
      const size_t row = (size_t)(qt * BQT + r);
      t.q[i] = *reinterpret_cast<const bf16x8*>(base + row * ld + h * D + ch * 8);
      t.o[i] = *reinterpret_cast<const bf16x8*>(obase + row * (H * D) + h * D + ch * 8);
    }
    if (tid < BQT) { t.l = lse_bh[qt * BQT + tid] * LOG2E; t.d = dl_bh[qt * BQT + tid]; }
  };
  auto store_tile = [&](int buf, int qt, const QRegs& t) {
#pragma unroll
    for (int i = 0; i < NSTG; ++i) {
      int cc = tid + i * NTHR, r = cc >> 3, ch = cc & 7;
      *reinterpret_cast<bf16x8*>(Qs + buf * BQT * D + swz(r, ch * 8)) = t.q[i];
      *reinterpret_cast<bf16x8*>(Os + buf * BQT * D + swz(r, ch * 8)) = t.o[i];
    }
    if (tid < BQT) {
      const float sq = slope2 * (float)(qt * BQT + tid);
      float* R = rc + buf * 4 * BQT + tid;
      R[0] = (-t.l - sq) * invc;
      R[BQT] = (-t.l + sq) * invc;
      R[2 * BQT] = -t.l * invc;
      R[3 * BQT] = -t.d;
    }
  };

  f32x16 dk[2], dv[2];
#pragma unroll
  for (int i = 0; i < 16; ++i) { dk[0][i] = dk[1][i] = dv[0][i] = dv[1][i] = 0.f; }

  const int nt = S / BQT;
  {
    QRegs t;
    load_tile(0, t);
    store_tile(0, 0, t);
  }
  __syncthreads();
  const int g16 = lane >> 4, i16 = lane & 15;
  const float kjf = (float)kj;

  for (int qt = 0; qt < nt; ++qt) {
    const int buf = qt & 1;
    QRegs nx;
    if (qt + 1 < nt) load_tile(qt + 1, nx);
    const bf16* Q = Qs + buf * BQT * D;
    const bf16* O = Os + buf * BQT * D;
    const float* RC = rc + buf * 4 * BQT;
    // stage 1: S and dP for both 32-query halves (16 MFMAs) before any per-half VALU tail, so
    // the second half's MFMAs run under the first half's exp work
    f32x16 sa[2], pa[2];
#pragma unroll
    for (int qh = 0; qh < 2; ++qh) {
      const int qb = qt * BQT + qh * 32;  // first query of this half (uniform)
      const int sel = qb > kw0 ? 0 : (qb < kw0 ? 1 : 2);
      // register r = 4g + e  <->  query qb + 8g + 4hh + e
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) {
        const f32x4 l4 = *reinterpret_cast<const f32x4*>(RC + sel * BQT + qh * 32 + 8 * g4 + 4 * hh);
        const f32x4 d4 = *reinterpret_cast<const f32x4*>(RC + 3 * BQT + qh * 32 + 8 * g4 + 4 * hh);
#pragma unroll
        for (int e = 0; e < 4; ++e) { sa[qh][4 * g4 + e] = l4[e]; pa[qh][4 * g4 + e] = d4[e]; }
      }
      const int r0 = qh * 32 + kl;  // A-operand row = query
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const bf16x8 aq = *reinterpret_cast<const bf16x8*>(Q + swz(r0, 16 * s + 8 * hh));
        const bf16x8 ao = *reinterpret_cast<const bf16x8*>(O + swz(r0, 16 * s + 8 * hh));
        sa[qh] = mfma(aq, kf[s], sa[qh]);  // (S - LSE2 -+ slope2 q) / c   [q][key]
        pa[qh] = mfma(ao, vf[s], pa[qh]);  // dP - delta
      }
    }
    // stage 2 per half: P, dS (one tail for every block class), then dV^T += dO^T P,
    // dK^T += Q^T dS
#pragma unroll
    for (int qh = 0; qh < 2; ++qh) {
      const int qb = qt * BQT + qh * 32;
      const bool after = qb > kw0;  // every query after every key (32-aligned blocks)
      const bool before = qb < kw0;
      float U = kbias;
      if (after || before) {
        U = fmaf(after ? slope2 : -slope2, kjf, kbias);
      } else {
        const float lq = (float)(qb + 4 * hh - kj);  // q - k at register offset 0
#pragma unroll
        for (int r = 0; r < 16; ++r) sa[qh][r] = fmaf(-sl_t, fabsf(lq + (float)aoff(r)), sa[qh][r]);
      }
      bf16x8 pb[2], sb[2];
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float p = ex2(fmaf(sa[qh][r], c, U));
        pb[r >> 3][r & 7] = (bf16)p;
        sb[r >> 3][r & 7] = (bf16)(p * pa[qh][r]);
      }
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const int qrow = qh * 32 + 16 * s + 4 * (g16 >> 1) + (i16 >> 2);
#pragma unroll
        for (int dt = 0; dt < 2; ++dt) {
          const int dcol = 32 * dt + 16 * (g16 & 1) + 4 * (i16 & 3);
          const bf16x8 ao = cat(tr_read(O + swz(qrow, dcol)), tr_read(O + swz(qrow + 8, dcol)));
          const bf16x8 aq = cat(tr_read(Q + swz(qrow, dcol)), tr_read(Q + swz(qrow + 8, dcol)));
          dv[dt] = mfma(ao, pb[s], dv[dt]);
          dk[dt] = mfma(aq, sb[s], dk[dt]);
        }
      }
    }
    if (qt + 1 < nt) store_tile(buf ^ 1, qt + 1, nx);
    __syncthreads();
  }
  if (kj < S) {
    bf16* row = dqkv + ((size_t)b * S + kj) * ld + h * D;
#pragma unroll
    for (int dt = 0; dt < 2; ++dt)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        bf16x4 vk, vv;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          vk[e] = (bf16)(dk[dt][4 * g + e] * scale);
          vv[e] = (bf16)dv[dt][4 * g + e];
        }
        *reinterpret_cast<bf16x4*>(row + H * D + 32 * dt + 8 * g + 4 * hh) = vk;
        *reinterpret_cast<bf16x4*>(row + 2 * H * D + 32 * dt + 8 * g + 4 * hh) = vv;
      }
  }
  if (dbias_part) {  // partial rows are per 128 keys (dna_attn_dbias_part_rows)
    const int nk = (S + BKW - 1) / BKW;
    float* prow = dbias_part + ((size_t)b * nk + kblk * (NW / 4)) * ld + h * D;
    block_colsum64_nw<NW>(reinterpret_cast<float*>(smem), dk, scale, kj < S, prow + H * D, ld);
    block_colsum64_nw<NW>(reinterpret_cast<float*>(smem), dv, 1.f, kj < S, prow + 2 * H * D, ld);
  }
}

// dQ with queries on lanes: per 32-key half, S^T from the ALiBi vector of a separable block,
// P = exp2(S c + U - LSE2), dS = P (dP - delta) with dP^T started from -delta,
// dQ^T += K^T dS^T. Also writes delta for the dK/dV kernel and the fused bias-gradient column
// partials (as dq_bf16_kernel).
template <int NW>
__global__ __launch_bounds__(NW * 64, 8 / NW) void dq2_bf16_kernel(
    const bf16* __restrict__ qkv, const bf16* __restrict__ out, const bf16* __restrict__ dout,
    const float* __restrict__ lse, float* __restrict__ delta,
    const uint8_t* __restrict__ key_valid, const float* __restrict__ slopes, int S, int H,
    float c, float scale, bf16* __restrict__ dqkv, float* __restrict__ dbias_part) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  bf16* Ks = reinterpret_cast<bf16*>(smem);     // [2][64*64] swizzled
  bf16* Vs = Ks + 2 * BK * D;                    // [2][64*64] swizzled
  float* kb = reinterpret_cast<float*>(Vs + 2 * BK * D);

  constexpr int NTHR = NW * 64, QPB = NW * 32;  // threads, queries per workgroup
  constexpr int NSTG = 512 / NTHR;
  int qblk, h, b;
  decode_block((S + QPB - 1) / QPB, H, qblk, h, b);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int ql = lane & 31, hh = lane >> 5;
  const int ld = 3 * H * D;
  const bf16* base = qkv + (size_t)b * S * ld;
  const int q0 = qblk * QPB + wave * 32;  // uniform
  const int qi = q0 + ql;
  const int qrow = min(qi, S - 1);
  const float slope2 = slopes[h] * LOG2E;
  const float invc = 1.f / c;
  const float sl_t = slope2 * invc;
  const float lse2 = lse[((size_t)b * H + h) * S + qrow] * LOG2E;

  bf16x8 qf[4], df[4];
  const size_t orow_off = ((size_t)b * S + qrow) * (H * D) + h * D;
  float dl = 0.f;  // delta = rowsum(dO * O): this lane holds half the row, lane^32 the other
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    qf[s] = *reinterpret_cast<const bf16x8*>(base + (size_t)qrow * ld + h * D + 16 * s + 8 * hh);
    df[s] = *reinterpret_cast<const bf16x8*>(dout + orow_off + 16 * s + 8 * hh);
    const bf16x8 o8 = *reinterpret_cast<const bf16x8*>(out + orow_off + 16 * s + 8 * hh);
#pragma unroll
    for (int j = 0; j < 8; ++j) dl = fmaf((float)df[s][j], (float)o8[j], dl);
  }
  dl = pair_sum(dl);
  if (hh == 0 && qi < S) delta[((size_t)b * H + h) * S + qi] = dl;
  f32x16 negd;
#pragma unroll
  for (int r = 0; r < 16; ++r) negd[r] = -dl;

  struct KVRegs { bf16x8 k[NSTG], v[NSTG]; };
  auto load_tile = [&](int kt, KVRegs& t, float& bias) {
#pragma unroll
    for (int i = 0; i < NSTG; ++i) {
      int cc = tid + i * NTHR, r = cc >> 3, ch = cc & 7;
      const bf16* src = base + (size_t)(kt * BK + r) * ld + h * D + ch * 8;
      t.k[i] = *reinterpret_cast<const bf16x8*>(src + H * D);
      t.v[i] = *reinterpret_cast<const bf16x8*>(src + 2 * H * D);
    }
    bias = 0.f;
    if (tid < BK && key_valid) bias = key_valid[(size_t)b * S + kt * BK + tid] ? 0.f : PAD_BIAS * LOG2E;
  };
  auto store_tile = [&](int buf, const KVRegs& t, float bias) {
#pragma unroll
    for (int i = 0; i < NSTG; ++i) {
      int cc = tid + i * NTHR, r = cc >> 3, ch = cc & 7;
      *reinterpret_cast<bf16x8*>(Ks + buf * BK * D + swz(r, ch * 8)) = t.k[i];
      *reinterpret_cast<bf16x8*>(Vs + buf * BK * D + swz(r, ch * 8)) = t.v[i];
    }
    if (tid < BK) kb[buf * BK + tid] = bias;
  };

  f32x16 dq[2];
#pragma unroll
  for (int i = 0; i < 16; ++i) { dq[0][i] = 0.f; dq[1][i] = 0.f; }

  const int nt = S / BK;
  {
    KVRegs t; float bias;
    load_tile(0, t, bias);
    store_tile(0, t, bias);
  }
  __syncthreads();
  const int g16 = lane >> 4, i16 = lane & 15;

  for (int kt = 0; kt < nt; ++kt) {
    const int buf = kt & 1;
    KVRegs nx; float nbias = 0.f;
    if (kt + 1 < nt) load_tile(kt + 1, nx, nbias);
    const bf16* K = Ks + buf * BK * D;
    const bf16* V = Vs + buf * BK * D;
    const float* kbias = kb + buf * BK;
    const bool haspad = key_valid && wave_any(kbias[lane] != 0.f);
#pragma unroll
    for (int kh = 0; kh < 2; ++kh) {
      const int kb2 = kt * BK + 32 * kh;  // uniform
      const bool generic = haspad || kb2 == q0;
      const bool left = kb2 < q0;
      const float dqk = (float)(kb2 + 4 * hh - qi);  // k - q at register offset 0
      const int r0 = kh * 32 + ql;
      f32x16 sa, pa;
      {
        bf16x8 ak[4];
#pragma unroll
        for (int s = 0; s < 4; ++s) ak[s] = *reinterpret_cast<const bf16x8*>(K + swz(r0, 16 * s + 8 * hh));
        if (generic) {
          f32x16 z;
#pragma unroll
          for (int i = 0; i < 16; ++i) z[i] = 0.f;
          sa = mfma(ak[0], qf[0], z);
        } else if (left) {
          f32x16 ini;
#pragma unroll
          for (int r = 0; r < 16; ++r) ini[r] = sl_t * (float)aoff(r);
          sa = mfma(ak[0], qf[0], ini);
        } else {
          f32x16 ini;
#pragma unroll
          for (int r = 0; r < 16; ++r) ini[r] = -sl_t * (float)aoff(r);
          sa = mfma(ak[0], qf[0], ini);
        }
#pragma unroll
        for (int s = 1; s < 4; ++s) sa = mfma(ak[s], qf[s], sa);
      }
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const bf16x8 av = *reinterpret_cast<const bf16x8*>(V + swz(r0, 16 * s + 8 * hh));
        pa = mfma(av, df[s], s == 0 ? negd : pa);
      }
      // both paths leave exponent = sa * c + off (off per lane): one tail code path
      float off = -lse2;
      if (!generic) {
        off += left ? slope2 * dqk : -slope2 * dqk;
      } else {
#pragma unroll
        for (int g4 = 0; g4 < 4; ++g4) {
          const f32x4 pb = *reinterpret_cast<const f32x4*>(kbias + 32 * kh + 8 * g4 + 4 * hh);
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int r = 4 * g4 + e;
            sa[r] = fmaf(fmaf(-slope2, fabsf(dqk + (float)aoff(r)), pb[e]), invc, sa[r]);
          }
        }
      }
      bf16x8 db[2];
#pragma unroll
      for (int r = 0; r < 16; ++r) db[r >> 3][r & 7] = (bf16)(ex2(fmaf(sa[r], c, off)) * pa[r]);
      // dQ^T[d][q] += K^T[d][key] dS^T[key][q]   (k-steps over 16 keys)
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const int krow = kh * 32 + 16 * s + 4 * (g16 >> 1) + (i16 >> 2);
#pragma unroll
        for (int dt = 0; dt < 2; ++dt) {
          const int dcol = 32 * dt + 16 * (g16 & 1) + 4 * (i16 & 3);
          const bf16x8 a = cat(tr_read(K + swz(krow, dcol)), tr_read(K + swz(krow + 8, dcol)));
          dq[dt] = mfma(a, db[s], dq[dt]);
        }
      }
    }
    if (kt + 1 < nt) store_tile(buf ^ 1, nx, nbias);
    __syncthreads();
  }
  if (qi < S) {
    bf16* row = dqkv + ((size_t)b * S + qi) * ld + h * D;
#pragma unroll
    for (int dt = 0; dt < 2; ++dt)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        bf16x4 v;
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = (bf16)(dq[dt][4 * g + e] * scale);
        *reinterpret_cast<bf16x4*>(row + 32 * dt + 8 * g + 4 * hh) = v;
      }
  }
  if (dbias_part) {  // partial rows are per 128 queries (dna_attn_dbias_part_rows)
    const int nq = (S + BQ - 1) / BQ;
    block_colsum64_nw<NW>(reinterpret_cast<float*>(smem), dq, scale, qi < S,
                          dbias_part + ((size_t)b * nq + qblk * (NW / 4)) * ld + h * D, ld);
  }
}

// ----------------------------------------------------------------------------- bf16 backward, v3
// One fused kernel, one workgroup per (batch, head) for S = 128*KB: 4 waves, wave w owns keys
// [w*32*KB, (w+1)*32*KB) and keeps their dK^T / dV^T in 4*KB f32x16 accumulators for the whole
// pass, so dK and dV need no sum across workgroups. The workgroup sweeps the queries in slices of
// 32 (Q, dO and the row constants of a slice double-buffered in LDS, K resident in LDS):
//  phase 1 (per wave, per 32-key block, keys on the lane as in dkdv2): S' and dP' started from
//    the row constants, P = exp2(S' c + U), dS = P dP', dV^T += dO^T P, dK^T += Q^T dS, and dS
//    written transposed ([key][q]) to an LDS image;
//  phase 2: dQ^T = K^T dS^T over all S keys, split over the 4 waves as (32-d half) x (key half);
//    the two key-half partials are summed in a fixed order through LDS (deterministic).
// S and dP are computed once per score block (five MFMA products instead of the seven of the
// dq2 + dkdv2 pair), and Q, dO, O and LSE are read once per (batch, head).
template <int CTRL>
__device__ __forceinline__ float dppf(float x) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, x), CTRL,
                                                               0xF, 0xF, false));
}
// sum over the 32 lanes of a wave half (every lane of the half gets the total)
__device__ __forceinline__ float sum32(float x) {
  x += dppf<0xB1>(x);   // quad_perm [1,0,3,2]
  x += dppf<0x4E>(x);   // quad_perm [2,3,0,1]
  x += dppf<0x141>(x);  // row_half_mirror
  x += dppf<0x140>(x);  // row_mirror
  return x + __shfl_xor(x, 16, 64);
}

// dst += A B with the accumulator pinned to AGPRs: the 4*KB dK^T / dV^T tiles of a wave fill the
// accumulator file, every other MFMA of the kernel is in VGPR form (attention.hip is built with
// -mllvm -amdgpu-mfma-vgpr-form=1). hipcc pads nothing inside asm: s_nop 1 covers a VALU write
// (bf16 packing of P / dS) or v_accvgpr_write (zero init) of an operand just before; the chain
// on one accumulator needs no wait states; readers of the result wait via acc_fence().
__device__ __forceinline__ void mfma_acc(f32x16& acc, const bf16x8& a, const bf16x8& b) {
  asm volatile("s_nop 1\n\tv_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+a"(acc) : "v"(a), "v"(b));
}
// wait states between the last MFMA writing `acc` and any other reader of it (16-pass XDL)
__device__ __forceinline__ void acc_fence(f32x16& x, f32x16& y) {
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" : "+a"(x), "+a"(y));
}

// LDS: K image, Q/dO images, dS^T image, row constants, then (at >= 64 KiB, past the epilogue's
// 64 KiB dK/dV staging that reuses the start) the dQ partials and the dS row sums
template <int KB>
constexpr size_t bwd3_red_off() {
  constexpr size_t a = (size_t)128 * KB * D * 2 + 4 * 32 * D * 2 + (size_t)128 * KB * 32 * 2 + 2 * 4 * 32 * 4;
  return a > 65536 ? a : 65536;
}
constexpr int CS_LD = 36;  // colsum staging row stride in floats ([d][key], 16-B aligned rows)
// epilogue staging: for KB = 4 it reuses the Q/dO/dS^T images (48 KiB, dead by then), else it
// gets its own region after the dS row sums
template <int KB>
constexpr bool bwd3_stage_alias() { return (size_t)4 * 32 * D * 2 + (size_t)128 * KB * 32 * 2 >= 4 * 64 * CS_LD * 4; }
template <int KB>
constexpr size_t bwd3_lds() {
  return bwd3_red_off<KB>() + 2 * 1024 * 4 + (size_t)128 * KB * 2 * 4 +
         (bwd3_stage_alias<KB>() ? 0 : 4 * 64 * CS_LD * 4);
}

#ifndef DNA_BWD3_STAMP
#define DNA_BWD3_STAMP 0
#endif
#if DNA_BWD3_STAMP
// timing probe (debug builds only): s_memtime at phase boundaries of block 0's waves
__device__ unsigned long long g_bwd3_stamps[4][16][6];
#define BWD3_STAMP(t, k)                                                              \
  do {                                                                                \
    const unsigned long long ts_ = __builtin_amdgcn_s_memtime();                     \
    if (blockIdx.x == 0 && lane == 0 && (t) < 16) g_bwd3_stamps[wave][(t)][(k)] = ts_; \
  } while (0)
#else
#define BWD3_STAMP(t, k) do {} while (0)
#endif
// V bit 0: fused bias-gradient column sums; bit 1: per-step sched_barriers in the pipelined
// phase 1 (keeps the softmax tail between the previous block's dV/dK MFMAs; A/B via
// DNA_ATTN_BWD3_SB)
template <int KB, int V>
__global__ __launch_bounds__(256, 1) void bwd3_bf16_kernel(
    const bf16* __restrict__ qkv, const bf16* __restrict__ out, const bf16* __restrict__ dout,
    const float* __restrict__ lse, const uint8_t* __restrict__ key_valid,
    const float* __restrict__ slopes, int H, float c, float scale, bf16* __restrict__ dqkv,
    float* __restrict__ dbias_part) {
  constexpr bool DB = V & 1;  // fused bias-gradient column sums
  constexpr bool DBL = DB, DBE = DB;
  constexpr bool PIPE_SB = (V & 2) != 0;
  constexpr int S = 128 * KB;   // keys = queries of one (batch, head)
  constexpr int KPW = 32 * KB;  // keys per wave
  constexpr int NS = S / 32;    // query slices
  constexpr int KS2 = S / 32;   // 16-key steps of one key half (phase 2)
  extern __shared__ __attribute__((aligned(16))) char smem[];
  bf16* Kimg = reinterpret_cast<bf16*>(smem);          // [S][64] swz
  bf16* Qimg = Kimg + S * D;                            // [2][32][64] swz
  bf16* Oimg = Qimg + 2 * 32 * D;                       // [2][32][64] dO, swz
  bf16* dST = Oimg + 2 * 32 * D;                        // [S][32] dS^T, 8-B chunks XOR (row>>1)&7
  float* rc = reinterpret_cast<float*>(dST + S * 32);  // [2][4][32] row constants (as dkdv2)
  float* red = reinterpret_cast<float*>(smem + bwd3_red_off<KB>());  // [2][1024] dQ^T partials
                                                                      // of key half 1

  const int bh = blockIdx.x, h = bh % H, b = bh / H;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int kl = lane & 31, hh = lane >> 5;
  const int g16 = lane >> 4, i16 = lane & 15;
  const int ld = 3 * H * D;
  const bf16* base = qkv + (size_t)b * S * ld;
  const size_t obase = (size_t)b * S * (H * D) + h * D;
  const float slope2 = slopes[h] * LOG2E;
  const float invc = 1.f / c;
  const float sl_t = slope2 * invc;
  const float* lse_bh = lse + ((size_t)b * H + h) * S;

  {  // K image of all S keys
    constexpr int NCH = S * 8 / 256;
    bf16x8 kt[NCH];
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
      const int cc = tid + 256 * i;
      kt[i] = *reinterpret_cast<const bf16x8*>(base + (size_t)(cc >> 3) * ld + H * D + h * D + (cc & 7) * 8);
    }
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
      const int cc = tid + 256 * i;
      *reinterpret_cast<bf16x8*>(Kimg + swz(cc >> 3, (cc & 7) * 8)) = kt[i];
    }
  }
  bf16x8 vf[KB][4];  // V of this wave's keys as the B operand of dP' (key on the lane)
  unsigned padm = 0;  // bit kb: key wave*KPW + 32kb + kl is a pad key
#pragma unroll
  for (int kb = 0; kb < KB; ++kb) {
    const int kj = wave * KPW + 32 * kb + kl;
#pragma unroll
    for (int s = 0; s < 4; ++s)
      vf[kb][s] = *reinterpret_cast<const bf16x8*>(base + (size_t)kj * ld + 2 * H * D + h * D + 16 * s + 8 * hh);
    if (key_valid && !key_valid[(size_t)b * S + kj]) padm |= 1u << kb;
  }

  // query-slice staging: thread -> (row sr, 16-B chunk sc) of Q, dO and O
  struct SRegs { bf16x8 q, o, d; float l; };
  // the staging indices come from an opaque copy of tid per slice (see `tid_t` in the loop):
  // otherwise the compiler keeps every per-lane 64-bit row address live across the whole loop
  auto load_slice = [&](int t, SRegs& x, int tid_t) {
    const int sr = tid_t >> 3, sc = tid_t & 7;
    const int q = 32 * t + sr;
    x.q = *reinterpret_cast<const bf16x8*>(base + (size_t)q * ld + h * D + sc * 8);
    x.o = *reinterpret_cast<const bf16x8*>(out + obase + (size_t)q * (H * D) + sc * 8);
    x.d = *reinterpret_cast<const bf16x8*>(dout + obase + (size_t)q * (H * D) + sc * 8);
    x.l = lse_bh[q];
  };
  auto store_slice = [&](int buf, int t, const SRegs& x, int tid_t) {
    const int sr = tid_t >> 3, sc = tid_t & 7;
    *reinterpret_cast<bf16x8*>(Qimg + buf * 32 * D + swz(sr, sc * 8)) = x.q;
    *reinterpret_cast<bf16x8*>(Oimg + buf * 32 * D + swz(sr, sc * 8)) = x.d;
    float dl = 0.f;  // delta = rowsum(dO * O) over the row's 8 chunks (8 consecutive lanes)
#pragma unroll
    for (int j = 0; j < 8; ++j) dl = fmaf((float)x.d[j], (float)x.o[j], dl);
    dl += dppf<0xB1>(dl);   // quad_perm [1,0,3,2]
    dl += dppf<0x4E>(dl);   // quad_perm [2,3,0,1]: quad sum in every lane
    dl += dppf<0x141>(dl);  // row_half_mirror: + the other quad of the 8-lane row group
    if (sc == 0) {
      const float l2 = x.l * LOG2E, sq = slope2 * (float)(32 * t + sr);
      float* R = rc + buf * 128 + sr;
      R[0] = (-l2 - sq) * invc;  // query after the key block
      R[32] = (-l2 + sq) * invc; // query before
      R[64] = -l2 * invc;        // diagonal block
      R[96] = -dl;
    }
  };

  f32x16 dk[KB][2], dv[KB][2];
  // sig[kb] = sum over the queries this lane holds of dS[q][key]: the dQ column sums of the bias
  // gradient are sum_key K[key][d] * sum_q dS[q][key] (per-key sums, contracted with K in the
  // epilogue), so the loop carries KB floats instead of per-slice cross-lane reductions
  // (kept in LDS, sigl[hh][key] -- consecutive keys on consecutive lanes, conflict-free -- read
  // early in each block and written back by the owner lane:
  // four loop-carried registers more push the loop over the register file)
  float* sigl = red + 2 * 1024;
  if (DBL)
    for (int i = tid; i < 2 * S; i += 256) sigl[i] = 0.f;
#pragma unroll
  for (int kb = 0; kb < KB; ++kb) {
#pragma unroll
    for (int i = 0; i < 16; ++i) { dk[kb][0][i] = dk[kb][1][i] = dv[kb][0][i] = dv[kb][1][i] = 0.f; }
  }
  const int dth = wave & 1, kh2 = wave >> 1;  // phase-2 role: 32-d half, key half
  const bf16* Kw = Kimg + wave * KPW * D;     // this wave's keys in the K image
  bf16* dSTw = dST + wave * KPW * 32;         // ... and in the dS^T image
  const bf16* Kh = Kimg + kh2 * (S / 2) * D;  // phase-2 key half
  const bf16* dSTh = dST + kh2 * (S / 2) * 32;
  {
    SRegs x;
    load_slice(0, x, tid);
    store_slice(0, 0, x, tid);
  }
  __syncthreads();

  for (int t = 0; t < NS; ++t) {
    BWD3_STAMP(t, 0);
    const int buf = t & 1;
    int tid_t = tid;  // opaque per slice: lane-derived values are recomputed, not kept live
    asm volatile("" : "+v"(tid_t));
    const int kl_t = tid_t & 31;
    unsigned padm_t = padm;
    asm volatile("" : "+v"(padm_t));
    SRegs nx;  // next slice's Q / O / dO / LSE: loaded in the drain step of phase 1 (kb == KB,
               // no S' / dP' registers live), stored to LDS after phase 2
    const bf16* Q = Qimg + buf * 32 * D;
    const bf16* O = Oimg + buf * 32 * D;
    const float* RC = rc + buf * 128;
    const int qb = 32 * t;
    // ---- phase 1, software-pipelined over the key blocks: iteration kb computes S'/dP' of block
    // kb (8 MFMAs), then issues the 8 dV/dK MFMAs of block kb-1 one per step, each followed by
    // the exp / dS work of two scores of block kb, so the softmax tail runs under the matrix pipe
    // (one wave per SIMD: overlap has to come from this wave's own instruction order; the
    // sched_barriers keep the compiler from regrouping it)
    bf16x8 pbp[2], sbp[2];  // P and dS (bf16) of the previous block
    const int tq = 4 * (g16 >> 1) + (i16 >> 2);  // tr-read row of lane
    auto tr_pair = [&](const bf16* img, int j) {  // A operand (dO^T or Q^T) of pair j = (s2, dt)
      const int qrow = 16 * (j >> 1) + tq;
      const int dcol = 32 * (j & 1) + 16 * (g16 & 1) + 4 * (i16 & 3);
      return cat(tr_read(img + swz(qrow, dcol)), tr_read(img + swz(qrow + 8, dcol)));
    };
    // Q and dO fragments of the slice (A operands of every block's S' / dP' MFMAs): read once per
    // slice -- re-read per block, each MFMA waited a full LDS latency on its own fragment (the
    // compiler cannot reuse LDS reads across the block's dS^T stores)
    bf16x8 qfr[4], ofr[4];
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      qfr[s] = *reinterpret_cast<const bf16x8*>(Q + swz(kl, 16 * s + 8 * hh));
      ofr[s] = *reinterpret_cast<const bf16x8*>(O + swz(kl, 16 * s + 8 * hh));
    }
#pragma unroll
    for (int kb = 0; kb <= KB; ++kb) {
      __builtin_amdgcn_sched_barrier(0);
      if (kb == KB && t + 1 < NS) load_slice(t + 1, nx, tid_t);
      const int kbase = wave * KPW + 32 * kb;  // uniform
      const bool after = qb > kbase, before = qb < kbase;
      f32x16 sa, pa;
      float U = 0.f;
      if (kb < KB) {
        const int sel = after ? 0 : (before ? 1 : 2);
#pragma unroll
        for (int g4 = 0; g4 < 4; ++g4) {
          const f32x4 l4 = *reinterpret_cast<const f32x4*>(RC + sel * 32 + 8 * g4 + 4 * hh);
#pragma unroll
          for (int e = 0; e < 4; ++e) sa[4 * g4 + e] = l4[e];
        }
        // -delta of the slice's rows (the dP' initial accumulator), re-read per block beside the
        // S' row constants rather than held in 16 registers across the block loop
#pragma unroll
        for (int g4 = 0; g4 < 4; ++g4) {
          const f32x4 d4 = *reinterpret_cast<const f32x4*>(RC + 96 + 8 * g4 + 4 * hh);
#pragma unroll
          for (int e = 0; e < 4; ++e) pa[4 * g4 + e] = d4[e];
        }
        // kbase is a multiple of 32, so swz(kbase + kl, c) = kbase*D + swz(kl, c): written this
        // way the block offset folds into the ds_read immediate instead of costing a register
        bf16x8 kr[4];
#pragma unroll
        for (int s = 0; s < 4; ++s)
          kr[s] = *reinterpret_cast<const bf16x8*>(Kw + kb * 32 * D + swz(kl, 16 * s + 8 * hh));
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          pa = mfma(ofr[s], vf[kb][s], pa);  // dP - delta
          sa = mfma(qfr[s], kr[s], sa);      // (S - LSE2 -+ slope2 q) / c   [q][key]
        }
        const float kbias = ((padm_t >> kb) & 1) ? PAD_BIAS * LOG2E : 0.f;
        U = (after || before) ? fmaf(after ? slope2 : -slope2, (float)(kbase + kl_t), kbias) : kbias;
        if (!after && !before) {
          // diagonal block (qb == kbase): q - k at register offset 0 is 4hh - kl. Opaque to the
          // optimizer, which would otherwise keep the 16 loop-invariant |q - k| in registers
          float lq = (float)(4 * hh - kl);
          asm volatile("" : "+v"(lq));
#pragma unroll
          for (int r = 0; r < 16; ++r) sa[r] = fmaf(-sl_t, fabsf(lq + (float)aoff(r)), sa[r]);
        }
      }
      __builtin_amdgcn_sched_barrier(0);
      bf16x8 pb[2], sb[2];
      // dO^T / Q^T operands of the dV / dK MFMAs, two pairs in flight (even / odd pair slots):
      // pair j + 2's transposed reads are issued as soon as pair j's MFMAs have taken their
      // operands, so each read has a whole pair of MFMAs and score work to land
      bf16x8 ao[2], aq[2];
      float ssum = 0.f;
      const float sold = (DBL && kb < KB) ? sigl[hh * S + kbase + kl_t] : 0.f;
      if (kb > 0) {
        ao[0] = tr_pair(O, 0); aq[0] = tr_pair(Q, 0);
        ao[1] = tr_pair(O, 1); aq[1] = tr_pair(Q, 1);
      }
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        if (kb > 0) {  // dV/dK MFMA i of block kb-1: pair j = i >> 1 = (s2, dt), dV then dK
          const int j = i >> 1;
          if ((i & 1) == 0) {
            mfma_acc(dv[kb - 1][j & 1], ao[j & 1], pbp[j >> 1]);
          } else {
            mfma_acc(dk[kb - 1][j & 1], aq[j & 1], sbp[j >> 1]);
            if (j < 2) { ao[j & 1] = tr_pair(O, j + 2); aq[j & 1] = tr_pair(Q, j + 2); }
          }
        }
        if (kb < KB) {  // scores 2i, 2i+1 of block kb
#pragma unroll
          for (int r = 2 * i; r < 2 * i + 2; ++r) {
            const float pr = ex2(fmaf(sa[r], c, U));
            const float ds = pr * pa[r];
            pb[r >> 3][r & 7] = (bf16)pr;
            sb[r >> 3][r & 7] = (bf16)ds;
            if (DBL) ssum += ds;
          }
        }
        if (PIPE_SB) __builtin_amdgcn_sched_barrier(0);
      }
      if (kb > 0) {
        // dS^T image of block kb-1: register group g holds q = 8g + 4hh + 0..3 of key kl (the
        // chunk swizzle ((key >> 1) & 7) depends on kl only, blocks being 32-aligned). A 16-lane
        // ds_write_b64 group (kl 0..15) then covers all 32 banks of its (a/4) mod 32 map: the
        // odd / even kl split the two 64-B halves, (kl >> 1) & 7 the 8-B slots (the former
        // (kl >> 2) & 7 key put kl and kl + 2 on one bank: a 2-way conflict on every write)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const bf16x8& src = sbp[g >> 1];
          const bf16x4 v = {src[4 * (g & 1)], src[4 * (g & 1) + 1], src[4 * (g & 1) + 2], src[4 * (g & 1) + 3]};
          *reinterpret_cast<bf16x4*>(dSTw + (kb - 1) * 32 * 32 + kl * 32 + 4 * ((2 * g + hh) ^ ((kl >> 1) & 7))) = v;
        }
      }
      if (kb < KB) {
        if (DBL) sigl[hh * S + kbase + kl_t] = sold + ssum;
        pbp[0] = pb[0]; pbp[1] = pb[1];
        sbp[0] = sb[0]; sbp[1] = sb[1];
      }
    }
    BWD3_STAMP(t, 1);
    __syncthreads();
    BWD3_STAMP(t, 2);
    // ---- phase 2: dQ^T[32 dth + d][q] over keys [kh2*S/2, (kh2+1)*S/2)
    f32x16 dq;
#pragma unroll
    for (int i = 0; i < 16; ++i) dq[i] = 0.f;
    {
      const int dcol = 32 * dth + 16 * (g16 & 1) + 4 * (i16 & 3);
      const int qc = 4 * (g16 & 1) + (i16 & 3);  // 8-B chunk of q = 16(g16&1) + 4(i16&3)
      // rows 16ks + r (r = 4hh + (i16>>2), and + 8): swz(16ks + r, c) = 16ks*D + swz(r, c); the
      // dS^T chunk swizzle ((row >> 1) & 7) = (r >> 1) & 7 does not depend on ks
      const int rr = 4 * (g16 >> 1) + (i16 >> 2);
      const int ka0 = swz(rr, dcol), ka1 = swz(rr + 8, dcol);
      const int sa0 = rr * 32 + 4 * (qc ^ ((rr >> 1) & 7));
      const int sa1 = (rr + 8) * 32 + 4 * (qc ^ (((rr + 8) >> 1) & 7));
      // operands of step ks + PF are read while step ks multiplies (LDS latency off the chain)
      constexpr int PF = KS2 < 4 ? KS2 : 4;
      bf16x8 ra[PF], rb[PF];
      auto rd = [&](int ks, bf16x8& a, bf16x8& bb) {
        a = cat(tr_read(Kh + 16 * ks * D + ka0), tr_read(Kh + 16 * ks * D + ka1));
        bb = cat(tr_read(dSTh + 16 * ks * 32 + sa0), tr_read(dSTh + 16 * ks * 32 + sa1));
      };
#pragma unroll
      for (int ks = 0; ks < PF; ++ks) rd(ks, ra[ks], rb[ks]);
#pragma unroll
      for (int ks = 0; ks < KS2; ++ks) {
        dq = mfma(ra[ks % PF], rb[ks % PF], dq);
        if (ks + PF < KS2) rd(ks + PF, ra[ks % PF], rb[ks % PF]);
      }
    }
    // key-half partials: the two waves of a 32-d half each finish two of the four register
    // groups (g = 2*kh2, 2*kh2 + 1), exchanging the other two through LDS; own + partner is the
    // same fp32 sum either way round (a + b == b + a), so dQ stays deterministic
    float* rw = red + dth * 1024;
#pragma unroll
    for (int g2 = 0; g2 < 2; ++g2) {
      const int g = 2 * (1 - kh2) + g2;
      *reinterpret_cast<f32x4*>(rw + g * 256 + lane * 4) = f32x4{dq[4 * g], dq[4 * g + 1], dq[4 * g + 2], dq[4 * g + 3]};
    }
    BWD3_STAMP(t, 3);
    if (t + 1 < NS) store_slice(buf ^ 1, t + 1, nx, tid_t);
    __syncthreads();
    BWD3_STAMP(t, 4);
    {
      bf16* row = dqkv + ((size_t)b * S + qb + kl) * ld + h * D + 32 * dth;
#pragma unroll
      for (int g2 = 0; g2 < 2; ++g2) {
        const int g = 2 * kh2 + g2;
        const f32x4 v = *reinterpret_cast<const f32x4*>(rw + g * 256 + lane * 4);
        bf16x4 o;
#pragma unroll
        for (int e = 0; e < 4; ++e) o[e] = (bf16)((dq[4 * g + e] + v[e]) * scale);
        *reinterpret_cast<bf16x4*>(row + 8 * g + 4 * hh) = o;
      }
    }
    BWD3_STAMP(t, 5);
  }

  // ---- dK, dV rows of this wave's keys
#pragma unroll
  for (int kb = 0; kb < KB; ++kb)
#pragma unroll
    for (int dt = 0; dt < 2; ++dt) acc_fence(dk[kb][dt], dv[kb][dt]);
#pragma unroll
  for (int kb = 0; kb < KB; ++kb) {
    bf16* row = dqkv + ((size_t)b * S + wave * KPW + 32 * kb + kl) * ld + h * D;
#pragma unroll
    for (int dt = 0; dt < 2; ++dt)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        bf16x4 vk, vv;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          vk[e] = (bf16)(dk[kb][dt][4 * g + e] * scale);
          vv[e] = (bf16)dv[kb][dt][4 * g + e];
        }
        *reinterpret_cast<bf16x4*>(row + H * D + 32 * dt + 8 * g + 4 * hh) = vk;
        *reinterpret_cast<bf16x4*>(row + 2 * H * D + 32 * dt + 8 * g + 4 * hh) = vv;
      }
  }
  if (DBE) {  // column sums per 128 keys: per-wave sums via LDS, then 4/KB waves per row
    // re-read the accumulators below instead of keeping the 256 values read for the stores live
#pragma unroll
    for (int kb = 0; kb < KB; ++kb)
#pragma unroll
      for (int dt = 0; dt < 2; ++dt) asm volatile("" : "+a"(dk[kb][dt]), "+a"(dv[kb][dt]));
    __syncthreads();  // the last slice's dQ partials in `red` have been read
    // lane ids opaque here, so no epilogue address is computed (and kept live) before the loop
    int lane_e = lane;
    asm volatile("" : "+v"(lane_e));
    const int kl_e = lane_e & 31, hh_e = lane_e >> 5;
    float* cs = red;  // [wave][dQ, dK, dV][64]
    // per tensor: each lane_e writes its per-key partials (key kl_e) into a wave-private [64 d][key]
    // image, then lane_e = d sums its row of 32 keys (LDS is in order within a wave: no barriers)
    float* st = (bwd3_stage_alias<KB>() ? reinterpret_cast<float*>(Qimg)
                                        : red + 2 * 1024 + 2 * S) + wave * 64 * CS_LD;
    auto rowsum = [&](float* dst) {
      f32x4 a = *reinterpret_cast<const f32x4*>(st + lane_e * CS_LD);
#pragma unroll
      for (int k = 4; k < 32; k += 4) {
        const f32x4 v = *reinterpret_cast<const f32x4*>(st + lane_e * CS_LD + k);
        a[0] += v[0]; a[1] += v[1]; a[2] += v[2]; a[3] += v[3];
      }
      *dst = (a[0] + a[1]) + (a[2] + a[3]);
    };
    {  // dQ part: sum_kb K[key][d] * sigma[key] over this lane_e's half of d; sigma needs both lane_e
       // halves' query rows
      float sgm[KB];
#pragma unroll
      for (int kb = 0; kb < KB; ++kb) {
        const int key = wave * KPW + 32 * kb + kl_e;
        sgm[kb] = sigl[key] + sigl[S + key];
      }
#pragma unroll
      for (int cc = 0; cc < 4; ++cc) {
        float a8[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int kb = 0; kb < KB; ++kb) {
          const int r = wave * KPW + 32 * kb + kl_e;
          const bf16x8 v = *reinterpret_cast<const bf16x8*>(Kimg + r * D + (((4 * hh_e + cc) ^ swz_key(r)) << 3));
#pragma unroll
          for (int e = 0; e < 8; ++e) a8[e] = fmaf((float)v[e], sgm[kb], a8[e]);
        }
#pragma unroll
        for (int e = 0; e < 8; ++e) st[(32 * hh_e + 8 * cc + e) * CS_LD + kl_e] = a8[e] * scale;
      }
      rowsum(cs + (wave * 3) * 64 + lane_e);
    }
#pragma unroll
    for (int ts = 0; ts < 2; ++ts) {  // dK (scaled), dV
#pragma unroll
      for (int dt = 0; dt < 2; ++dt)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          float sum = 0.f;
#pragma unroll
          for (int kb = 0; kb < KB; ++kb) sum += ts == 0 ? dk[kb][dt][r] : dv[kb][dt][r];
          st[(32 * dt + aoff(r) + 4 * hh_e) * CS_LD + kl_e] = ts == 0 ? sum * scale : sum;
        }
      rowsum(cs + (wave * 3 + 1 + ts) * 64 + lane_e);
    }
    __syncthreads();
    for (int i = tid; i < KB * 192; i += 256) {
      const int j = i / 192, ts = (i >> 6) % 3, d = i & 63;
      float sum = 0.f;
#pragma unroll
      for (int w = 0; w < 4 / KB; ++w) sum += cs[((j * 4 / KB + w) * 3 + ts) * 64 + d];
      dbias_part[((size_t)b * KB + j) * ld + ts * H * D + h * D + d] = sum;
    }
  }
}

// ----------------------------------------------------------------------------- fp32 path
// One thread per query (forward, dQ) or per key (dK/dV); K/V (or Q/dO) tiles staged in LDS.
constexpr int F32_TILE = 64;

__device__ __forceinline__ float bias_nat(float slope, int i, int j, const uint8_t* kv, size_t off) {
  float bb = -slope * fabsf((float)(i - j));
  if (kv && !kv[off + j]) bb += PAD_BIAS;
  return bb;
}

__global__ __launch_bounds__(64) void fwd_f32_kernel(const float* __restrict__ qkv,
                                                      const uint8_t* __restrict__ kv,
                                                      const float* __restrict__ slopes, int S,
                                                      int H, float scale, float* __restrict__ out,
                                                      float* __restrict__ lse) {
  __shared__ float Kt[F32_TILE][D + 1], Vt[F32_TILE][D + 1];
  const int h = blockIdx.y, b = blockIdx.z, t = threadIdx.x;
  const int qi = blockIdx.x * F32_TILE + t;
  const int ld = 3 * H * D;
  const float* base = qkv + (size_t)b * S * ld;
  const float slope = slopes[h];
  float q[D], o[D];
  const int qr = min(qi, S - 1);
  for (int d = 0; d < D; ++d) { q[d] = base[(size_t)qr * ld + h * D + d]; o[d] = 0.f; }
  float m = -INFINITY, l = 0.f;
  for (int k0 = 0; k0 < S; k0 += F32_TILE) {
    __syncthreads();
    for (int idx = t; idx < F32_TILE * D; idx += 64) {
      int r = idx / D, d = idx % D, j = min(k0 + r, S - 1);
      Kt[r][d] = base[(size_t)j * ld + H * D + h * D + d];
      Vt[r][d] = base[(size_t)j * ld + 2 * H * D + h * D + d];
    }
    __syncthreads();
    const int kn = min(F32_TILE, S - k0);
    for (int r = 0; r < kn; ++r) {
      float sdot = 0.f;
      for (int d = 0; d < D; ++d) sdot = fmaf(q[d], Kt[r][d], sdot);
      float x = sdot * scale + bias_nat(slope, qi, k0 + r, kv, (size_t)b * S);
      float mn = fmaxf(m, x);
      float a = __expf(m - mn), p = __expf(x - mn);
      l = l * a + p;
      for (int d = 0; d < D; ++d) o[d] = fmaf(p, Vt[r][d], o[d] * a);
      m = mn;
    }
  }
  if (qi < S) {
    float* orow = out + ((size_t)b * S + qi) * (H * D) + h * D;
    for (int d = 0; d < D; ++d) orow[d] = o[d] / l;
    lse[((size_t)b * H + h) * S + qi] = m + __logf(l);
  }
}

__global__ __launch_bounds__(64) void dq_f32_kernel(const float* __restrict__ qkv,
                                                     const float* __restrict__ dout,
                                                     const float* __restrict__ lse,
                                                     const float* __restrict__ delta,
                                                     const uint8_t* __restrict__ kv,
                                                     const float* __restrict__ slopes, int S,
                                                     int H, float scale, float* __restrict__ dqkv) {
  __shared__ float Kt[F32_TILE][D + 1], Vt[F32_TILE][D + 1];
  const int h = blockIdx.y, b = blockIdx.z, t = threadIdx.x;
  const int qi = blockIdx.x * F32_TILE + t;
  const int ld = 3 * H * D;
  const float* base = qkv + (size_t)b * S * ld;
  const float slope = slopes[h];
  const int qr = min(qi, S - 1);
  float q[D], g[D], dq[D];
  for (int d = 0; d < D; ++d) {
    q[d] = base[(size_t)qr * ld + h * D + d];
    g[d] = dout[((size_t)b * S + qr) * (H * D) + h * D + d];
    dq[d] = 0.f;
  }
  const float L = lse[((size_t)b * H + h) * S + qr], dl = delta[((size_t)b * H + h) * S + qr];
  for (int k0 = 0; k0 < S; k0 += F32_TILE) {
    __syncthreads();
    for (int idx = t; idx < F32_TILE * D; idx += 64) {
      int r = idx / D, d = idx % D, j = min(k0 + r, S - 1);
      Kt[r][d] = base[(size_t)j * ld + H * D + h * D + d];
      Vt[r][d] = base[(size_t)j * ld + 2 * H * D + h * D + d];
    }
    __syncthreads();
    const int kn = min(F32_TILE, S - k0);
    for (int r = 0; r < kn; ++r) {
      float sdot = 0.f, pdot = 0.f;
      for (int d = 0; d < D; ++d) { sdot = fmaf(q[d], Kt[r][d], sdot); pdot = fmaf(g[d], Vt[r][d], pdot); }
      float p = __expf(sdot * scale + bias_nat(slope, qi, k0 + r, kv, (size_t)b * S) - L);
      float dsv = p * (pdot - dl) * scale;
      for (int d = 0; d < D; ++d) dq[d] = fmaf(dsv, Kt[r][d], dq[d]);
    }
  }
  if (qi < S) {
    float* row = dqkv + ((size_t)b * S + qi) * ld + h * D;
    for (int d = 0; d < D; ++d) row[d] = dq[d];
  }
}

__global__ __launch_bounds__(64) void dkdv_f32_kernel(const float* __restrict__ qkv,
                                                       const float* __restrict__ dout,
                                                       const float* __restrict__ lse,
                                                       const float* __restrict__ delta,
                                                       const uint8_t* __restrict__ kv,
                                                       const float* __restrict__ slopes, int S,
                                                       int H, float scale,
                                                       float* __restrict__ dqkv) {
  __shared__ float Qt[F32_TILE][D + 1], Gt[F32_TILE][D + 1];
  __shared__ float Lt[F32_TILE], Dt[F32_TILE];
  const int h = blockIdx.y, b = blockIdx.z, t = threadIdx.x;
  const int kj = blockIdx.x * F32_TILE + t;
  const int ld = 3 * H * D;
  const float* base = qkv + (size_t)b * S * ld;
  const float slope = slopes[h];
  const int kr = min(kj, S - 1);
  float k[D], v[D], dk[D], dv[D];
  for (int d = 0; d < D; ++d) {
    k[d] = base[(size_t)kr * ld + H * D + h * D + d];
    v[d] = base[(size_t)kr * ld + 2 * H * D + h * D + d];
    dk[d] = dv[d] = 0.f;
  }
  const float kb = (kv && !kv[(size_t)b * S + kr]) ? PAD_BIAS : 0.f;
  for (int q0 = 0; q0 < S; q0 += F32_TILE) {
    __syncthreads();
    for (int idx = t; idx < F32_TILE * D; idx += 64) {
      int r = idx / D, d = idx % D, i = min(q0 + r, S - 1);
      Qt[r][d] = base[(size_t)i * ld + h * D + d];
      Gt[r][d] = dout[((size_t)b * S + i) * (H * D) + h * D + d];
    }
    if (t < F32_TILE) {
      int i = min(q0 + t, S - 1);
      Lt[t] = lse[((size_t)b * H + h) * S + i];
      Dt[t] = delta[((size_t)b * H + h) * S + i];
    }
    __syncthreads();
    const int qn = min(F32_TILE, S - q0);
    for (int r = 0; r < qn; ++r) {
      float sdot = 0.f, pdot = 0.f;
      for (int d = 0; d < D; ++d) { sdot = fmaf(Qt[r][d], k[d], sdot); pdot = fmaf(Gt[r][d], v[d], pdot); }
      float p = __expf(sdot * scale - slope * fabsf((float)(q0 + r - kj)) + kb - Lt[r]);
      float dsv = p * (pdot - Dt[r]) * scale;
      for (int d = 0; d < D; ++d) { dv[d] = fmaf(p, Gt[r][d], dv[d]); dk[d] = fmaf(dsv, Qt[r][d], dk[d]); }
    }
  }
  if (kj < S) {
    float* row = dqkv + ((size_t)b * S + kj) * ld + h * D;
    for (int d = 0; d < D; ++d) { row[H * D + d] = dk[d]; row[2 * H * D + d] = dv[d]; }
  }
}

constexpr size_t FWD_LDS = 2 * (2 * BK * D * sizeof(bf16)) + 2 * BK * sizeof(float);
constexpr size_t DKDV_LDS = 2 * (2 * BQT * D * sizeof(bf16)) + 4 * BQT * sizeof(float);
constexpr size_t DKDV2_LDS = 2 * (2 * BQT * D * sizeof(bf16)) + 8 * BQT * sizeof(float);

}  // namespace attn
}  // namespace dna

using namespace dna;
using namespace dna::attn;

static int check_common(const void* qkv, const float* slopes, int batch, int seqlen, int heads,
                        int head_dim, int dtype, const char* fn) {
  DNA_CHECK_ARG(qkv && slopes, "%s: null pointer", fn);
  DNA_CHECK_ARG(batch > 0 && seqlen > 0 && heads > 0, "%s: bad shape b=%d S=%d H=%d", fn, batch,
                seqlen, heads);
  if (head_dim != D) {
    set_error("%s: head_dim %d unsupported (64 only)", fn, head_dim);
    return DNA_ERR_UNSUPPORTED;
  }
  DNA_CHECK_ARG(dtype == DNA_F32 || dtype == DNA_BF16, "%s: bad dtype %d", fn, dtype);
  if (dtype == DNA_BF16 && seqlen % BK != 0) {
    set_error("%s: bf16 path needs seqlen %% 64 == 0 (got %d)", fn, seqlen);
    return DNA_ERR_UNSUPPORTED;
  }
  return DNA_OK;
}

extern "C" int dna_attn_fwd(const void* qkv, const uint8_t* key_valid, const float* slopes,
                            int batch, int seqlen, int heads, int head_dim, int dtype,
                            float softmax_scale, void* out, float* lse, void* stream) {
  int st = check_common(qkv, slopes, batch, seqlen, heads, head_dim, dtype, "dna_attn_fwd");
  if (st) return st;
  DNA_CHECK_ARG(out && lse, "dna_attn_fwd: null output");
  hipStream_t s = as_stream(stream);
  if (dtype == DNA_BF16) {
    // A/B switch for benchmarks: DNA_ATTN_FWD=1 runs the v1 forward
    static const int forced = getenv("DNA_ATTN_FWD") ? atoi(getenv("DNA_ATTN_FWD")) : 0;
    if (forced == 1) {
      dim3 grid(((seqlen + BQ - 1) / BQ) * heads * batch);
      hipLaunchKernelGGL(fwd_bf16_kernel, grid, dim3(256), FWD_LDS, s, (const bf16*)qkv,
                         key_valid, slopes, seqlen, heads, softmax_scale * LOG2E, (bf16*)out, lse);
    } else {
      if (forced == 4) {  // four 32-query blocks per wave, 1 wave per SIMD (A/B)
        dim3 grid(((seqlen + 511) / 512) * heads * batch);
        hipLaunchKernelGGL((fwd2_bf16_kernel<4>), grid, dim3(256), FWD_LDS, s, (const bf16*)qkv,
                           key_valid, slopes, seqlen, heads, softmax_scale * LOG2E, (bf16*)out, lse);
      } else if (forced == 3) {  // one 32-query block per wave, 3 waves per SIMD (A/B)
        dim3 grid(((seqlen + 127) / 128) * heads * batch);
        hipLaunchKernelGGL((fwd2_bf16_kernel<1>), grid, dim3(256), FWD_LDS, s, (const bf16*)qkv,
                           key_valid, slopes, seqlen, heads, softmax_scale * LOG2E, (bf16*)out, lse);
      } else if (forced != 2 && forced != 8 && fwd_dma_lds(seqlen) <= 96 * 1024) {
        // default: the LDS-DMA K/V ring (0.731 -> 0.712 ms at b = 512, interleaved A/B in
        // profiles/r06/ab_attn_fwd_dma.txt); DNA_ATTN_FWD=2 runs the register-staged form
        static const bool attr = [] {
          (void)hipFuncSetAttribute((const void*)fwd2_bf16_kernel<2, 4, true>,
                                    hipFuncAttributeMaxDynamicSharedMemorySize, 96 * 1024);
          return true;
        }();
        (void)attr;
        dim3 grid(((seqlen + BQ2 - 1) / BQ2) * heads * batch);
        hipLaunchKernelGGL((fwd2_bf16_kernel<2, 4, true>), grid, dim3(256), fwd_dma_lds(seqlen), s,
                           (const bf16*)qkv, key_valid, slopes, seqlen, heads,
                           softmax_scale * LOG2E, (bf16*)out, lse);
      } else if (forced == 8) {  // eight waves, 512 queries per workgroup (A/B)
        dim3 grid(((seqlen + 511) / 512) * heads * batch);
        hipLaunchKernelGGL((fwd2_bf16_kernel<2, 8>), grid, dim3(512), FWD_LDS, s, (const bf16*)qkv,
                           key_valid, slopes, seqlen, heads, softmax_scale * LOG2E, (bf16*)out, lse);
      } else {
        dim3 grid(((seqlen + BQ2 - 1) / BQ2) * heads * batch);
        hipLaunchKernelGGL((fwd2_bf16_kernel<2>), grid, dim3(256), FWD_LDS, s, (const bf16*)qkv,
                           key_valid, slopes, seqlen, heads, softmax_scale * LOG2E, (bf16*)out, lse);
      }
    }
  } else {
    dim3 grid((seqlen + F32_TILE - 1) / F32_TILE, heads, batch);
    hipLaunchKernelGGL(fwd_f32_kernel, grid, dim3(64), 0, s, (const float*)qkv, key_valid, slopes,
                       seqlen, heads, softmax_scale, (float*)out, lse);
  }
  DNA_LAUNCH_CHECK("dna_attn_fwd");
  return DNA_OK;
}

template <int KB>
static void launch_bwd3(const void* qkv, const void* out, const void* dout, const float* lse,
                        const uint8_t* key_valid, const float* slopes, int batch, int heads, float c,
                        float scale, void* dqkv, float* dbias_part, hipStream_t s) {
  static const bool attr = [] {
    const void* ks[] = {(const void*)bwd3_bf16_kernel<KB, 0>, (const void*)bwd3_bf16_kernel<KB, 1>,
                        (const void*)bwd3_bf16_kernel<KB, 2>, (const void*)bwd3_bf16_kernel<KB, 3>};
    for (const void* k : ks)
      (void)hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bwd3_lds<KB>());
    return true;
  }();
  (void)attr;
  // DNA_ATTN_BWD3_SB=1 (A/B): per-step sched_barriers in the software-pipelined phase 1
  static const bool sb = getenv("DNA_ATTN_BWD3_SB") && atoi(getenv("DNA_ATTN_BWD3_SB")) == 1;
  const dim3 grid(batch * heads);
  const size_t lds = bwd3_lds<KB>();
  auto args = [&](auto kern, float* part) {
    hipLaunchKernelGGL(kern, grid, dim3(256), lds, s, (const bf16*)qkv, (const bf16*)out,
                       (const bf16*)dout, lse, key_valid, slopes, heads, c, scale, (bf16*)dqkv, part);
  };
  if (!dbias_part) {
    if (sb) args(bwd3_bf16_kernel<KB, 2>, nullptr);
    else args(bwd3_bf16_kernel<KB, 0>, nullptr);
  } else {
    if (sb) args(bwd3_bf16_kernel<KB, 3>, dbias_part);
    else args(bwd3_bf16_kernel<KB, 1>, dbias_part);
  }
}

extern "C" int dna_attn_bwd_ex(const void* qkv, const void* out, const void* dout,
                               const float* lse, const uint8_t* key_valid, const float* slopes,
                               int batch, int seqlen, int heads, int head_dim, int dtype,
                               float softmax_scale, void* dqkv, float* delta_ws, float* dbias_part,
                               void* stream) {
  int st = check_common(qkv, slopes, batch, seqlen, heads, head_dim, dtype, "dna_attn_bwd");
  if (st) return st;
  DNA_CHECK_ARG(out && dout && lse && dqkv && delta_ws, "dna_attn_bwd: null pointer");
  hipStream_t s = as_stream(stream);
  const int rows = batch * seqlen;
  const int nd = (rows * heads + 255) / 256;
  // DNA_ATTN_BWD: 3 (default) fused one-workgroup-per-(batch, head) kernel where S is 128, 256
  // or 512, else the v2 pair; 2 forces the v2 pair, 1 the v1 pair (benchmarks / A/B)
  static const int bwd_ver = getenv("DNA_ATTN_BWD") ? atoi(getenv("DNA_ATTN_BWD")) : 3;
  const bool bwd_v1 = bwd_ver == 1;
  if (dtype == DNA_BF16 && bwd_ver == 3 && (seqlen == 128 || seqlen == 256 || seqlen == 512)) {
    const float c = softmax_scale * LOG2E;
    if (seqlen == 512)
      launch_bwd3<4>(qkv, out, dout, lse, key_valid, slopes, batch, heads, c, softmax_scale, dqkv, dbias_part, s);
    else if (seqlen == 256)
      launch_bwd3<2>(qkv, out, dout, lse, key_valid, slopes, batch, heads, c, softmax_scale, dqkv, dbias_part, s);
    else
      launch_bwd3<1>(qkv, out, dout, lse, key_valid, slopes, batch, heads, c, softmax_scale, dqkv, dbias_part, s);
  } else if (dtype == DNA_BF16 && !bwd_v1) {
    // dQ kernel also produces delta = rowsum(dO*O), consumed by the dK/dV kernel after it.
    // 8-wave workgroups (256 queries / keys each) when the sequence fills them: half the
    // K/V and Q/dO re-streaming of 4-wave ones. Colsum scratch: NW*32 rows x 64 floats.
    static const int nw_env = getenv("DNA_ATTN_BWD_NW") ? atoi(getenv("DNA_ATTN_BWD_NW")) : 8;
    const bool w8 = nw_env == 8 && seqlen % 256 == 0;
    const size_t red = (w8 ? 8 : 4) * 32 * 64 * sizeof(float);
    const size_t dq_lds = std::max(FWD_LDS, dbias_part ? red : (size_t)0);
    const size_t kv_lds = std::max(DKDV2_LDS, dbias_part ? red : (size_t)0);
    if (w8) {
      hipLaunchKernelGGL((dq2_bf16_kernel<8>), dim3((seqlen / 256) * heads * batch), dim3(512),
                         dq_lds, s, (const bf16*)qkv, (const bf16*)out, (const bf16*)dout, lse,
                         delta_ws, key_valid, slopes, seqlen, heads, softmax_scale * LOG2E,
                         softmax_scale, (bf16*)dqkv, dbias_part);
      hipLaunchKernelGGL((dkdv2_bf16_kernel<8>), dim3((seqlen / 256) * heads * batch), dim3(512),
                         kv_lds, s, (const bf16*)qkv, (const bf16*)dout, lse, delta_ws, key_valid,
                         slopes, seqlen, heads, softmax_scale * LOG2E, softmax_scale, (bf16*)dqkv,
                         dbias_part);
    } else {
      hipLaunchKernelGGL((dq2_bf16_kernel<4>), dim3(((seqlen + BQ - 1) / BQ) * heads * batch),
                         dim3(256), dq_lds, s, (const bf16*)qkv, (const bf16*)out,
                         (const bf16*)dout, lse, delta_ws, key_valid, slopes, seqlen, heads,
                         softmax_scale * LOG2E, softmax_scale, (bf16*)dqkv, dbias_part);
      hipLaunchKernelGGL((dkdv2_bf16_kernel<4>), dim3(((seqlen + BKW - 1) / BKW) * heads * batch),
                         dim3(256), kv_lds, s, (const bf16*)qkv, (const bf16*)dout, lse, delta_ws,
                         key_valid, slopes, seqlen, heads, softmax_scale * LOG2E, softmax_scale,
                         (bf16*)dqkv, dbias_part);
    }
  } else if (dtype == DNA_BF16) {  // v1 kernels (DNA_ATTN_BWD=1, benchmarks)
    hipLaunchKernelGGL(dq_bf16_kernel, dim3(((seqlen + BQ - 1) / BQ) * heads * batch), dim3(256),
                       FWD_LDS, s, (const bf16*)qkv, (const bf16*)out, (const bf16*)dout, lse,
                       delta_ws, key_valid, slopes, seqlen, heads, softmax_scale * LOG2E,
                       softmax_scale, (bf16*)dqkv, dbias_part);
    hipLaunchKernelGGL(dkdv_bf16_kernel, dim3(((seqlen + BKW - 1) / BKW) * heads * batch), dim3(256),
                       DKDV_LDS, s, (const bf16*)qkv, (const bf16*)dout, lse, delta_ws, key_valid,
                       slopes, seqlen, heads, softmax_scale * LOG2E, softmax_scale, (bf16*)dqkv,
                       dbias_part);
  } else {
    DNA_CHECK_ARG(!dbias_part, "dna_attn_bwd_ex: fused bias-gradient partials need the bf16 path");
    hipLaunchKernelGGL(delta_kernel<float>, dim3(nd), dim3(256), 0, s, (const float*)out,
                       (const float*)dout, rows, heads, seqlen, delta_ws);
    dim3 grid((seqlen + F32_TILE - 1) / F32_TILE, heads, batch);
    hipLaunchKernelGGL(dq_f32_kernel, grid, dim3(64), 0, s, (const float*)qkv, (const float*)dout,
                       lse, delta_ws, key_valid, slopes, seqlen, heads, softmax_scale,
                       (float*)dqkv);
    hipLaunchKernelGGL(dkdv_f32_kernel, grid, dim3(64), 0, s, (const float*)qkv,
                       (const float*)dout, lse, delta_ws, key_valid, slopes, seqlen, heads,
                       softmax_scale, (float*)dqkv);
  }
  DNA_LAUNCH_CHECK("dna_attn_bwd");
  return DNA_OK;
}

extern "C" int dna_attn_bwd(const void* qkv, const void* out, const void* dout, const float* lse,
                            const uint8_t* key_valid, const float* slopes, int batch, int seqlen,
                            int heads, int head_dim, int dtype, float softmax_scale, void* dqkv,
                            float* delta_ws, void* stream) {
  return dna_attn_bwd_ex(qkv, out, dout, lse, key_valid, slopes, batch, seqlen, heads, head_dim,
                         dtype, softmax_scale, dqkv, delta_ws, nullptr, stream);
}

#if DNA_BWD3_STAMP
extern "C" int dna_attn_debug_stamps(unsigned long long* out) {  // debug builds only
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_bwd3_stamps), sizeof(g_bwd3_stamps)) == hipSuccess ? 0 : 1;
}
#endif

extern "C" int dna_attn_dbias_part_rows(int batch, int seqlen) {
  return batch * ((seqlen + BQ - 1) / BQ);
}
