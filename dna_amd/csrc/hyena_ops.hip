// HyenaOperator data movement around the long convolution (reference
// src/models/sequence/hyena.py:421-509), fused for gfx950. The reference runs, per layer:
//   u = in_proj(x) [B, L, C] -> rearrange "b l d -> b d l" -> depthwise causal Conv1d (kernel K,
//   padding K-1, first L outputs) -> split into x_0 .. x_{order-1}, v (d channels each) ->
//   v = v * x_{order-1} -> long conv -> ... -> y = v * x_0 -> rearrange back -> out_proj.
// Here:
//   shortconv_fwd : u (token-major) -> x_0 .. x_{order-2} and v*x_{order-1}, channel-major, in one
//                   pass (transpose through LDS; the conv needs a (K-1)-row halo);
//   gate_out_fwd  : y = v_conv * x_0, channel-major in, token-major out (for out_proj);
//   gate_out_bwd  : dy (token-major) -> d(v_conv) = dy x_0 and dx_0 = dy v_conv, channel-major;
//   shortconv_bwd : d(x_0..x_{order-2}), d(v*x_{order-1}) -> du (token-major), recomputing the
//                   conv outputs it needs from u; dw, dbias as per-block partials (reduced by
//                   dna_colsum_f32 in a fixed order: deterministic).
// Tiles: 64 positions x 32 channels per block of 256 threads (small LDS footprint -> several
// blocks per CU); tiles load with 16-byte vectors; for the conv, lane = position (coalesced
// channel-major rows) and wave = an 8-channel slice. All math in fp32; HBM-bound.
#include <stdlib.h>

#include "common.h"

namespace dna {
namespace hyop {

constexpr int TP = 64;   // positions per tile
constexpr int TC = 32;   // channels per tile
constexpr int CPW = TC / 4;  // channels per wave in the conv phases
constexpr int PAD = 1;   // LDS row padding (floats)
typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2;

template <typename T>
__device__ __forceinline__ T cvt(float v) { return from_f32<T>(v); }

template <typename T, int LO, int HI>
struct TokTile {
  static constexpr int VE = 16 / sizeof(T);      // elements per vector
  static constexpr int VPR = TC / VE;            // vectors per row
  static constexpr int ROWS = TP + LO + HI;
  static constexpr int NIT = (ROWS * VPR + 255) / 256;  // per group and thread (256-thread blocks)
};
template <typename T, int LO, int HI, int G, int NIT = TokTile<T, LO, HI>::NIT>
__device__ __forceinline__ void tok_fetch(uint4 (&raw)[G][NIT], const T* src,
                                          int L, int ldc, int t0, int d, int col0) {
  using TT = TokTile<T, LO, HI>;
#pragma unroll
  for (int g = 0; g < G; ++g)
#pragma unroll
    for (int it = 0; it < TT::NIT; ++it) {
      const int i = threadIdx.x + it * 256;
      const int r = i / TT::VPR, cv = (i - r * TT::VPR) * TT::VE;
      const int t = t0 - LO + r;
      raw[g][it] = make_uint4(0u, 0u, 0u, 0u);
      if (i < TT::ROWS * TT::VPR && t >= 0 && t < L)
        raw[g][it] = *reinterpret_cast<const uint4*>(src + (size_t)t * ldc + g * d + col0 + cv);
    }
}
template <typename T, int LO, int HI, int G, int NIT = TokTile<T, LO, HI>::NIT>
__device__ __forceinline__ void tok_store(float* lds, const uint4 (&raw)[G][NIT]) {
  using TT = TokTile<T, LO, HI>;
#pragma unroll
  for (int g = 0; g < G; ++g)
#pragma unroll
    for (int it = 0; it < TT::NIT; ++it) {
      const int i = threadIdx.x + it * 256;
      if (i >= TT::ROWS * TT::VPR) continue;
      const int r = i / TT::VPR, cv = (i - r * TT::VPR) * TT::VE;
      float* dst = lds + (g * TT::ROWS + r) * (TC + PAD) + cv;
      const T* e = reinterpret_cast<const T*>(&raw[g][it]);
#pragma unroll
      for (int q = 0; q < TT::VE; ++q) dst[q] = to_f32(e[q]);
    }
}
// The u tile in the backward's LDS: bf16 rows kept as bf16 (68-B rows: 34 elements), fp32 as fp32
// (TC + PAD); the raw 16-B vectors stored as 4-B words (rows are 4-B aligned).
template <typename T> struct UTile {
  typedef T type;
  static constexpr int LW = sizeof(T) == 2 ? TC + 2 : TC + PAD;
};
template <typename T, int LO, int HI, int G, int NIT = TokTile<T, LO, HI>::NIT>
__device__ __forceinline__ void tok_store_raw(T* lds, const uint4 (&raw)[G][NIT]) {
  using TT = TokTile<T, LO, HI>;
  constexpr int LW = UTile<T>::LW;
#pragma unroll
  for (int g = 0; g < G; ++g)
#pragma unroll
    for (int it = 0; it < NIT; ++it) {
      const int i = threadIdx.x + it * 256;
      if (i >= TT::ROWS * TT::VPR) continue;
      const int r = i / TT::VPR, cv = (i - r * TT::VPR) * TT::VE;
      uint32_t* dst = reinterpret_cast<uint32_t*>(lds + (g * TT::ROWS + r) * LW + cv);
      dst[0] = raw[g][it].x; dst[1] = raw[g][it].y; dst[2] = raw[g][it].z; dst[3] = raw[g][it].w;
    }
}
// Load rows [t0 - LO, t0 + TP + HI) x channels [g*d + col0, + TC) of the G channel groups of a
// token-major [L, ldc] matrix into lds[g][row][TC + PAD] (zero outside [0, L)), 16-byte vectors
// along the channels. Every load of a thread (all groups) is issued before the first LDS store:
// these kernels are memory-latency bound (PMC: 78-92 % of wave cycles in s_waitcnt), and a
// load -> convert -> store loop kept one 16-B load per thread in flight.
template <typename T, int LO, int HI, int G>
__device__ __forceinline__ void load_tok_tiles(float* lds, const T* src, int L, int ldc, int t0,
                                               int d, int col0) {
  uint4 raw[G][TokTile<T, LO, HI>::NIT];
  tok_fetch<T, LO, HI, G>(raw, src, L, ldc, t0, d, col0);
  tok_store<T, LO, HI, G>(lds, raw);
}

struct Fwd {
  const void* u; const float* w; const float* bias; int B, L, d, order, K;
  void* xs; void* vx;
  int nct;  // channel tiles per block, run one after the other (see nct_for)
};

template <typename T, int K, int ORD>
__global__ __launch_bounds__(256) void shortconv_fwd_kernel(Fwd a) {
  extern __shared__ float smem[];
  constexpr int G = ORD + 1;  // channel groups x_0 .. x_{order-1}, v (compile-time: exact unrolls)
  const int C = G * a.d;
  const int t0 = blockIdx.x * TP, b = blockIdx.z;
  const int R = TP + K - 1;  // rows incl. halo
  const T* u = (const T*)a.u + (size_t)b * a.L * C;
  for (int ct = 0; ct < a.nct; ++ct) {
  const int c0 = (blockIdx.y * a.nct + ct) * TC;
  if (ct > 0) __syncthreads();  // the previous tile's LDS reads are done
  load_tok_tiles<T, K - 1, 0, G>(smem, u, a.L, C, t0, a.d, c0);
  __syncthreads();
  // lane = (channel jj of the wave's 8, chunk pc of 8 positions): the lane's 8 outputs of a group
  // come from K + 7 LDS reads of one column and leave as one 16-B (bf16) / two 16-B (fp32) store
  // of the channel-major row (when L % 8 == 0); bank = 8 pc + jj: conflict-free
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int jj = lane >> 3, pc = lane & 7;
  const int j = wv * CPW + jj, c = c0 + j, tl0 = t0 + 8 * pc;
  const bool full = (a.L & 7) == 0 && tl0 + 8 <= a.L;
  float last[8];  // conv of group order-1 (x_{order-1})
#pragma unroll
  for (int g = 0; g < G; ++g) {
    const int ch = g * a.d + c;
    const float* tl = smem + g * R * (TC + PAD) + j;
    float xv[8 + K - 1];
#pragma unroll
    for (int i = 0; i < 8 + K - 1; ++i) xv[i] = tl[(8 * pc + i) * (TC + PAD)];
    float wk[K];
#pragma unroll
    for (int k = 0; k < K; ++k) wk[k] = a.w[ch * K + k];
    const float bc = a.bias[ch];
    float o[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      float acc = bc;
#pragma unroll
      for (int k = 0; k < K; ++k) acc = fmaf(wk[k], xv[i + k], acc);
      o[i] = acc;
    }
    if (g == ORD - 1) {
#pragma unroll
      for (int i = 0; i < 8; ++i) last[i] = o[i];
      continue;
    }
    if (g == ORD) {
#pragma unroll
      for (int i = 0; i < 8; ++i) o[i] *= last[i];
    }
    T* row = g < ORD - 1 ? (T*)a.xs + ((size_t)b * (ORD - 1) * a.d + g * a.d + c) * a.L
                         : (T*)a.vx + ((size_t)b * a.d + c) * a.L;
    if (full) {
      if constexpr (sizeof(T) == 2) {
        bf16x8 v;
#pragma unroll
        for (int i = 0; i < 8; ++i) v[i] = (bf16)o[i];
        *reinterpret_cast<bf16x8*>(row + tl0) = v;
      } else {
        *reinterpret_cast<float4*>(row + tl0) = make_float4(o[0], o[1], o[2], o[3]);
        *reinterpret_cast<float4*>(row + tl0 + 4) = make_float4(o[4], o[5], o[6], o[7]);
      }
    } else {
#pragma unroll
      for (int i = 0; i < 8; ++i)
        if (tl0 + i < a.L) row[tl0 + i] = cvt<T>(o[i]);
    }
  }
  }
}

// 8 consecutive elements <-> fp32 (one 16-B bf16 / two 16-B fp32 accesses; p 16-B aligned)
template <typename T>
__device__ __forceinline__ void ld8(const T* p, float (&v)[8]) {
  if constexpr (sizeof(T) == 2) {
    const bf16x8 q = *reinterpret_cast<const bf16x8*>(p);
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = (float)q[i];
  } else {
    const float4 x = *reinterpret_cast<const float4*>(p), y = *reinterpret_cast<const float4*>(p + 4);
    v[0] = x.x; v[1] = x.y; v[2] = x.z; v[3] = x.w; v[4] = y.x; v[5] = y.y; v[6] = y.z; v[7] = y.w;
  }
}
template <typename T>
__device__ __forceinline__ void st8(T* p, const float (&v)[8]) {
  if constexpr (sizeof(T) == 2) {
    bf16x8 q;
#pragma unroll
    for (int i = 0; i < 8; ++i) q[i] = (bf16)v[i];
    *reinterpret_cast<bf16x8*>(p) = q;
  } else {
    *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
    *reinterpret_cast<float4*>(p + 4) = make_float4(v[4], v[5], v[6], v[7]);
  }
}
// bounded forms (the tail of a row, or rows not 16-B aligned)
template <typename T>
__device__ __forceinline__ void ld8b(const T* p, int n, float (&v)[8]) {
#pragma unroll
  for (int i = 0; i < 8; ++i) v[i] = i < n ? to_f32(p[i]) : 0.f;
}
template <typename T>
__device__ __forceinline__ void st8b(T* p, int n, const float (&v)[8]) {
#pragma unroll
  for (int i = 0; i < 8; ++i)
    if (i < n) p[i] = cvt<T>(v[i]);
}

// y[b, t, c] = yc[b, c, t] * x0[b, c, t]. Channel-major side: lane = (channel of the wave's 8,
// chunk of 8 positions), 16-B accesses; token-major side: lane = (row of 16, 8-channel chunk of
// 4), one 16-B access per row (vec: L, d and the batch stride multiples of 8, aligned rows).
// LDS rows of TP + 2 floats: both phases conflict-free or 2-way.
constexpr int GW = TP + 2;
template <typename T>
__global__ __launch_bounds__(256) void gate_out_fwd_kernel(const T* yc, const T* x0, int L, int d,
                                                           size_t x0_bstride, int vec, T* y) {
  __shared__ float tile[TC][GW];
  const int t0 = blockIdx.x * TP, c0 = blockIdx.y * TC, b = blockIdx.z;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  {
    const int j = wv * CPW + (lane >> 3), pc = lane & 7, t = t0 + 8 * pc;
    const T* py = yc + ((size_t)b * d + c0 + j) * L + t;
    const T* px = x0 + (size_t)b * x0_bstride + (size_t)(c0 + j) * L + t;
    float vy[8], vx[8];
    if (vec && t + 8 <= L) { ld8(py, vy); ld8(px, vx); }
    else { ld8b(py, L - t, vy); ld8b(px, L - t, vx); }
#pragma unroll
    for (int i = 0; i < 8; ++i) tile[j][8 * pc + i] = vy[i] * vx[i];
  }
  __syncthreads();
  const int cc8 = 8 * (lane & 3), rsub = lane >> 2;
  for (int r = wv * 16 + rsub; r < TP; r += 64) {
    const int t = t0 + r;
    if (t >= L) break;
    float v[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = tile[cc8 + e][r];
    T* o = y + ((size_t)b * L + t) * d + c0 + cc8;
    if (vec) st8(o, v);
    else st8b(o, 8, v);
  }
}

// dyc = dy * x0, dx0 = dy * yc (channel-major outputs; dy token-major); the same two lane maps
template <typename T>
__global__ __launch_bounds__(256) void gate_out_bwd_kernel(const T* dy, const T* yc, const T* x0,
                                                           int L, int d, size_t x_bstride, int vec,
                                                           T* dyc, T* dx0) {
  __shared__ float tile[TP][TC + PAD];
  const int t0 = blockIdx.x * TP, c0 = blockIdx.y * TC, b = blockIdx.z;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int j = wv * CPW + (lane >> 3), pc = lane & 7, tl0 = t0 + 8 * pc;
  const size_t o = ((size_t)b * d + c0 + j) * L + tl0;
  const size_t ox = (size_t)b * x_bstride + (size_t)(c0 + j) * L + tl0;
  const bool full = vec && tl0 + 8 <= L;
  // the channel-major loads first (registers), then dy through LDS
  float vx[8], vy[8];
  if (full) { ld8(x0 + ox, vx); ld8(yc + o, vy); }
  else { ld8b(x0 + ox, L - tl0, vx); ld8b(yc + o, L - tl0, vy); }
  const int cc8 = 8 * (lane & 3), rsub = lane >> 2;
  for (int r = wv * 16 + rsub; r < TP; r += 64) {
    const int t = t0 + r;
    float v[8];
    const T* p = dy + ((size_t)b * L + t) * d + c0 + cc8;
    if (t >= L) {
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = 0.f;
    } else if (vec) ld8(p, v);
    else ld8b(p, 8, v);
#pragma unroll
    for (int e = 0; e < 8; ++e) tile[r][cc8 + e] = v[e];
  }
  __syncthreads();
  if (tl0 >= L) return;
  float g[8], a[8], c[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    g[i] = tile[8 * pc + i][j];
    a[i] = g[i] * vx[i];
    c[i] = g[i] * vy[i];
  }
  if (full) { st8(dyc + o, a); st8(dx0 + ox, c); }
  else { st8b(dyc + o, L - tl0, a); st8b(dx0 + ox, L - tl0, c); }
}

// The implicit filter's ExponentialModulation fused with the [L, C] -> [O][C/O][L] transpose the
// long convolution reads (reference hyena.py:140-163 and :438-441): k[o][v][t] = h[t][c] *
// (exp(-tpos[t] * |delta[c]|) + shift), c = v * O + o. One 64 x 64 LDS tile per block; the
// backward runs the same transpose the other way, dh[t][c] = dk[o][v][t] * (same factor).
constexpr int MT = 64;
__device__ __forceinline__ float modf_(const float* tpos, const float* delta, float shift, int t, int c) {
  return expf(-tpos[t] * fabsf(delta[c])) + shift;
}
template <typename TH>
__global__ __launch_bounds__(256) void modulate_t_fwd_kernel(const TH* __restrict__ h, const float* __restrict__ tpos,
                                                             const float* __restrict__ delta, float shift,
                                                             int L, int C, int O, float* __restrict__ k) {
  __shared__ float tile[MT][MT + 1];
  const int t0 = blockIdx.x * MT, c0 = blockIdx.y * MT;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  for (int r = wv; r < MT; r += 4) {
    const int t = t0 + r, c = c0 + lane;
    tile[r][lane] = (t < L && c < C) ? to_f32(h[(size_t)t * C + c]) * modf_(tpos, delta, shift, t, c) : 0.f;
  }
  __syncthreads();
  const int V = C / O;
  for (int r = wv; r < MT; r += 4) {
    const int c = c0 + r, t = t0 + lane;
    if (c < C && t < L) k[((size_t)(c % O) * V + c / O) * L + t] = tile[lane][r];
  }
}
template <typename TH>
__global__ __launch_bounds__(256) void modulate_t_bwd_kernel(const float* __restrict__ dk, const float* __restrict__ tpos,
                                                             const float* __restrict__ delta, float shift,
                                                             int L, int C, int O, TH* __restrict__ dh) {
  __shared__ float tile[MT][MT + 1];
  const int t0 = blockIdx.x * MT, c0 = blockIdx.y * MT;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int V = C / O;
  for (int r = wv; r < MT; r += 4) {
    const int c = c0 + r, t = t0 + lane;
    tile[r][lane] = (c < C && t < L) ? dk[((size_t)(c % O) * V + c / O) * L + t] : 0.f;
  }
  __syncthreads();
  for (int r = wv; r < MT; r += 4) {
    const int t = t0 + r, c = c0 + lane;
    if (t < L && c < C) dh[(size_t)t * C + c] = cvt<TH>(tile[lane][r] * modf_(tpos, delta, shift, t, c));
  }
}

struct Bwd {
  const void* u; const float* w; const float* bias; int B, L, d, order, K;
  const void* dxs; const void* dvx; void* du; float* part;  // part [B * nL][C][K + 1]
};

// duc (d of the conv outputs) at positions [t0, t0 + TP + K - 1), then
//   du[t, ch]  = sum_k w[ch][k] duc[t + K - 1 - k]
//   dw[ch][k] += sum_{t in tile} duc[t] u[t - (K - 1 - k)],  dbias[ch] += sum_{t in tile} duc[t]
// Work split (all 256 threads busy in every phase): the duc rows of a wave's 8 channels are one
// flat (channel, row) range over the lanes, so the K - 1 halo rows do not cost a second full pass;
// du is written as channel pairs (4-B bf16 / 8-B fp32 stores, 16 pairs x 4 rows per wave pass);
// the dw / dbias tile sums are split into 4 row quarters per (group, channel) and combined in LDS
// in a fixed order before the per-tile partial is written (deterministic).
// A block runs NCT channel tiles of one position tile, software-pipelined: every HBM load of tile
// ct + 1 (its u rows and its d(x) / d(v x) rows, into registers) is issued right after tile ct's
// u rows reach LDS, so it is in flight during tile ct's compute and stores; the first tile's
// d(x) and u loads are issued together (one round trip before the first barrier).
template <typename T, int K, int ORD, int NCT>
__global__ __launch_bounds__(256, sizeof(T) == 2 && NCT <= 2 && ORD == 2 && K <= 3 ? 4 : 1) void shortconv_bwd_kernel(Bwd a) {
  extern __shared__ float smem[];
  constexpr int G = ORD + 1;
  constexpr int RU = TP + 2 * (K - 1);  // u rows: [t0 - (K-1), t0 + TP + K - 1)
  constexpr int RD = TP + K - 1;        // duc rows: [t0, t0 + TP + K - 1)
  constexpr int LW = TC + PAD;
  // duc for a tile's positions plus the K-1 after it (0 at t >= L: cropped conv outputs). A lane
  // takes (channel jj of the wave's 8, chunk of 8 positions): its d(x_g) / d(v x) loads are 16-B
  // vectors of the channel-major rows (when L % 8 == 0: every row 16-B aligned); rows past the
  // duc tile (RD) or past L are dropped / zero.
  constexpr int NCH = (RD + 7) / 8;                 // position chunks per channel
  constexpr int NQ = (CPW * NCH + 63) / 64;         // items per lane
  constexpr int DW = sizeof(T) == 2 ? 1 : 2;        // 16-B words per 8 elements
  constexpr int NIT = TokTile<T, K - 1, K - 1>::NIT;
  const int C = G * a.d;
  const int t0 = blockIdx.x * TP, b = blockIdx.z;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  constexpr int LU = UTile<T>::LW;
  T* us = reinterpret_cast<T*>(smem);                                  // [G][RU][LU], T
  float* ds = reinterpret_cast<float*>(us + G * RU * LU);             // [G][RD][LW]
  // [4][G * TC][K + 1] row-quarter sums, over the u tile once the dw phase has read it (one more
  // barrier; with the bf16 u tile 40 KB per block: four blocks per CU)
  float* red = smem;
  static_assert(4 * G * TC * (K + 1) * 4 <= G * RU * LU * (int)sizeof(T), "red must fit in the u tile");
  static_assert((G * RU * LU * sizeof(T)) % 4 == 0, "ds must be 4-B aligned");
  const T* u = (const T*)a.u + (size_t)b * a.L * C;
  const bool vec = (a.L & 7) == 0;
  struct Regs {
    uint4 raw[G][NIT];      // u tile rows (token-major, 16-B vectors)
    uint4 dg[NQ][ORD][DW];  // [g < ORD-1]: d(x_g), [ORD-1]: d(v x); 8 positions per item
  };
  auto fetch = [&](Regs& r, int c0) __attribute__((always_inline)) {
#pragma unroll
    for (int n = 0; n < NQ; ++n) {
      const int q = lane + 64 * n;
      const int jj = q / NCH, pc = q - jj * NCH;
      const int c = c0 + wv * CPW + jj, t = t0 + 8 * pc;
      const bool okq = q < CPW * NCH;
#pragma unroll
      for (int g = 0; g < ORD; ++g) {
        const T* row = g < ORD - 1 ? (const T*)a.dxs + ((size_t)b * (ORD - 1) * a.d + g * a.d + c) * a.L
                                   : (const T*)a.dvx + ((size_t)b * a.d + c) * a.L;
#pragma unroll
        for (int h = 0; h < DW; ++h) r.dg[n][g][h] = make_uint4(0u, 0u, 0u, 0u);
        if (okq && vec && t + 8 <= a.L) {
#pragma unroll
          for (int h = 0; h < DW; ++h) r.dg[n][g][h] = *reinterpret_cast<const uint4*>(row + t + h * (8 / DW));
        } else if (okq) {
          T* e = reinterpret_cast<T*>(&r.dg[n][g][0]);
#pragma unroll
          for (int i = 0; i < 8; ++i)
            if (t + i < a.L) e[i] = row[t + i];
        }
      }
    }
    tok_fetch<T, K - 1, K - 1, G>(r.raw, u, a.L, C, t0, a.d, c0);
  };
  Regs cur;
  fetch(cur, blockIdx.y * NCT * TC);
#pragma unroll
  for (int ct = 0; ct < NCT; ++ct) {
  const int c0 = (blockIdx.y * NCT + ct) * TC;
  if (ct > 0) __syncthreads();  // the previous tile's LDS reads are done
  tok_store_raw<T, K - 1, K - 1, G>(us, cur.raw);
  __syncthreads();
  Regs nxt;
  if (ct + 1 < NCT) fetch(nxt, c0 + TC);
#pragma unroll
  for (int n = 0; n < NQ; ++n) {
    const int q = lane + 64 * n;
    if (q >= CPW * NCH) break;
    const int jj = q / NCH, pc = q - jj * NCH;
    const int j = wv * CPW + jj, c = c0 + j;
    // the two recomputed conv outputs (groups order-1, order) need u rows rr .. rr + K - 1
    const int chl = (ORD - 1) * a.d + c, chv = ORD * a.d + c;
    float wl[K], wvv[K];
#pragma unroll
    for (int k = 0; k < K; ++k) { wl[k] = a.w[chl * K + k]; wvv[k] = a.w[chv * K + k]; }
    const float bl = a.bias[chl], bv = a.bias[chv];
    const T* tl_l = us + (ORD - 1) * RU * LU;
    const T* tl_v = us + ORD * RU * LU;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int rr = 8 * pc + i;
      if (rr >= RD) break;
      const int t = t0 + rr;
      float conv_last = 0.f, conv_v = 0.f;
      if (t < a.L) {
        conv_last = bl;
        conv_v = bv;
#pragma unroll
        for (int k = 0; k < K; ++k) {
          conv_last = fmaf(wl[k], to_f32(tl_l[(rr + k) * LU + j]), conv_last);
          conv_v = fmaf(wvv[k], to_f32(tl_v[(rr + k) * LU + j]), conv_v);
        }
      }
      const float dvx = to_f32(reinterpret_cast<const T*>(&cur.dg[n][ORD - 1][0])[i]);
#pragma unroll
      for (int g = 0; g < G; ++g) {
        float v;
        if (g < ORD - 1) v = to_f32(reinterpret_cast<const T*>(&cur.dg[n][g < ORD - 1 ? g : 0][0])[i]);
        else v = g == ORD - 1 ? dvx * conv_v : dvx * conv_last;
        ds[(g * RD + rr) * LW + j] = v;
      }
    }
  }
  __syncthreads();
  // du (token-major): lane = (row in 16, 8-channel chunk in 4): one 16-B (bf16) / 2 x 16-B
  // (fp32) store per lane and row; 4 waves x 16 rows per pass
  T* du = (T*)a.du + (size_t)b * a.L * C;
  const int cc8 = 8 * (lane & 3), rsub = lane >> 2;
  for (int g = 0; g < G; ++g) {
    const int ch = g * a.d + c0 + cc8;
    float w8[8][K];
#pragma unroll
    for (int e = 0; e < 8; ++e)
#pragma unroll
      for (int k = 0; k < K; ++k) w8[e][k] = a.w[(ch + e) * K + k];
    const float* dl = ds + g * RD * LW;
    for (int r = wv * 16 + rsub; r < TP; r += 64) {
      const int t = t0 + r;
      if (t >= a.L) break;
      float acc[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[e] = 0.f;
#pragma unroll
      for (int k = 0; k < K; ++k) {
        const float* src = dl + (r + K - 1 - k) * LW + cc8;
#pragma unroll
        for (int e = 0; e < 8; ++e) acc[e] = fmaf(w8[e][k], src[e], acc[e]);
      }
      T* o = du + (size_t)t * C + ch;
      if constexpr (sizeof(T) == 2) {
        bf16x8 v;
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = (bf16)acc[e];
        *reinterpret_cast<bf16x8*>(o) = v;
      } else {
        *reinterpret_cast<float4*>(o) = make_float4(acc[0], acc[1], acc[2], acc[3]);
        *reinterpret_cast<float4*>(o + 4) = make_float4(acc[4], acc[5], acc[6], acc[7]);
      }
    }
  }
  // dw / dbias: (row quarter, group, channel) per thread, 16 rows each
  constexpr int items = 4 * G * TC;
  constexpr int NH = (items + 255) / 256;  // items per thread
  float sw[NH][K + 1];
#pragma unroll
  for (int h = 0; h < NH; ++h) {
    const int it = threadIdx.x + 256 * h;
#pragma unroll
    for (int k = 0; k <= K; ++k) sw[h][k] = 0.f;
    if (it >= items) continue;
    const int qr = it / (G * TC), gc = it - qr * (G * TC);
    const int g = gc / TC, j = gc - g * TC;
    const float* dl = ds + g * RD * LW;
    const T* ul = us + g * RU * LU;
#pragma unroll 4
    for (int r = 16 * qr; r < 16 * qr + 16; ++r) {
      const float dv = dl[r * LW + j];  // duc at t0 + r (0 past L)
#pragma unroll
      for (int k = 0; k < K; ++k) sw[h][k] = fmaf(dv, to_f32(ul[(r + k) * LU + j]), sw[h][k]);  // u[t - (K-1-k)]
      sw[h][K] += dv;
    }
  }
  __syncthreads();  // every read of the u tile is done: red overwrites it
#pragma unroll
  for (int h = 0; h < NH; ++h) {
    const int it = threadIdx.x + 256 * h;
    if (it < items) {
#pragma unroll
      for (int k = 0; k <= K; ++k) red[it * (K + 1) + k] = sw[h][k];
    }
  }
  __syncthreads();
  const int nL = gridDim.x;
  float* prow = a.part + ((size_t)b * nL + blockIdx.x) * C * (K + 1);
  for (int e = threadIdx.x; e < G * TC * (K + 1); e += blockDim.x) {
    const int gc = e / (K + 1), k = e - gc * (K + 1);
    const int g = gc / TC, j = gc - g * TC;
    const float v = ((red[e] + red[G * TC * (K + 1) + e]) + red[2 * G * TC * (K + 1) + e]) +
                    red[3 * G * TC * (K + 1) + e];
    prow[(size_t)(g * a.d + c0 + j) * (K + 1) + k] = v;
  }
  if (ct + 1 < NCT) cur = nxt;
  }
}

// Channel tiles per block for the short-conv backward: the 32-channel tiles of a 128-B
// token-major line run in one block, so the later tiles' u rows are L2 hits (PMC: the one-tile
// kernel fetched 2x its algorithmic bytes), software-pipelined (above). bf16: 2 tiles per block
// (the bf16 u tile + fp32 duc tile are 40 KB and 119 VGPRs: four blocks per CU); fp32: 4 tiles
// (three blocks per CU). Config D 0.347 -> 0.237 ms per call over the round-5 steps
// (profiles/r05/ab_shortconv_pipelined.txt). DNA_HYENA_NCT = 1 | 2 | 4 overrides (A/B); fewer
// when d / 32 does not divide.
inline int nct_for(int d, int dtype) {
  static const int env = getenv("DNA_HYENA_NCT") ? atoi(getenv("DNA_HYENA_NCT")) : 0;
  const int want = env > 0 ? env : (dtype == DNA_BF16 ? 2 : 4);
  for (int n = want >= 4 ? 4 : want >= 2 ? 2 : 1; n > 1; n /= 2)
    if ((d / TC) % n == 0) return n;
  return 1;
}

template <typename F>
int dispatch_k(int K, F&& f) {
  switch (K) {
    case 2: f(std::integral_constant<int, 2>()); return 0;
    case 3: f(std::integral_constant<int, 3>()); return 0;
    case 4: f(std::integral_constant<int, 4>()); return 0;
    default: return -1;
  }
}
// (K, order) -> f(K, ORD) for K in 2..4, order in 2..4 (hy_check validated both)
template <typename F>
int dispatch_k_ord(int K, int order, F&& f) {
  return dispatch_k(K, [&](auto kk) {
    switch (order) {
      case 2: f(kk, std::integral_constant<int, 2>()); break;
      case 3: f(kk, std::integral_constant<int, 3>()); break;
      default: f(kk, std::integral_constant<int, 4>()); break;
    }
  });
}

}  // namespace hyop
}  // namespace dna

using namespace dna;
using namespace dna::hyop;

static int hy_check(int B, int L, int d, int order, int K, int dtype, const char* fn) {
  DNA_CHECK_ARG(B > 0 && L > 0 && d > 0 && d % 64 == 0, "%s: d %% 64 == 0 required (d=%d)", fn, d);
  DNA_CHECK_ARG(order >= 2 && order <= 4, "%s: order %d unsupported (2..4)", fn, order);
  DNA_CHECK_ARG(K >= 2 && K <= 4, "%s: short filter order %d unsupported (2..4)", fn, K);
  DNA_CHECK_ARG(dtype == DNA_F32 || dtype == DNA_BF16, "%s: bad dtype", fn);
  return DNA_OK;
}

extern "C" int dna_hyena_shortconv_fwd(const void* u, int dtype, const float* w, const float* bias,
                                       int B, int L, int d, int order, int K, void* xs, void* vx,
                                       void* stream) {
  int st = hy_check(B, L, d, order, K, dtype, "dna_hyena_shortconv_fwd");
  if (st) return st;
  DNA_CHECK_ARG(u && w && bias && vx && (order == 2 || xs), "dna_hyena_shortconv_fwd: null pointer");
  DNA_CHECK_ARG(((uintptr_t)u & 15) == 0, "dna_hyena_shortconv_fwd: u must be 16-byte aligned");
  Fwd a{u, w, bias, B, L, d, order, K, xs, vx, 1};  // two tiles per block: 2 % slower here
  const dim3 grid((L + TP - 1) / TP, d / TC / a.nct, B);
  const size_t lds = (size_t)(order + 1) * (TP + K - 1) * (TC + PAD) * sizeof(float);
  hipStream_t s = as_stream(stream);
  dispatch_k_ord(K, order, [&](auto kk, auto oo) {
    constexpr int KK = decltype(kk)::value, OO = decltype(oo)::value;
    if (dtype == DNA_F32)
      hipLaunchKernelGGL((shortconv_fwd_kernel<float, KK, OO>), grid, dim3(256), lds, s, a);
    else
      hipLaunchKernelGGL((shortconv_fwd_kernel<bf16, KK, OO>), grid, dim3(256), lds, s, a);
  });
  DNA_LAUNCH_CHECK("dna_hyena_shortconv_fwd");
  return DNA_OK;
}

extern "C" size_t dna_hyena_shortconv_part_elems(int B, int L, int d, int order, int K) {
  return (size_t)B * ((L + TP - 1) / TP) * (order + 1) * d * (K + 1);
}

extern "C" int dna_hyena_shortconv_bwd(const void* u, int dtype, const float* w, const float* bias,
                                       int B, int L, int d, int order, int K, const void* dxs,
                                       const void* dvx, void* du, float* part, void* stream) {
  int st = hy_check(B, L, d, order, K, dtype, "dna_hyena_shortconv_bwd");
  if (st) return st;
  DNA_CHECK_ARG(u && w && bias && dvx && du && part && (order == 2 || dxs),
                "dna_hyena_shortconv_bwd: null pointer");
  DNA_CHECK_ARG(((uintptr_t)u & 15) == 0, "dna_hyena_shortconv_bwd: u must be 16-byte aligned");
  Bwd a{u, w, bias, B, L, d, order, K, dxs, dvx, du, part};
  const int nct = nct_for(d, dtype);
  const dim3 grid((L + TP - 1) / TP, d / TC / nct, B);
  const size_t es = dtype == DNA_BF16 ? 2 : 4;
  const size_t lu = dtype == DNA_BF16 ? TC + 2 : TC + PAD;
  const size_t lds = (size_t)(order + 1) * ((TP + 2 * (K - 1)) * lu * es + (TP + K - 1) * (TC + PAD) * sizeof(float));
  DNA_CHECK_ARG(lds <= 160 * 1024, "dna_hyena_shortconv_bwd: order %d needs %zu B of LDS", order, lds);
  hipStream_t s = as_stream(stream);
  dispatch_k_ord(K, order, [&](auto kk, auto oo) {
    constexpr int KK = decltype(kk)::value, OO = decltype(oo)::value;
    auto go = [&](auto k) {
      if (lds > 65536) (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
      hipLaunchKernelGGL(k, grid, dim3(256), lds, s, a);
    };
    if (dtype == DNA_F32)
      nct == 4 ? go(shortconv_bwd_kernel<float, KK, OO, 4>) : nct == 2 ? go(shortconv_bwd_kernel<float, KK, OO, 2>)
                                                            : go(shortconv_bwd_kernel<float, KK, OO, 1>);
    else
      nct == 4 ? go(shortconv_bwd_kernel<bf16, KK, OO, 4>) : nct == 2 ? go(shortconv_bwd_kernel<bf16, KK, OO, 2>)
                                                           : go(shortconv_bwd_kernel<bf16, KK, OO, 1>);
  });
  DNA_LAUNCH_CHECK("dna_hyena_shortconv_bwd");
  return DNA_OK;
}

// the 16-B paths of the gate kernels: every row start 16-B aligned (d % 32 == 0 already)
static int gate_vec(int L, size_t bstride, std::initializer_list<const void*> ptrs) {
  int ok = L % 8 == 0 && bstride % 8 == 0;
  for (const void* p : ptrs) ok = ok && ((uintptr_t)p & 15) == 0;
  return ok;
}

extern "C" int dna_hyena_gate_out_fwd(const void* yc, const void* x0, int dtype, int B, int L, int d,
                                      size_t x0_bstride, void* y, void* stream) {
  DNA_CHECK_ARG(yc && x0 && y && B > 0 && L > 0 && d % TC == 0, "dna_hyena_gate_out_fwd: bad args");
  const dim3 grid((L + TP - 1) / TP, d / TC, B);
  hipStream_t s = as_stream(stream);
  const int vec = gate_vec(L, x0_bstride, {yc, x0, y});
  if (dtype == DNA_F32)
    hipLaunchKernelGGL(gate_out_fwd_kernel<float>, grid, dim3(256), 0, s, (const float*)yc,
                       (const float*)x0, L, d, x0_bstride, vec, (float*)y);
  else if (dtype == DNA_BF16)
    hipLaunchKernelGGL(gate_out_fwd_kernel<bf16>, grid, dim3(256), 0, s, (const bf16*)yc,
                       (const bf16*)x0, L, d, x0_bstride, vec, (bf16*)y);
  else
    DNA_CHECK_ARG(false, "dna_hyena_gate_out_fwd: bad dtype");
  DNA_LAUNCH_CHECK("dna_hyena_gate_out_fwd");
  return DNA_OK;
}

extern "C" int dna_hyena_gate_out_bwd(const void* dy, const void* yc, const void* x0, int dtype,
                                      int B, int L, int d, size_t x_bstride, void* dyc, void* dx0,
                                      void* stream) {
  DNA_CHECK_ARG(dy && yc && x0 && dyc && dx0 && B > 0 && L > 0 && d % TC == 0,
                "dna_hyena_gate_out_bwd: bad args");
  const dim3 grid((L + TP - 1) / TP, d / TC, B);
  hipStream_t s = as_stream(stream);
  const int vec = gate_vec(L, x_bstride, {dy, yc, x0, dyc, dx0});
  if (dtype == DNA_F32)
    hipLaunchKernelGGL(gate_out_bwd_kernel<float>, grid, dim3(256), 0, s, (const float*)dy,
                       (const float*)yc, (const float*)x0, L, d, x_bstride, vec, (float*)dyc, (float*)dx0);
  else if (dtype == DNA_BF16)
    hipLaunchKernelGGL(gate_out_bwd_kernel<bf16>, grid, dim3(256), 0, s, (const bf16*)dy,
                       (const bf16*)yc, (const bf16*)x0, L, d, x_bstride, vec, (bf16*)dyc, (bf16*)dx0);
  else
    DNA_CHECK_ARG(false, "dna_hyena_gate_out_bwd: bad dtype");
  DNA_LAUNCH_CHECK("dna_hyena_gate_out_bwd");
  return DNA_OK;
}

extern "C" int dna_hyena_modulate_t_fwd(const void* h, int dtype, const float* tpos, const float* delta,
                                        float shift, int L, int C, int O, float* k, void* stream) {
  DNA_CHECK_ARG(h && tpos && delta && k && L > 0 && C > 0 && O > 0 && C % O == 0,
                "dna_hyena_modulate_t_fwd: bad args");
  const dim3 grid((L + MT - 1) / MT, (C + MT - 1) / MT);
  hipStream_t s = as_stream(stream);
  if (dtype == DNA_F32)
    hipLaunchKernelGGL(modulate_t_fwd_kernel<float>, grid, dim3(256), 0, s, (const float*)h, tpos, delta,
                       shift, L, C, O, k);
  else if (dtype == DNA_BF16)
    hipLaunchKernelGGL(modulate_t_fwd_kernel<bf16>, grid, dim3(256), 0, s, (const bf16*)h, tpos, delta,
                       shift, L, C, O, k);
  else
    DNA_CHECK_ARG(false, "dna_hyena_modulate_t_fwd: bad dtype");
  DNA_LAUNCH_CHECK("dna_hyena_modulate_t_fwd");
  return DNA_OK;
}

extern "C" int dna_hyena_modulate_t_bwd(const float* dk, const float* tpos, const float* delta, float shift,
                                        int L, int C, int O, void* dh, int dtype, void* stream) {
  DNA_CHECK_ARG(dk && tpos && delta && dh && L > 0 && C > 0 && O > 0 && C % O == 0,
                "dna_hyena_modulate_t_bwd: bad args");
  const dim3 grid((L + MT - 1) / MT, (C + MT - 1) / MT);
  hipStream_t s = as_stream(stream);
  if (dtype == DNA_F32)
    hipLaunchKernelGGL(modulate_t_bwd_kernel<float>, grid, dim3(256), 0, s, dk, tpos, delta, shift, L, C,
                       O, (float*)dh);
  else if (dtype == DNA_BF16)
    hipLaunchKernelGGL(modulate_t_bwd_kernel<bf16>, grid, dim3(256), 0, s, dk, tpos, delta, shift, L, C,
                       O, (bf16*)dh);
  else
    DNA_CHECK_ARG(false, "dna_hyena_modulate_t_bwd: bad dtype");
  DNA_LAUNCH_CHECK("dna_hyena_modulate_t_bwd");
  return DNA_OK;
}
