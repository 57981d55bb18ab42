// Fused (bias, GELU, dropout, residual) + LayerNorm and the embedding LayerNorm, fwd + bwd.
//
// One wave per row; cols % 256 == 0 rows (DNABERT-2-117M: 768) use the vector mapping where a
// lane owns 4 consecutive columns per 256-column slab (one Philox call per 4 dropout bits);
// other widths (64, 128 in the small test configs) use a strided mapping.
// HBM-bound: per row element fwd reads x (2-4 B) + residual (4 B), writes y (4 B) + y_bf16 (2 B).
// Backward recomputes the pre-LN value from x, bias and residual (no saved activation besides
// mean/rstd), then reduces dgamma/dbeta/dbias through per-block partials (deterministic).
#include <type_traits>

#include "common.h"

namespace dna {
namespace ln {

constexpr int WAVES = 4;  // rows per block in the forward
constexpr int BWD_BLOCKS = 512;

// column of value k of a lane
template <bool VEC>
__device__ __forceinline__ int col_of(int k, int lane) {
  return VEC ? ((k >> 2) << 8) + (lane << 2) + (k & 3) : (k << 6) + lane;
}

template <typename T, int NV, bool VEC>
__device__ __forceinline__ void load_row(const T* p, int lane, float (&v)[NV]) {
  if constexpr (VEC && sizeof(T) == 4) {
#pragma unroll
    for (int k = 0; k < NV; k += 4) {
      f32x4 t = *reinterpret_cast<const f32x4*>(p + col_of<VEC>(k, lane));
      v[k] = t[0]; v[k + 1] = t[1]; v[k + 2] = t[2]; v[k + 3] = t[3];
    }
  } else if constexpr (VEC) {
#pragma unroll
    for (int k = 0; k < NV; k += 4) {
      bf16x4 t = *reinterpret_cast<const bf16x4*>(p + col_of<VEC>(k, lane));
      v[k] = (float)t[0]; v[k + 1] = (float)t[1]; v[k + 2] = (float)t[2]; v[k + 3] = (float)t[3];
    }
  } else {
#pragma unroll
    for (int k = 0; k < NV; ++k) v[k] = to_f32(p[col_of<VEC>(k, lane)]);
  }
}

template <typename T, int NV, bool VEC>
__device__ __forceinline__ void store_row(T* p, int lane, const float (&v)[NV]) {
  if constexpr (VEC && sizeof(T) == 4) {
#pragma unroll
    for (int k = 0; k < NV; k += 4)
      *reinterpret_cast<f32x4*>(p + col_of<VEC>(k, lane)) = f32x4{v[k], v[k + 1], v[k + 2], v[k + 3]};
  } else if constexpr (VEC) {
#pragma unroll
    for (int k = 0; k < NV; k += 4)
      *reinterpret_cast<bf16x4*>(p + col_of<VEC>(k, lane)) =
          bf16x4{(bf16)v[k], (bf16)v[k + 1], (bf16)v[k + 2], (bf16)v[k + 3]};
  } else {
#pragma unroll
    for (int k = 0; k < NV; ++k) p[col_of<VEC>(k, lane)] = from_f32<T>(v[k]);
  }
}

// A row's NV values of a lane as loaded (bf16 kept packed until used), so loads issued for the
// next row are not waited for by a conversion right after them.
template <typename T, int NV, bool VEC>
struct RawRow {
  static constexpr bool PK = VEC && sizeof(T) == 2;
  typename std::conditional<PK, bf16x4, T>::type q[PK ? NV / 4 : NV];
  __device__ __forceinline__ void load(const T* p, int lane) {
    if constexpr (PK) {
#pragma unroll
      for (int k = 0; k < NV; k += 4) q[k / 4] = *reinterpret_cast<const bf16x4*>(p + col_of<VEC>(k, lane));
    } else if constexpr (VEC) {
#pragma unroll
      for (int k = 0; k < NV; k += 4) {
        f32x4 t = *reinterpret_cast<const f32x4*>(p + col_of<VEC>(k, lane));
        q[k] = t[0]; q[k + 1] = t[1]; q[k + 2] = t[2]; q[k + 3] = t[3];
      }
    } else {
#pragma unroll
      for (int k = 0; k < NV; ++k) q[k] = p[col_of<VEC>(k, lane)];
    }
  }
  __device__ __forceinline__ void get(float (&v)[NV]) const {
    if constexpr (PK) {
#pragma unroll
      for (int k = 0; k < NV; ++k) v[k] = (float)q[k / 4][k & 3];
    } else {
#pragma unroll
      for (int k = 0; k < NV; ++k) v[k] = to_f32(q[k]);
    }
  }
};

// dropout keep bits for the NV values of a lane in row `row`
template <int NV, bool VEC>
__device__ __forceinline__ void keep_bits(bool (&keep)[NV], int row, int cols, int lane,
                                          uint64_t seed, uint64_t off, uint32_t th) {
  const uint64_t rbase = (uint64_t)row * cols;
  if constexpr (VEC) {
#pragma unroll
    for (int k = 0; k < NV; k += 4) {
      uint32_t m = dropout_keep4(seed, off, (rbase + col_of<VEC>(k, lane)) >> 2, th);
#pragma unroll
      for (int e = 0; e < 4; ++e) keep[k + e] = (m >> e) & 1;
    }
  } else {
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      uint64_t e = rbase + col_of<VEC>(k, lane);
      keep[k] = (dropout_keep4(seed, off, e >> 2, th) >> (e & 3)) & 1;
    }
  }
}

struct FwdArgs {
  const void* x; const float* bias; int act; float p; uint32_t th; float kscale;
  uint64_t seed, off; const float* res; const float* gamma; const float* beta;
  int rows, cols; float eps; float* y; bf16* yb; float* mean; float* rstd;
  int rms;  // RMSNorm: no mean subtraction, no beta, mean[] not written
  float* sum;  // pre-norm residual stream (x + residual, fp32) of dna_add_ln_fwd, or null
};

template <typename TX, int NV, bool VEC>
__global__ __launch_bounds__(256) void fwd_kernel(FwdArgs a) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * WAVES + (threadIdx.x >> 6);
  if (row >= a.rows) return;
  const size_t ro = (size_t)row * a.cols;
  float v[NV];
  load_row<TX, NV, VEC>(reinterpret_cast<const TX*>(a.x) + ro, lane, v);
  if (a.bias) {
    float bb[NV];
    load_row<float, NV, VEC>(a.bias, lane, bb);
#pragma unroll
    for (int k = 0; k < NV; ++k) v[k] += bb[k];
  }
  if (a.act == DNA_ACT_GELU) {
#pragma unroll
    for (int k = 0; k < NV; ++k) v[k] = gelu_erf(v[k]);
  }
  if (a.p > 0.f) {
    bool keep[NV];
    keep_bits<NV, VEC>(keep, row, a.cols, lane, a.seed, a.off, a.th);
#pragma unroll
    for (int k = 0; k < NV; ++k) v[k] = keep[k] ? v[k] * a.kscale : 0.f;
  }
  if (a.res) {
    float r[NV];
    load_row<float, NV, VEC>(a.res + ro, lane, r);
#pragma unroll
    for (int k = 0; k < NV; ++k) v[k] += r[k];
  }
  if (a.sum) store_row<float, NV, VEC>(a.sum + ro, lane, v);
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < NV; ++k) s += v[k];
  const float mu = a.rms ? 0.f : wave_sum(s) / a.cols;
  float q = 0.f;
#pragma unroll
  for (int k = 0; k < NV; ++k) { float d = v[k] - mu; q += d * d; }
  const float rs = rsqrtf(wave_sum(q) / a.cols + a.eps);
  float g[NV], be[NV];
  load_row<float, NV, VEC>(a.gamma, lane, g);
  if (a.beta) load_row<float, NV, VEC>(a.beta, lane, be);
  else {
#pragma unroll
    for (int k = 0; k < NV; ++k) be[k] = 0.f;
  }
#pragma unroll
  for (int k = 0; k < NV; ++k) v[k] = (v[k] - mu) * rs * g[k] + be[k];
  if (a.y) store_row<float, NV, VEC>(a.y + ro, lane, v);
  if (a.yb) store_row<bf16, NV, VEC>(a.yb + ro, lane, v);
  if (lane == 0) {
    if (!a.rms) a.mean[row] = mu;
    a.rstd[row] = rs;
  }
}

struct BwdArgs {
  const float* dy; const bf16* dyb; const void* x; const float* bias; int act; float p;
  uint32_t th; float kscale; uint64_t seed, off; const float* res; const float* gamma;
  const float* mean; const float* rstd; int rows, cols; float* dres; void* dx;
  float* part;  // [gridDim.x][3][cols]: dgamma, dbeta, dbias
  int rms;      // RMSNorm backward: mean taken as 0, no mean-gradient term
  const float* dsum;  // dna_add_ln_bwd: gradient of the pre-norm sum output, added to the LN's
  const float* yin;   // dna_ln_bwd_from_y: the forward's fp32 output y; x_hat = (y - beta) / gamma
  const float* beta;  //   replaces the recomputation from x (+ bias, dropout) + residual
};

template <int NV, bool VEC>
__device__ __forceinline__ void block_partials(float (&acc0)[NV], float (&acc1)[NV],
                                               float (&acc2)[NV], int cols, float* part) {
  extern __shared__ __attribute__((aligned(16))) float red[];  // [WAVES][3][cols]
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    const int c = col_of<VEC>(k, lane);
    red[(w * 3 + 0) * cols + c] = acc0[k];
    red[(w * 3 + 1) * cols + c] = acc1[k];
    red[(w * 3 + 2) * cols + c] = acc2[k];
  }
  __syncthreads();
  for (int i = threadIdx.x; i < 3 * cols; i += blockDim.x) {
    float s = 0.f;
#pragma unroll
    for (int ww = 0; ww < WAVES; ++ww) s += red[ww * 3 * cols + i];
    part[(size_t)blockIdx.x * 3 * cols + i] = s;
  }
}

// The row loop is software-pipelined for short rows: the next row's inputs (x, residual, dy, the
// sum's gradient, mean / rstd) are loaded into raw registers before this row is computed, so each
// wave keeps two rows' loads in flight (the optional inputs under wave-uniform branches).
template <typename TX, int NV, bool VEC>
__global__ __launch_bounds__(256) void bwd_kernel(BwdArgs a) {
  const int lane = threadIdx.x & 63;
  const int gw = blockIdx.x * WAVES + (threadIdx.x >> 6), nw = gridDim.x * WAVES;
  float acc_g[NV], acc_b[NV], acc_x[NV], gam[NV], bias[NV];
#pragma unroll
  for (int k = 0; k < NV; ++k) { acc_g[k] = acc_b[k] = acc_x[k] = 0.f; bias[k] = 0.f; }
  load_row<float, NV, VEC>(a.gamma, lane, gam);
  if (a.bias) load_row<float, NV, VEC>(a.bias, lane, bias);
  const float inv_cols = 1.f / a.cols;
  float ginv[NV], bet[NV];
  if (a.yin) {
    load_row<float, NV, VEC>(a.beta, lane, bet);
#pragma unroll
    for (int k = 0; k < NV; ++k) ginv[k] = gam[k] != 0.f ? 1.f / gam[k] : 0.f;
  }
  struct In {
    RawRow<TX, NV, VEC> x;
    RawRow<float, NV, VEC> r, dy, ds;
    RawRow<bf16, NV, VEC> dyb;
    float mu, rs;
  };
  auto fetch = [&](In& f, int row) __attribute__((always_inline)) {
    const size_t ro = (size_t)row * a.cols;
    f.x.load(reinterpret_cast<const TX*>(a.x) + ro, lane);
    if (a.res) f.r.load(a.res + ro, lane);
    if (a.dy) f.dy.load(a.dy + ro, lane);
    if (a.dyb) f.dyb.load(a.dyb + ro, lane);
    if (a.dsum) f.ds.load(a.dsum + ro, lane);
    f.mu = a.rms ? 0.f : a.mean[row];
    f.rs = a.rstd[row];
  };
  // rows of up to 512 columns; at 768 (DNABERT-2) the second row set takes the kernel past 256
  // VGPRs and the plain loop below is faster (0.58 vs 0.61 ms, profiles/r05/ab_ln_bwd_prefetch.txt)
  constexpr bool PF = NV <= 8;
  if (!PF || a.yin) {  // (the from-y backward always takes the plain loop)
    for (int row = gw; row < a.rows; row += nw) {
      const size_t ro = (size_t)row * a.cols;
      float u[NV], v[NV];
      bool keep[NV];
      float mu;
      if (a.yin) {  // x_hat from the output: (y - beta) / gamma (act none; mean not needed)
        load_row<float, NV, VEC>(a.yin + ro, lane, v);
#pragma unroll
        for (int k = 0; k < NV; ++k) { v[k] = (v[k] - bet[k]) * ginv[k]; u[k] = 0.f; }
        if (a.p > 0.f) keep_bits<NV, VEC>(keep, row, a.cols, lane, a.seed, a.off, a.th);
        mu = 0.f;
      } else {
      load_row<TX, NV, VEC>(reinterpret_cast<const TX*>(a.x) + ro, lane, u);
#pragma unroll
      for (int k = 0; k < NV; ++k) { u[k] += bias[k]; v[k] = a.act == DNA_ACT_GELU ? gelu_erf(u[k]) : u[k]; }
      if (a.p > 0.f) {
        keep_bits<NV, VEC>(keep, row, a.cols, lane, a.seed, a.off, a.th);
#pragma unroll
        for (int k = 0; k < NV; ++k) v[k] = keep[k] ? v[k] * a.kscale : 0.f;
      }
      if (a.res) {
        float r[NV];
        load_row<float, NV, VEC>(a.res + ro, lane, r);
#pragma unroll
        for (int k = 0; k < NV; ++k) v[k] += r[k];
      }
      mu = a.rms ? 0.f : a.mean[row];
      }
      const float rs = a.rstd[row];
      float g[NV];
#pragma unroll
      for (int k = 0; k < NV; ++k) g[k] = 0.f;
      if (a.dy) load_row<float, NV, VEC>(a.dy + ro, lane, g);
      if (a.dyb) {
        float t[NV];
        load_row<bf16, NV, VEC>(a.dyb + ro, lane, t);
#pragma unroll
        for (int k = 0; k < NV; ++k) g[k] += t[k];
      }
      float s1 = 0.f, s2 = 0.f;
#pragma unroll
      for (int k = 0; k < NV; ++k) {
        const float xh = a.yin ? v[k] : (v[k] - mu) * rs;
        v[k] = xh;
        acc_g[k] += g[k] * xh;
        acc_b[k] += g[k];
        const float gy = g[k] * gam[k];
        g[k] = gy;
        s1 += gy;
        s2 += gy * xh;
      }
      const float c1 = a.rms ? 0.f : wave_sum(s1) * inv_cols, c2 = wave_sum(s2) * inv_cols;
#pragma unroll
      for (int k = 0; k < NV; ++k) g[k] = rs * (g[k] - c1 - v[k] * c2);  // d(pre-LN sum)
      if (a.dsum) {  // the sum's other consumers (the residual stream): total gradient of the sum
        float t[NV];
        load_row<float, NV, VEC>(a.dsum + ro, lane, t);
#pragma unroll
        for (int k = 0; k < NV; ++k) g[k] += t[k];
      }
      if (a.dres) store_row<float, NV, VEC>(a.dres + ro, lane, g);
#pragma unroll
      for (int k = 0; k < NV; ++k) {
        float d = g[k];
        if (a.p > 0.f) d = keep[k] ? d * a.kscale : 0.f;
        if (a.act == DNA_ACT_GELU) d *= gelu_erf_grad(u[k]);
        g[k] = d;
        acc_x[k] += d;
      }
      store_row<TX, NV, VEC>(reinterpret_cast<TX*>(a.dx) + ro, lane, g);
    }
  } else {
  In nx;
  if (gw < a.rows) fetch(nx, gw);
  for (int row = gw; row < a.rows; row += nw) {
    const size_t ro = (size_t)row * a.cols;
    const In cur = nx;
    // the next row (the last row again past the end: an L2 hit, no branch around the loads)
    fetch(nx, row + nw < a.rows ? row + nw : row);
    float u[NV], v[NV];
    cur.x.get(u);
#pragma unroll
    for (int k = 0; k < NV; ++k) { u[k] += bias[k]; v[k] = a.act == DNA_ACT_GELU ? gelu_erf(u[k]) : u[k]; }
    bool keep[NV];
    if (a.p > 0.f) {
      keep_bits<NV, VEC>(keep, row, a.cols, lane, a.seed, a.off, a.th);
#pragma unroll
      for (int k = 0; k < NV; ++k) v[k] = keep[k] ? v[k] * a.kscale : 0.f;
    }
    if (a.res) {
      float r[NV];
      cur.r.get(r);
#pragma unroll
      for (int k = 0; k < NV; ++k) v[k] += r[k];
    }
    const float mu = cur.mu, rs = cur.rs;
    float g[NV];
#pragma unroll
    for (int k = 0; k < NV; ++k) g[k] = 0.f;
    if (a.dy) cur.dy.get(g);
    if (a.dyb) {
      float t[NV];
      cur.dyb.get(t);
#pragma unroll
      for (int k = 0; k < NV; ++k) g[k] += t[k];
    }
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      const float xh = (v[k] - mu) * rs;
      v[k] = xh;
      acc_g[k] += g[k] * xh;
      acc_b[k] += g[k];
      const float gy = g[k] * gam[k];
      g[k] = gy;
      s1 += gy;
      s2 += gy * xh;
    }
    const float c1 = a.rms ? 0.f : wave_sum(s1) * inv_cols, c2 = wave_sum(s2) * inv_cols;
#pragma unroll
    for (int k = 0; k < NV; ++k) g[k] = rs * (g[k] - c1 - v[k] * c2);  // d(pre-LN sum)
    if (a.dsum) {  // the sum's other consumers (the residual stream): total gradient of the sum
      float t[NV];
      cur.ds.get(t);
#pragma unroll
      for (int k = 0; k < NV; ++k) g[k] += t[k];
    }
    if (a.dres) store_row<float, NV, VEC>(a.dres + ro, lane, g);
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      float d = g[k];
      if (a.p > 0.f) d = keep[k] ? d * a.kscale : 0.f;
      if (a.act == DNA_ACT_GELU) d *= gelu_erf_grad(u[k]);
      g[k] = d;
      acc_x[k] += d;
    }
    store_row<TX, NV, VEC>(reinterpret_cast<TX*>(a.dx) + ro, lane, g);
  }
  }
  block_partials<NV, VEC>(acc_g, acc_b, acc_x, a.cols, a.part);
}

// Embedding LN: v = word_emb[id] + type_row; y = dropout(LN(v)).
struct EmbFwdArgs {
  const int64_t* ids; const float* E; const float* tt; const float* gamma; const float* beta;
  int rows, cols, vocab; float eps, p; uint32_t th; float kscale; uint64_t seed, off;
  float* y; bf16* yb; float* mean; float* rstd;
};

template <int NV, bool VEC>
__global__ __launch_bounds__(256) void emb_fwd_kernel(EmbFwdArgs a) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * WAVES + (threadIdx.x >> 6);
  if (row >= a.rows) return;
  long id = (long)a.ids[row];
  id = id < 0 ? 0 : (id >= a.vocab ? a.vocab - 1 : id);
  float v[NV], t[NV];
  load_row<float, NV, VEC>(a.E + (size_t)id * a.cols, lane, v);
  load_row<float, NV, VEC>(a.tt, lane, t);
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < NV; ++k) { v[k] += t[k]; s += v[k]; }
  const float mu = wave_sum(s) / a.cols;
  float q = 0.f;
#pragma unroll
  for (int k = 0; k < NV; ++k) { float d = v[k] - mu; q += d * d; }
  const float rs = rsqrtf(wave_sum(q) / a.cols + a.eps);
  float g[NV], be[NV];
  load_row<float, NV, VEC>(a.gamma, lane, g);
  load_row<float, NV, VEC>(a.beta, lane, be);
#pragma unroll
  for (int k = 0; k < NV; ++k) v[k] = (v[k] - mu) * rs * g[k] + be[k];
  if (a.p > 0.f) {
    bool keep[NV];
    keep_bits<NV, VEC>(keep, row, a.cols, lane, a.seed, a.off, a.th);
#pragma unroll
    for (int k = 0; k < NV; ++k) v[k] = keep[k] ? v[k] * a.kscale : 0.f;
  }
  const size_t ro = (size_t)row * a.cols;
  if (a.y) store_row<float, NV, VEC>(a.y + ro, lane, v);
  if (a.yb) store_row<bf16, NV, VEC>(a.yb + ro, lane, v);
  if (lane == 0) { a.mean[row] = mu; a.rstd[row] = rs; }
}

struct EmbBwdArgs {
  const float* dy; const bf16* dyb; const int64_t* ids; const float* E; const float* tt;
  const float* gamma; const float* mean; const float* rstd; int rows, cols, vocab, pad_idx;
  float p; uint32_t th; float kscale; uint64_t seed, off; float* dE; float* part;
  float* drows;  // if set: d(embedding row) per token is written here instead of atomics into dE
};

template <int NV, bool VEC>
__global__ __launch_bounds__(256) void emb_bwd_kernel(EmbBwdArgs a) {
  const int lane = threadIdx.x & 63;
  const int gw = blockIdx.x * WAVES + (threadIdx.x >> 6), nw = gridDim.x * WAVES;
  float acc_g[NV], acc_b[NV], acc_t[NV], gam[NV], tt[NV];
#pragma unroll
  for (int k = 0; k < NV; ++k) acc_g[k] = acc_b[k] = acc_t[k] = 0.f;
  load_row<float, NV, VEC>(a.gamma, lane, gam);
  load_row<float, NV, VEC>(a.tt, lane, tt);
  const float inv_cols = 1.f / a.cols;
  for (int row = gw; row < a.rows; row += nw) {
    const size_t ro = (size_t)row * a.cols;
    long id = (long)a.ids[row];
    id = id < 0 ? 0 : (id >= a.vocab ? a.vocab - 1 : id);
    float v[NV], g[NV];
    load_row<float, NV, VEC>(a.E + (size_t)id * a.cols, lane, v);
#pragma unroll
    for (int k = 0; k < NV; ++k) { v[k] += tt[k]; g[k] = 0.f; }
    if (a.dy) load_row<float, NV, VEC>(a.dy + ro, lane, g);
    if (a.dyb) {
      float t[NV];
      load_row<bf16, NV, VEC>(a.dyb + ro, lane, t);
#pragma unroll
      for (int k = 0; k < NV; ++k) g[k] += t[k];
    }
    if (a.p > 0.f) {
      bool keep[NV];
      keep_bits<NV, VEC>(keep, row, a.cols, lane, a.seed, a.off, a.th);
#pragma unroll
      for (int k = 0; k < NV; ++k) g[k] = keep[k] ? g[k] * a.kscale : 0.f;
    }
    const float mu = a.mean[row], rs = a.rstd[row];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      const float xh = (v[k] - mu) * rs;
      v[k] = xh;
      acc_g[k] += g[k] * xh;
      acc_b[k] += g[k];
      const float gy = g[k] * gam[k];
      g[k] = gy;
      s1 += gy;
      s2 += gy * xh;
    }
    const float c1 = wave_sum(s1) * inv_cols, c2 = wave_sum(s2) * inv_cols;
    const bool to_table = id != a.pad_idx;
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      const float d = rs * (g[k] - c1 - v[k] * c2);
      acc_t[k] += d;
      g[k] = d;
    }
    if (a.drows) {
      store_row<float, NV, VEC>(a.drows + ro, lane, g);
    } else if (to_table) {
      float* drow = a.dE + (size_t)id * a.cols;
#pragma unroll
      for (int k = 0; k < NV; ++k) atomicAdd(drow + col_of<VEC>(k, lane), g[k]);
    }
  }
  block_partials<NV, VEC>(acc_g, acc_b, acc_t, a.cols, a.part);
}

// sum partials over blocks: out_q[c] = sum_b part[b][q][c]. Block = 64 columns x 16 row
// groups (coalesced 256-B rows), 8 independent loads in flight per thread, fixed summation
// order (deterministic).
constexpr int RP_GROUPS = 16;
__global__ __launch_bounds__(64 * RP_GROUPS) void reduce_partials(const float* __restrict__ part,
                                                                  int nblocks, int cols,
                                                                  float* o0, float* o1, float* o2,
                                                                  int acc = 0) {
  __shared__ float red[RP_GROUPS][64];
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  const int i = blockIdx.x * 64 + tx;
  const size_t ld = (size_t)3 * cols;
  float s = 0.f;
  if (i < 3 * cols) {
    float v[8];
    int b = ty;
    for (; b + 7 * RP_GROUPS < nblocks; b += 8 * RP_GROUPS) {
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = part[(size_t)(b + u * RP_GROUPS) * ld + i];
#pragma unroll
      for (int u = 0; u < 8; ++u) s += v[u];
    }
    for (; b < nblocks; b += RP_GROUPS) s += part[(size_t)b * ld + i];
  }
  red[ty][tx] = s;
  __syncthreads();
  if (ty == 0 && i < 3 * cols) {
#pragma unroll
    for (int g = 1; g < RP_GROUPS; ++g) s += red[g][tx];
    const int q = i / cols, c = i % cols;
    float* o = q == 0 ? o0 : (q == 1 ? o1 : o2);
    // acc: o += s (the parameter's fp32 gradient, as AccumulateGrad's add would do it)
    if (o) o[c] = acc ? o[c] + s : s;
  }
}

template <typename F>
int dispatch_cols(int cols, F&& f) {
  if (cols % 256 == 0) {
    switch (cols / 64) {
      case 4: f(std::integral_constant<int, 4>(), std::true_type()); return DNA_OK;
      case 8: f(std::integral_constant<int, 8>(), std::true_type()); return DNA_OK;
      case 12: f(std::integral_constant<int, 12>(), std::true_type()); return DNA_OK;
      case 16: f(std::integral_constant<int, 16>(), std::true_type()); return DNA_OK;
      default: break;
    }
  } else if (cols % 64 == 0) {
    switch (cols / 64) {
      case 1: f(std::integral_constant<int, 1>(), std::false_type()); return DNA_OK;
      case 2: f(std::integral_constant<int, 2>(), std::false_type()); return DNA_OK;
      case 3: f(std::integral_constant<int, 3>(), std::false_type()); return DNA_OK;
      default: break;
    }
  }
  set_error("layernorm: cols=%d unsupported (64, 128, 192 or a multiple of 256 up to 1024)", cols);
  return DNA_ERR_UNSUPPORTED;
}

inline int bwd_blocks(int rows, int cols) {
  // DNA_LN_BWD_BLOCKS: A/B switch for the grid cap (more blocks = more rows in flight, more
  // [3][cols] partials for reduce_partials). Rows below 768 columns get twice the blocks: a
  // wave's row is then too short to keep enough bytes in flight (d = 256, config D: 0.200 ->
  // 0.126 ms per call at 1024 blocks; 768 columns: 512 stays best, profiles/r05)
  static const int cap = getenv("DNA_LN_BWD_BLOCKS") ? atoi(getenv("DNA_LN_BWD_BLOCKS")) : 0;
  const int lim = cap >= 64 ? cap : (cols < 768 ? 2 * BWD_BLOCKS : BWD_BLOCKS);
  int nb = (rows + WAVES - 1) / WAVES;
  return nb < lim ? nb : lim;
}

}  // namespace ln
}  // namespace dna

using namespace dna;
using namespace dna::ln;

extern "C" size_t dna_ln_bwd_workspace(int rows, int cols) {
  return (size_t)bwd_blocks(rows, cols) * 3 * cols * sizeof(float);
}

extern "C" int dna_ln_fwd(const void* x, int x_dtype, const float* bias, int act, float p_drop,
                          uint64_t seed, uint64_t offset, const float* residual,
                          const float* gamma, const float* beta, int rows, int cols, float eps,
                          float* y, void* y_bf16, float* mean, float* rstd, void* stream) {
  DNA_CHECK_ARG(x && gamma && beta && mean && rstd, "dna_ln_fwd: null pointer");
  DNA_CHECK_ARG(y || y_bf16, "dna_ln_fwd: no output");
  DNA_CHECK_ARG(rows >= 0 && p_drop >= 0.f && p_drop < 1.f, "dna_ln_fwd: bad rows/p");
  DNA_CHECK_ARG(x_dtype == DNA_F32 || x_dtype == DNA_BF16, "dna_ln_fwd: bad dtype");
  if (rows == 0) return DNA_OK;
  FwdArgs a{x, bias, act, p_drop, dropout_threshold(p_drop), 1.f / (1.f - p_drop), seed, offset,
            residual, gamma, beta, rows, cols, eps, y, (bf16*)y_bf16, mean, rstd, 0, nullptr};
  hipStream_t s = as_stream(stream);
  dim3 grid((rows + WAVES - 1) / WAVES);
  int st = dispatch_cols(cols, [&](auto nv, auto vec) {
    constexpr int NV = decltype(nv)::value;
    constexpr bool VEC = decltype(vec)::value;
    if (x_dtype == DNA_BF16)
      hipLaunchKernelGGL((fwd_kernel<bf16, NV, VEC>), grid, dim3(256), 0, s, a);
    else
      hipLaunchKernelGGL((fwd_kernel<float, NV, VEC>), grid, dim3(256), 0, s, a);
  });
  if (st) return st;
  DNA_LAUNCH_CHECK("dna_ln_fwd");
  return DNA_OK;
}

extern "C" int dna_ln_bwd(const float* dy, const void* dy_bf16, const void* x, int x_dtype,
                          const float* bias, int act, float p_drop, uint64_t seed, uint64_t offset,
                          const float* residual, const float* gamma, const float* mean,
                          const float* rstd, int rows, int cols, float* dresidual, void* dx,
                          float* dgamma, float* dbeta, float* dbias, void* workspace,
                          size_t workspace_bytes, void* stream) {
  DNA_CHECK_ARG(x && gamma && mean && rstd && dx, "dna_ln_bwd: null pointer");
  DNA_CHECK_ARG(x_dtype == DNA_F32 || x_dtype == DNA_BF16, "dna_ln_bwd: bad dtype");
  if (rows == 0) return DNA_OK;
  DNA_CHECK_ARG(workspace && workspace_bytes >= dna_ln_bwd_workspace(rows, cols),
                "dna_ln_bwd: workspace too small (%zu < %zu)", workspace_bytes,
                dna_ln_bwd_workspace(rows, cols));
  const int nb = bwd_blocks(rows, cols);
  BwdArgs a{dy, (const bf16*)dy_bf16, x, bias, act, p_drop, dropout_threshold(p_drop),
            1.f / (1.f - p_drop), seed, offset, residual, gamma, mean, rstd, rows, cols,
            dresidual, dx, (float*)workspace, 0, nullptr};
  hipStream_t s = as_stream(stream);
  const size_t lds = (size_t)WAVES * 3 * cols * sizeof(float);
  int st = dispatch_cols(cols, [&](auto nv, auto vec) {
    constexpr int NV = decltype(nv)::value;
    constexpr bool VEC = decltype(vec)::value;
    if (x_dtype == DNA_BF16)
      hipLaunchKernelGGL((bwd_kernel<bf16, NV, VEC>), dim3(nb), dim3(256), lds, s, a);
    else
      hipLaunchKernelGGL((bwd_kernel<float, NV, VEC>), dim3(nb), dim3(256), lds, s, a);
  });
  if (st) return st;
  hipLaunchKernelGGL(reduce_partials, dim3((3 * cols + 63) / 64), dim3(64 * RP_GROUPS), 0, s,
                     (const float*)workspace, nb, cols, dgamma, dbeta, dbias, 0);
  DNA_LAUNCH_CHECK("dna_ln_bwd");
  return DNA_OK;
}

// The same backward with x_hat recomputed from the forward's fp32 output, x_hat = (y - beta) /
// gamma (act none only): it reads y instead of x and the residual -- one fp32 row instead of a
// bf16 and an fp32 row (3.2 instead of 3.6 GB per DNABERT-2 call at T = 262,144) -- and neither
// x nor the residual has to be kept for the backward. gamma must have no zero entries (those
// columns' x_hat cannot be recovered; they are taken as 0).
static int ln_bwd_from_y(const float* dy, const void* dy_bf16, const float* y, int x_dtype,
                         float p_drop, uint64_t seed, uint64_t offset, const float* gamma,
                         const float* beta, const float* rstd, int rows, int cols,
                         float* dresidual, void* dx, float* dgamma, float* dbeta, float* dbias,
                         void* workspace, size_t workspace_bytes, void* stream, int acc) {
  DNA_CHECK_ARG(y && gamma && beta && rstd && dx, "dna_ln_bwd_from_y: null pointer");
  DNA_CHECK_ARG(x_dtype == DNA_F32 || x_dtype == DNA_BF16, "dna_ln_bwd_from_y: bad dtype");
  if (rows == 0) return DNA_OK;
  DNA_CHECK_ARG(workspace && workspace_bytes >= dna_ln_bwd_workspace(rows, cols),
                "dna_ln_bwd_from_y: workspace too small (%zu < %zu)", workspace_bytes,
                dna_ln_bwd_workspace(rows, cols));
  const int nb = bwd_blocks(rows, cols);
  BwdArgs a{dy, (const bf16*)dy_bf16, nullptr, nullptr, DNA_ACT_NONE, p_drop,
            dropout_threshold(p_drop), 1.f / (1.f - p_drop), seed, offset, nullptr, gamma, nullptr,
            rstd, rows, cols, dresidual, dx, (float*)workspace, 0, nullptr, y, beta};
  hipStream_t s = as_stream(stream);
  const size_t lds = (size_t)WAVES * 3 * cols * sizeof(float);
  int st = dispatch_cols(cols, [&](auto nv, auto vec) {
    constexpr int NV = decltype(nv)::value;
    constexpr bool VEC = decltype(vec)::value;
    if (x_dtype == DNA_BF16)
      hipLaunchKernelGGL((bwd_kernel<bf16, NV, VEC>), dim3(nb), dim3(256), lds, s, a);
    else
      hipLaunchKernelGGL((bwd_kernel<float, NV, VEC>), dim3(nb), dim3(256), lds, s, a);
  });
  if (st) return st;
  hipLaunchKernelGGL(reduce_partials, dim3((3 * cols + 63) / 64), dim3(64 * RP_GROUPS), 0, s,
                     (const float*)workspace, nb, cols, dgamma, dbeta, dbias, acc);
  DNA_LAUNCH_CHECK("dna_ln_bwd_from_y");
  return DNA_OK;
}

extern "C" int dna_ln_bwd_from_y(const float* dy, const void* dy_bf16, const float* y, int x_dtype,
                                 float p_drop, uint64_t seed, uint64_t offset, const float* gamma,
                                 const float* beta, const float* rstd, int rows, int cols,
                                 float* dresidual, void* dx, float* dgamma, float* dbeta,
                                 float* dbias, void* workspace, size_t workspace_bytes,
                                 void* stream) {
  return ln_bwd_from_y(dy, dy_bf16, y, x_dtype, p_drop, seed, offset, gamma, beta, rstd, rows,
                       cols, dresidual, dx, dgamma, dbeta, dbias, workspace, workspace_bytes,
                       stream, 0);
}

// The same, adding dgamma / dbeta / dbias into the given (parameter-gradient) buffers instead
// of overwriting them: the fp32 flat gradient of a FlatParams-owned LayerNorm (dna_amd.flat),
// with no separate accumulate launch per parameter.
extern "C" int dna_ln_bwd_from_y_acc(const float* dy, const void* dy_bf16, const float* y,
                                     int x_dtype, float p_drop, uint64_t seed, uint64_t offset,
                                     const float* gamma, const float* beta, const float* rstd,
                                     int rows, int cols, float* dresidual, void* dx, float* dgamma,
                                     float* dbeta, float* dbias, void* workspace,
                                     size_t workspace_bytes, void* stream) {
  return ln_bwd_from_y(dy, dy_bf16, y, x_dtype, p_drop, seed, offset, gamma, beta, rstd, rows,
                       cols, dresidual, dx, dgamma, dbeta, dbias, workspace, workspace_bytes,
                       stream, 1);
}

// Pre-norm residual add + LayerNorm / RMSNorm (rms = 1: mamba_ssm's Block with fused_add_norm,
// modeling_caduceus.py; HyenaDNA / flash_attn Block with residual_in_fp32:
// residual = dropout(x) + residual; y = LN(residual), reference long_conv_lm.py:231-267 through
// flash_attn.modules.block.Block.forward): sum = x + residual (fp32, written), y = LN(sum) (fp32
// and / or bf16). The backward takes the gradient of `sum` from its other consumers (dsum: the
// next Block's residual add) and adds it to the LN's input gradient in the same pass: dres =
// total (fp32), dx = total in x's dtype -- the add node, its gradient accumulation and the cast
// of the mixer-output gradient are gone.
extern "C" int dna_add_ln_fwd(const void* x, int x_dtype, const float* residual, const float* gamma,
                              const float* beta, int rows, int cols, float eps, int rms, float* sum,
                              float* y, void* y_bf16, float* mean, float* rstd, void* stream) {
  DNA_CHECK_ARG(x && residual && gamma && sum && rstd && (rms || (beta && mean)),
                "dna_add_ln_fwd: null pointer");
  DNA_CHECK_ARG(y || y_bf16, "dna_add_ln_fwd: no output");
  DNA_CHECK_ARG(rows >= 0, "dna_add_ln_fwd: bad rows");
  DNA_CHECK_ARG(x_dtype == DNA_F32 || x_dtype == DNA_BF16, "dna_add_ln_fwd: bad dtype");
  if (rows == 0) return DNA_OK;
  FwdArgs a{x, nullptr, 0, 0.f, 0u, 1.f, 0, 0, residual, gamma, rms ? nullptr : beta, rows, cols,
            eps, y, (bf16*)y_bf16, rms ? nullptr : mean, rstd, rms ? 1 : 0, sum};
  hipStream_t s = as_stream(stream);
  dim3 grid((rows + WAVES - 1) / WAVES);
  int st = dispatch_cols(cols, [&](auto nv, auto vec) {
    constexpr int NV = decltype(nv)::value;
    constexpr bool VEC = decltype(vec)::value;
    if (x_dtype == DNA_BF16)
      hipLaunchKernelGGL((fwd_kernel<bf16, NV, VEC>), grid, dim3(256), 0, s, a);
    else
      hipLaunchKernelGGL((fwd_kernel<float, NV, VEC>), grid, dim3(256), 0, s, a);
  });
  if (st) return st;
  DNA_LAUNCH_CHECK("dna_add_ln_fwd");
  return DNA_OK;
}

extern "C" int dna_add_ln_bwd(const float* dy, const void* dy_bf16, const float* dsum, const void* x,
                              int x_dtype, const float* residual, const float* gamma,
                              const float* mean, const float* rstd, int rows, int cols, int rms,
                              float* dresidual, void* dx, float* dgamma, float* dbeta,
                              void* workspace, size_t workspace_bytes, void* stream) {
  DNA_CHECK_ARG(x && residual && gamma && rstd && dx && dresidual && (rms || mean),
                "dna_add_ln_bwd: null pointer");
  DNA_CHECK_ARG(x_dtype == DNA_F32 || x_dtype == DNA_BF16, "dna_add_ln_bwd: bad dtype");
  if (rows == 0) return DNA_OK;
  DNA_CHECK_ARG(workspace && workspace_bytes >= dna_ln_bwd_workspace(rows, cols),
                "dna_add_ln_bwd: workspace too small (%zu < %zu)", workspace_bytes,
                dna_ln_bwd_workspace(rows, cols));
  const int nb = bwd_blocks(rows, cols);
  BwdArgs a{dy, (const bf16*)dy_bf16, x, nullptr, 0, 0.f, 0u, 1.f, 0, 0, residual, gamma,
            rms ? nullptr : mean, rstd, rows, cols, dresidual, dx, (float*)workspace, rms ? 1 : 0, dsum};
  hipStream_t s = as_stream(stream);
  const size_t lds = (size_t)WAVES * 3 * cols * sizeof(float);
  int st = dispatch_cols(cols, [&](auto nv, auto vec) {
    constexpr int NV = decltype(nv)::value;
    constexpr bool VEC = decltype(vec)::value;
    if (x_dtype == DNA_BF16)
      hipLaunchKernelGGL((bwd_kernel<bf16, NV, VEC>), dim3(nb), dim3(256), lds, s, a);
    else
      hipLaunchKernelGGL((bwd_kernel<float, NV, VEC>), dim3(nb), dim3(256), lds, s, a);
  });
  if (st) return st;
  hipLaunchKernelGGL(reduce_partials, dim3((3 * cols + 63) / 64), dim3(64 * RP_GROUPS), 0, s,
                     (const float*)workspace, nb, cols, dgamma, rms ? (float*)nullptr : dbeta, (float*)nullptr, 0);
  DNA_LAUNCH_CHECK("dna_add_ln_bwd");
  return DNA_OK;
}

extern "C" int dna_embed_ln_fwd(const int64_t* ids, const float* word_emb, const float* type_row,
                                const float* gamma, const float* beta, int rows, int cols,
                                int vocab, float eps, float p_drop, uint64_t seed,
                                uint64_t offset, float* y, void* y_bf16, float* mean, float* rstd,
                                void* stream) {
  DNA_CHECK_ARG(ids && word_emb && type_row && gamma && beta && mean && rstd,
                "dna_embed_ln_fwd: null pointer");
  DNA_CHECK_ARG(y || y_bf16, "dna_embed_ln_fwd: no output");
  if (rows == 0) return DNA_OK;
  EmbFwdArgs a{ids, word_emb, type_row, gamma, beta, rows, cols, vocab, eps, p_drop,
               dropout_threshold(p_drop), 1.f / (1.f - p_drop), seed, offset, y,
               (bf16*)y_bf16, mean, rstd};
  hipStream_t s = as_stream(stream);
  int st = dispatch_cols(cols, [&](auto nv, auto vec) {
    constexpr int NV = decltype(nv)::value;
    constexpr bool VEC = decltype(vec)::value;
    hipLaunchKernelGGL((emb_fwd_kernel<NV, VEC>), dim3((rows + WAVES - 1) / WAVES), dim3(256), 0,
                       s, a);
  });
  if (st) return st;
  DNA_LAUNCH_CHECK("dna_embed_ln_fwd");
  return DNA_OK;
}

static int embed_ln_bwd_impl(const float* dy, const void* dy_bf16, const int64_t* ids,
                             const float* word_emb, const float* type_row, const float* gamma,
                             const float* mean, const float* rstd, int rows, int cols, int vocab,
                             int padding_idx, float p_drop, uint64_t seed, uint64_t offset,
                             float* dword_emb, float* drows, float* dtype_row, float* dgamma,
                             float* dbeta, void* workspace, size_t workspace_bytes,
                             void* stream) {
  DNA_CHECK_ARG(ids && word_emb && type_row && gamma && mean && rstd && (dword_emb || drows),
                "dna_embed_ln_bwd: null pointer");
  if (rows == 0) return DNA_OK;
  DNA_CHECK_ARG(workspace && workspace_bytes >= dna_ln_bwd_workspace(rows, cols),
                "dna_embed_ln_bwd: workspace too small");
  const int nb = bwd_blocks(rows, cols);
  EmbBwdArgs a{dy, (const bf16*)dy_bf16, ids, word_emb, type_row, gamma, mean, rstd, rows, cols,
               vocab, padding_idx, p_drop, dropout_threshold(p_drop), 1.f / (1.f - p_drop), seed,
               offset, dword_emb, (float*)workspace, drows};
  hipStream_t s = as_stream(stream);
  const size_t lds = (size_t)WAVES * 3 * cols * sizeof(float);
  int st = dispatch_cols(cols, [&](auto nv, auto vec) {
    constexpr int NV = decltype(nv)::value;
    constexpr bool VEC = decltype(vec)::value;
    hipLaunchKernelGGL((emb_bwd_kernel<NV, VEC>), dim3(nb), dim3(256), lds, s, a);
  });
  if (st) return st;
  // partial slots: 0 dgamma, 1 dbeta, 2 d(type_row)
  hipLaunchKernelGGL(reduce_partials, dim3((3 * cols + 63) / 64), dim3(64 * RP_GROUPS), 0, s,
                     (const float*)workspace, nb, cols, dgamma, dbeta, dtype_row, 0);
  DNA_LAUNCH_CHECK("dna_embed_ln_bwd");
  return DNA_OK;
}

extern "C" int dna_embed_ln_bwd(const float* dy, const void* dy_bf16, const int64_t* ids,
                                const float* word_emb, const float* type_row, const float* gamma,
                                const float* mean, const float* rstd, int rows, int cols,
                                int vocab, int padding_idx, float p_drop, uint64_t seed,
                                uint64_t offset, float* dword_emb, float* dtype_row,
                                float* dgamma, float* dbeta, void* workspace,
                                size_t workspace_bytes, void* stream) {
  return embed_ln_bwd_impl(dy, dy_bf16, ids, word_emb, type_row, gamma, mean, rstd, rows, cols,
                           vocab, padding_idx, p_drop, seed, offset, dword_emb, nullptr,
                           dtype_row, dgamma, dbeta, workspace, workspace_bytes, stream);
}

extern "C" int dna_embed_ln_bwd_rows(const float* dy, const void* dy_bf16, const int64_t* ids,
                                     const float* word_emb, const float* type_row,
                                     const float* gamma, const float* mean, const float* rstd,
                                     int rows, int cols, int vocab, float p_drop, uint64_t seed,
                                     uint64_t offset, float* drows, float* dtype_row,
                                     float* dgamma, float* dbeta, void* workspace,
                                     size_t workspace_bytes, void* stream) {
  return embed_ln_bwd_impl(dy, dy_bf16, ids, word_emb, type_row, gamma, mean, rstd, rows, cols,
                           vocab, -1, p_drop, seed, offset, nullptr, drows, dtype_row, dgamma,
                           dbeta, workspace, workspace_bytes, stream);
}

// ------------------------------------------------------------------------------------ RMSNorm
// y = x * rsqrt(mean(x^2) + eps) * gamma (mamba_ssm's RMSNorm as Caduceus' Blocks and norm_f use
// it; fp32 statistics): the LayerNorm kernels above with the mean fixed at 0 and no beta.
extern "C" int dna_rms_fwd(const void* x, int x_dtype, const float* gamma, int rows, int cols,
                           float eps, float* y, void* y_bf16, float* rstd, void* stream) {
  DNA_CHECK_ARG(x && gamma && rstd, "dna_rms_fwd: null pointer");
  DNA_CHECK_ARG(y || y_bf16, "dna_rms_fwd: no output");
  DNA_CHECK_ARG(rows >= 0, "dna_rms_fwd: bad rows");
  DNA_CHECK_ARG(x_dtype == DNA_F32 || x_dtype == DNA_BF16, "dna_rms_fwd: bad dtype");
  if (rows == 0) return DNA_OK;
  FwdArgs a{x, nullptr, DNA_ACT_NONE, 0.f, 0u, 1.f, 0, 0, nullptr, gamma, nullptr, rows, cols, eps,
            y, (bf16*)y_bf16, nullptr, rstd, 1};
  hipStream_t s = as_stream(stream);
  dim3 grid((rows + WAVES - 1) / WAVES);
  int st = dispatch_cols(cols, [&](auto nv, auto vec) {
    constexpr int NV = decltype(nv)::value;
    constexpr bool VEC = decltype(vec)::value;
    if (x_dtype == DNA_BF16)
      hipLaunchKernelGGL((fwd_kernel<bf16, NV, VEC>), grid, dim3(256), 0, s, a);
    else
      hipLaunchKernelGGL((fwd_kernel<float, NV, VEC>), grid, dim3(256), 0, s, a);
  });
  if (st) return st;
  DNA_LAUNCH_CHECK("dna_rms_fwd");
  return DNA_OK;
}

extern "C" int dna_rms_bwd(const float* dy, const void* dy_bf16, const void* x, int x_dtype,
                           const float* gamma, const float* rstd, int rows, int cols, void* dx,
                           float* dgamma, void* workspace, size_t workspace_bytes, void* stream) {
  DNA_CHECK_ARG(x && gamma && rstd && dx, "dna_rms_bwd: null pointer");
  DNA_CHECK_ARG(x_dtype == DNA_F32 || x_dtype == DNA_BF16, "dna_rms_bwd: bad dtype");
  if (rows == 0) return DNA_OK;
  DNA_CHECK_ARG(workspace && workspace_bytes >= dna_ln_bwd_workspace(rows, cols),
                "dna_rms_bwd: workspace too small (%zu < %zu)", workspace_bytes,
                dna_ln_bwd_workspace(rows, cols));
  const int nb = bwd_blocks(rows, cols);
  BwdArgs a{dy, (const bf16*)dy_bf16, x, nullptr, DNA_ACT_NONE, 0.f, 0u, 1.f, 0, 0, nullptr, gamma,
            nullptr, rstd, rows, cols, nullptr, dx, (float*)workspace, 1};
  hipStream_t s = as_stream(stream);
  const size_t lds = (size_t)WAVES * 3 * cols * sizeof(float);
  int st = dispatch_cols(cols, [&](auto nv, auto vec) {
    constexpr int NV = decltype(nv)::value;
    constexpr bool VEC = decltype(vec)::value;
    if (x_dtype == DNA_BF16)
      hipLaunchKernelGGL((bwd_kernel<bf16, NV, VEC>), dim3(nb), dim3(256), lds, s, a);
    else
      hipLaunchKernelGGL((bwd_kernel<float, NV, VEC>), dim3(nb), dim3(256), lds, s, a);
  });
  if (st) return st;
  hipLaunchKernelGGL(reduce_partials, dim3((3 * cols + 63) / 64), dim3(64 * RP_GROUPS), 0, s,
                     (const float*)workspace, nb, cols, dgamma, (float*)nullptr, (float*)nullptr, 0);
  DNA_LAUNCH_CHECK("dna_rms_bwd");
  return DNA_OK;
}
