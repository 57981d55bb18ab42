// Depthwise causal 1-D convolution (+ SiLU) over channel-major rows, fwd + bwd, gfx950.
//
// The Mamba block of Caduceus (reference src/models/caduceus/modeling_caduceus.py:68-121 ->
// mamba_ssm Mamba.forward, not vendored) runs x = silu(conv1d(x)[..., :L]) with a depthwise
// nn.Conv1d(d_inner, d_inner, kernel_size=d_conv, groups=d_inner, padding=d_conv-1) on
// x [B, d_inner, L] (the first half of the channel-major in_proj output):
//   out[b, c, t] = act(bias[c] + sum_{k<K} w[c][k] * x[b, c, t + k - (K-1)])      (x = 0 for t < 0)
// Backward (act = SiLU recomputed from x): g = dout * silu'(pre),
//   dx[t] = sum_k w[k] g[t + K-1-k]  (g = 0 past L),  dw[k] = sum_t g[t] x[t + k - (K-1)],
//   dbias = sum_t g[t]  -- dw/dbias as one partial row per block, summed by dna_colsum_f32.
// Element path: a block = 256 threads x 4 positions = 1024 positions of one (b, c) row, the K-1
// halo from LDS. 16-B path (L % 8 == 0, aligned rows; the Caduceus shapes): 8 positions per lane,
// halos by lane shuffles (below). HBM-bound (reads x, writes out; bwd reads x, dout, writes dx).
#include "common.h"

namespace dna {
namespace cconv {

constexpr int PER = 4;                  // positions per thread
constexpr int SEG = 256 * PER;          // positions per block
constexpr int MAXK = 8;

__device__ __forceinline__ float sigm(float x) {
  return __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(-x * 1.4426950408889634f));
}

template <typename T, int K>
__global__ __launch_bounds__(256) void fwd_kernel(const T* __restrict__ x, size_t x_bstride,
                                                  const float* __restrict__ w,
                                                  const float* __restrict__ bias, int C, int L,
                                                  int silu, T* __restrict__ out) {
  __shared__ float xs[SEG + MAXK];
  const int seg = blockIdx.x, c = blockIdx.y, b = blockIdx.z;
  const int t0 = seg * SEG;
  const T* row = x + (size_t)b * x_bstride + (size_t)c * L;
  for (int i = threadIdx.x; i < SEG + K - 1; i += 256) {
    const int t = t0 - (K - 1) + i;
    xs[i] = (t >= 0 && t < L) ? to_f32(row[t]) : 0.f;
  }
  __syncthreads();
  float wk[K];
#pragma unroll
  for (int k = 0; k < K; ++k) wk[k] = w[c * K + k];
  const float bc = bias ? bias[c] : 0.f;
  T* orow = out + ((size_t)b * C + c) * L;
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    const int i = j * 256 + threadIdx.x;  // coalesced
    const int t = t0 + i;
    if (t >= L) break;
    float acc = bc;
#pragma unroll
    for (int k = 0; k < K; ++k) acc = fmaf(wk[k], xs[i + k], acc);
    if (silu) acc *= sigm(acc);
    orow[t] = from_f32<T>(acc);
  }
}

template <typename T, int K>
__global__ __launch_bounds__(256) void bwd_kernel(const T* __restrict__ x, size_t x_bstride,
                                                  const float* __restrict__ w,
                                                  const float* __restrict__ bias,
                                                  const T* __restrict__ dout, int C, int L,
                                                  int silu, T* __restrict__ dx, size_t dx_bstride,
                                                  float* __restrict__ part) {
  __shared__ float xs[SEG + 2 * MAXK];   // x at [t0 - (K-1), t0 + SEG + K - 1)
  __shared__ float gs[SEG + MAXK];       // g at [t0, t0 + SEG + K - 1)
  __shared__ float red[4][MAXK + 1];
  const int seg = blockIdx.x, c = blockIdx.y, b = blockIdx.z;
  const int t0 = seg * SEG;
  const T* row = x + (size_t)b * x_bstride + (size_t)c * L;
  const T* drow = dout + ((size_t)b * C + c) * L;
  for (int i = threadIdx.x; i < SEG + 2 * (K - 1); i += 256) {
    const int t = t0 - (K - 1) + i;
    xs[i] = (t >= 0 && t < L) ? to_f32(row[t]) : 0.f;
  }
  __syncthreads();
  float wk[K];
#pragma unroll
  for (int k = 0; k < K; ++k) wk[k] = w[c * K + k];
  const float bc = bias ? bias[c] : 0.f;
  for (int i = threadIdx.x; i < SEG + K - 1; i += 256) {
    const int t = t0 + i;
    float g = 0.f;
    if (t < L) {
      g = to_f32(drow[t]);
      if (silu) {
        float pre = bc;
#pragma unroll
        for (int k = 0; k < K; ++k) pre = fmaf(wk[k], xs[i + k], pre);
        const float s = sigm(pre);
        g *= s * fmaf(pre, 1.f - s, 1.f);
      }
    }
    gs[i] = g;
  }
  __syncthreads();
  float sw[K + 1];
#pragma unroll
  for (int k = 0; k <= K; ++k) sw[k] = 0.f;
  T* dxrow = dx + (size_t)b * dx_bstride + (size_t)c * L;
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    const int i = j * 256 + threadIdx.x;
    const int t = t0 + i;
    if (t >= L) break;
    float acc = 0.f;
#pragma unroll
    for (int k = 0; k < K; ++k) acc = fmaf(wk[k], gs[i + K - 1 - k], acc);
    dxrow[t] = from_f32<T>(acc);
    const float g = gs[i];
#pragma unroll
    for (int k = 0; k < K; ++k) sw[k] = fmaf(g, xs[i + k], sw[k]);  // x[t + k - (K-1)]
    sw[K] += g;
  }
  // block reduction of the K+1 partial sums (fixed order: deterministic)
#pragma unroll
  for (int k = 0; k <= K; ++k) sw[k] = wave_sum(sw[k]);
  const int wv = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
#pragma unroll
    for (int k = 0; k <= K; ++k) red[wv][k] = sw[k];
  }
  __syncthreads();
  if (threadIdx.x <= K) {
    const float v = (red[0][threadIdx.x] + red[1][threadIdx.x]) + (red[2][threadIdx.x] + red[3][threadIdx.x]);
    part[((size_t)b * gridDim.x + seg) * C * (K + 1) + (size_t)c * (K + 1) + threadIdx.x] = v;
  }
}

// ---- vectorised forms (rows 16-B aligned, L % 8 == 0): a lane owns NV chunks of 8 consecutive
// positions (one 16-B bf16 / two 16-B fp32 loads per tensor and chunk, the same for the stores);
// chunk j of a wave covers 512 contiguous positions and the wave's NV chunks are adjacent. The K-1
// halo comes from the neighbouring lane by a shuffle, across a chunk edge from the other chunk's
// edge lane by readlane, and only at the wave's two edges from direct loads, issued together with
// the chunk loads (no second dependent memory round trip); no LDS, no block barrier in the
// forward. Block = 4 waves x NV x 512 positions of one row.
constexpr int VPL = 8;
constexpr int MAXNV = 2;
constexpr int WSPAN = 64 * VPL;  // positions per chunk of a wave

template <typename T>
__device__ __forceinline__ void ld8v(const T* p, float (&v)[VPL]) {
  if constexpr (sizeof(T) == 2) {
    const bf16x8 q = *reinterpret_cast<const bf16x8*>(p);
#pragma unroll
    for (int i = 0; i < VPL; ++i) v[i] = (float)q[i];
  } else {
    const f32x4 a = *reinterpret_cast<const f32x4*>(p), b = *reinterpret_cast<const f32x4*>(p + 4);
#pragma unroll
    for (int i = 0; i < 4; ++i) { v[i] = a[i]; v[4 + i] = b[i]; }
  }
}
template <typename T>
__device__ __forceinline__ void st8v(T* p, const float (&v)[VPL]) {
  if constexpr (sizeof(T) == 2) {
    bf16x8 q;
#pragma unroll
    for (int i = 0; i < VPL; ++i) q[i] = (bf16)v[i];
    *reinterpret_cast<bf16x8*>(p) = q;
  } else {
    *reinterpret_cast<f32x4*>(p) = f32x4{v[0], v[1], v[2], v[3]};
    *reinterpret_cast<f32x4*>(p + 4) = f32x4{v[4], v[5], v[6], v[7]};
  }
}

// first position of the lane's chunk j (L % 8 == 0: a chunk is wholly inside or past the row)
template <int NV>
__device__ __forceinline__ int chunk_t0(int j) {
  return blockIdx.x * (256 * VPL * NV) + (threadIdx.x >> 6) * (NV * WSPAN) + j * WSPAN + (threadIdx.x & 63) * VPL;
}
__device__ __forceinline__ float lane_of(float v, int l) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
}

template <typename T, int K, int NV>
__global__ __launch_bounds__(256) void fwd_vec_kernel(const T* __restrict__ x, size_t x_bstride,
                                                      const float* __restrict__ w,
                                                      const float* __restrict__ bias, int C, int L,
                                                      int silu, T* __restrict__ out) {
  constexpr int KH = K > 1 ? K - 1 : 1;
  const int c = blockIdx.y, b = blockIdx.z, lane = threadIdx.x & 63;
  const T* row = x + (size_t)b * x_bstride + (size_t)c * L;
  float v[NV][VPL], hp[KH];
  // every load first: the chunks and, on lane 0, the K-1 positions before the wave
#pragma unroll
  for (int j = 0; j < NV; ++j) {
    const int t0 = chunk_t0<NV>(j);
    if (t0 < L) ld8v(row + t0, v[j]);
    else {
#pragma unroll
      for (int i = 0; i < VPL; ++i) v[j][i] = 0.f;
    }
  }
#pragma unroll
  for (int k = 0; k < KH; ++k) {
    const int t = chunk_t0<NV>(0) - (K - 1) + k;
    hp[k] = (lane == 0 && t >= 0 && t < L) ? to_f32(row[t]) : 0.f;
  }
  float wk[K];
#pragma unroll
  for (int k = 0; k < K; ++k) wk[k] = w[c * K + k];
  const float bc = bias ? bias[c] : 0.f;
  T* orow = out + ((size_t)b * C + c) * L;
#pragma unroll
  for (int j = 0; j < NV; ++j) {
    const int t0 = chunk_t0<NV>(j);
    // h[k] = x[t0 - (K-1) + k]: the previous lane's last K-1 (lane 0: the previous chunk's lane 63)
    float h[KH];
#pragma unroll
    for (int k = 0; k < K - 1; ++k) {
      const float up = __shfl_up(v[j][VPL - (K - 1) + k], 1, 64);
      const float edge = j == 0 ? hp[k] : lane_of(v[j > 0 ? j - 1 : 0][VPL - (K - 1) + k], 63);
      h[k] = lane == 0 ? edge : up;
    }
    if (t0 < L) {
      float o[VPL];
#pragma unroll
      for (int i = 0; i < VPL; ++i) {
        float acc = bc;
#pragma unroll
        for (int k = 0; k < K; ++k) {
          const int q = i + k - (K - 1);  // x index relative to t0
          acc = fmaf(wk[k], q < 0 ? h[q + K - 1] : v[j][q], acc);
        }
        if (silu) acc *= sigm(acc);
        o[i] = acc;
      }
      st8v(orow + t0, o);
    }
  }
}

template <typename T, int K, int NV>
__global__ __launch_bounds__(256) void bwd_vec_kernel(const T* __restrict__ x, size_t x_bstride,
                                                      const float* __restrict__ w,
                                                      const float* __restrict__ bias,
                                                      const T* __restrict__ dout, int C, int L,
                                                      int silu, T* __restrict__ dx,
                                                      size_t dx_bstride, float* __restrict__ part) {
  constexpr int KH = K > 1 ? K - 1 : 1;
  __shared__ float red[4][MAXK + 1];
  const int c = blockIdx.y, b = blockIdx.z, lane = threadIdx.x & 63;
  const T* row = x + (size_t)b * x_bstride + (size_t)c * L;
  const T* drow = dout + ((size_t)b * C + c) * L;
  // every load first: x and dout of the chunks; lane 0 the x before the wave, lane 63 the x and
  // dout after it (for the g halo of the wave's last position)
  float xv[NV][VPL], dv[NV][VPL], xp[KH], xn[KH], dn[KH];
#pragma unroll
  for (int j = 0; j < NV; ++j) {
    const int t0 = chunk_t0<NV>(j);
    if (t0 < L) { ld8v(row + t0, xv[j]); ld8v(drow + t0, dv[j]); }
    else {
#pragma unroll
      for (int i = 0; i < VPL; ++i) xv[j][i] = dv[j][i] = 0.f;
    }
  }
#pragma unroll
  for (int k = 0; k < KH; ++k) {
    const int tp = chunk_t0<NV>(0) - (K - 1) + k, tn = chunk_t0<NV>(NV - 1) + VPL + k;
    xp[k] = (lane == 0 && tp >= 0 && tp < L) ? to_f32(row[tp]) : 0.f;
    const bool nx = lane == 63 && tn < L;
    xn[k] = nx ? to_f32(row[tn]) : 0.f;
    dn[k] = nx ? to_f32(drow[tn]) : 0.f;
  }
  float wk[K];
#pragma unroll
  for (int k = 0; k < K; ++k) wk[k] = w[c * K + k];
  const float bc = bias ? bias[c] : 0.f;
  auto gate = [&](float d, float pre) {  // dout * silu'(pre)
    const float s = sigm(pre);
    return d * (s * fmaf(pre, 1.f - s, 1.f));
  };
  // x before each lane's chunk: the previous lane's last K-1 (lane 0: the previous chunk's lane 63,
  // or the direct loads at the wave's start)
  float xh[NV][KH];
#pragma unroll
  for (int j = 0; j < NV; ++j) {
#pragma unroll
    for (int k = 0; k < K - 1; ++k) {
      const float up = __shfl_up(xv[j][VPL - (K - 1) + k], 1, 64);
      const float edge = j == 0 ? xp[k] : lane_of(xv[j > 0 ? j - 1 : 0][VPL - (K - 1) + k], 63);
      xh[j][k] = lane == 0 ? edge : up;
    }
  }
  // g = dout * silu'(pre) on the lane's positions (0 past L)
  float g[NV][VPL];
#pragma unroll
  for (int j = 0; j < NV; ++j) {
    const bool live = chunk_t0<NV>(j) < L;
#pragma unroll
    for (int i = 0; i < VPL; ++i) {
      float gi = dv[j][i];
      if (silu) {
        float pre = bc;
#pragma unroll
        for (int k = 0; k < K; ++k) {
          const int q = i + k - (K - 1);
          pre = fmaf(wk[k], q < 0 ? xh[j][q + K - 1] : xv[j][q], pre);
        }
        gi = gate(gi, pre);
      }
      g[j][i] = live ? gi : 0.f;
    }
  }
  // g at the wave's end (lane 63 of the last chunk): from the direct loads
  float gl[KH];
#pragma unroll
  for (int k = 0; k < K - 1; ++k) {
    float gk = dn[k];
    if (silu) {
      float pre = bc;
#pragma unroll
      for (int kk = 0; kk < K; ++kk) {
        const int q = VPL + k + kk - (K - 1);  // relative to the last chunk's t0
        pre = fmaf(wk[kk], q < VPL ? xv[NV - 1][q] : xn[q - VPL], pre);
      }
      gk = gate(gk, pre);
    }
    gl[k] = gk;
  }
  float sw[K + 1];
#pragma unroll
  for (int k = 0; k <= K; ++k) sw[k] = 0.f;
  T* dxrow = dx + (size_t)b * dx_bstride + (size_t)c * L;
#pragma unroll
  for (int j = 0; j < NV; ++j) {
    const int t0 = chunk_t0<NV>(j);
    // g after the lane: the next lane's first K-1 (lane 63: the next chunk's lane 0, or gl)
    float gh[KH];
#pragma unroll
    for (int k = 0; k < K - 1; ++k) {
      const float dn_ = __shfl_down(g[j][k], 1, 64);
      const float edge = j == NV - 1 ? gl[k] : lane_of(g[j < NV - 1 ? j + 1 : j][k], 0);
      gh[k] = lane == 63 ? edge : dn_;
    }
    if (t0 < L) {
      float o[VPL];
#pragma unroll
      for (int i = 0; i < VPL; ++i) {
        float acc = 0.f;
#pragma unroll
        for (int k = 0; k < K; ++k) {
          const int q = i + K - 1 - k;  // g index relative to t0
          acc = fmaf(wk[k], q < VPL ? g[j][q] : gh[q - VPL], acc);
        }
        o[i] = acc;
#pragma unroll
        for (int k = 0; k < K; ++k) {
          const int q = i + k - (K - 1);
          sw[k] = fmaf(g[j][i], q < 0 ? xh[j][q + K - 1] : xv[j][q], sw[k]);
        }
        sw[K] += g[j][i];
      }
      st8v(dxrow + t0, o);
    }
  }
#pragma unroll
  for (int k = 0; k <= K; ++k) sw[k] = wave_sum(sw[k]);
  const int wv = threadIdx.x >> 6;
  if (lane == 0) {
#pragma unroll
    for (int k = 0; k <= K; ++k) red[wv][k] = sw[k];
  }
  __syncthreads();
  if (threadIdx.x <= K) {
    const float s = (red[0][threadIdx.x] + red[1][threadIdx.x]) + (red[2][threadIdx.x] + red[3][threadIdx.x]);
    part[((size_t)b * gridDim.x + blockIdx.x) * C * (K + 1) + (size_t)c * (K + 1) + threadIdx.x] = s;
  }
}

template <typename F>
int dispatch(int dtype, int K, F&& f) {
  if (dtype != DNA_F32 && dtype != DNA_BF16) return -1;
  const bool fp = dtype == DNA_F32;
  switch (K) {
    case 2: fp ? f(float(), std::integral_constant<int, 2>()) : f(bf16(), std::integral_constant<int, 2>()); return 0;
    case 3: fp ? f(float(), std::integral_constant<int, 3>()) : f(bf16(), std::integral_constant<int, 3>()); return 0;
    case 4: fp ? f(float(), std::integral_constant<int, 4>()) : f(bf16(), std::integral_constant<int, 4>()); return 0;
    default: return -1;
  }
}

}  // namespace cconv
}  // namespace dna

using namespace dna;
using namespace dna::cconv;

// 8-position chunks per lane of the 16-B path (DNA_CCONV_NV = 1 | 2, default 2; an A/B switch)
static int conv_nv() {
  static const int nv = [] {
    const char* e = getenv("DNA_CCONV_NV");
    return e && atoi(e) == 1 ? 1 : MAXNV;
  }();
  return nv;
}
static int vseg() { return 256 * VPL * conv_nv(); }

// the 16-B path: every row start 16-B aligned (L and the batch stride multiples of 8 elements)
static bool conv_vec_ok(const void* p, size_t bstride, int L) {
  return ((uintptr_t)p & 15) == 0 && L % 8 == 0 && bstride % 8 == 0;
}

extern "C" int dna_causal_conv1d_fwd(const void* x, size_t x_bstride, int dtype, const float* w,
                                     const float* bias, int B, int C, int L, int K, int silu,
                                     void* out, void* stream) {
  DNA_CHECK_ARG(x && w && out && B > 0 && C > 0 && L > 0, "dna_causal_conv1d_fwd: bad args");
  const bool vec = conv_vec_ok(x, x_bstride, L) && conv_vec_ok(out, (size_t)C * L, L);
  const dim3 grid(vec ? (L + vseg() - 1) / vseg() : (L + SEG - 1) / SEG, C, B);
  hipStream_t s = as_stream(stream);
  const int st = dispatch(dtype, K, [&](auto t, auto kk) {
    using T = decltype(t);
    if (vec && conv_nv() == 1)
      hipLaunchKernelGGL((fwd_vec_kernel<T, decltype(kk)::value, 1>), grid, dim3(256), 0, s, (const T*)x,
                         x_bstride, w, bias, C, L, silu, (T*)out);
    else if (vec)
      hipLaunchKernelGGL((fwd_vec_kernel<T, decltype(kk)::value, MAXNV>), grid, dim3(256), 0, s, (const T*)x,
                         x_bstride, w, bias, C, L, silu, (T*)out);
    else
      hipLaunchKernelGGL((fwd_kernel<T, decltype(kk)::value>), grid, dim3(256), 0, s, (const T*)x,
                         x_bstride, w, bias, C, L, silu, (T*)out);
  });
  DNA_CHECK_ARG(st == 0, "dna_causal_conv1d_fwd: kernel size %d / dtype %d unsupported (2..4; f32/bf16)", K, dtype);
  DNA_LAUNCH_CHECK("dna_causal_conv1d_fwd");
  return DNA_OK;
}

// partial rows of the backward's dw / dbias: one per (batch, block); the 16-B path (L % 8 == 0)
// uses 2048 * NV-position blocks, the element path 1024
extern "C" size_t dna_causal_conv1d_part_rows(int B, int L) {
  return (size_t)B * (L % 8 == 0 ? (L + vseg() - 1) / vseg() : (L + SEG - 1) / SEG);
}

extern "C" int dna_causal_conv1d_bwd(const void* x, size_t x_bstride, int dtype, const float* w,
                                     const float* bias, const void* dout, int B, int C, int L,
                                     int K, int silu, void* dx, size_t dx_bstride, float* part,
                                     void* stream) {
  DNA_CHECK_ARG(x && w && dout && dx && part && B > 0 && C > 0 && L > 0,
                "dna_causal_conv1d_bwd: bad args");
  // the partial-row count must match dna_causal_conv1d_part_rows (it depends on L only): a
  // misaligned pointer with L % 8 == 0 is refused rather than run on the element kernel's rows
  const bool vec = L % 8 == 0 && conv_vec_ok(x, x_bstride, L) && conv_vec_ok(dout, (size_t)C * L, L) &&
                   conv_vec_ok(dx, dx_bstride, L);
  DNA_CHECK_ARG(vec || L % 8 != 0, "dna_causal_conv1d_bwd: L %% 8 == 0 needs 16-B aligned rows");
  const dim3 grid(vec ? (L + vseg() - 1) / vseg() : (L + SEG - 1) / SEG, C, B);
  hipStream_t s = as_stream(stream);
  const int st = dispatch(dtype, K, [&](auto t, auto kk) {
    using T = decltype(t);
    if (vec && conv_nv() == 1)
      hipLaunchKernelGGL((bwd_vec_kernel<T, decltype(kk)::value, 1>), grid, dim3(256), 0, s, (const T*)x,
                         x_bstride, w, bias, (const T*)dout, C, L, silu, (T*)dx, dx_bstride, part);
    else if (vec)
      hipLaunchKernelGGL((bwd_vec_kernel<T, decltype(kk)::value, MAXNV>), grid, dim3(256), 0, s, (const T*)x,
                         x_bstride, w, bias, (const T*)dout, C, L, silu, (T*)dx, dx_bstride, part);
    else
      hipLaunchKernelGGL((bwd_kernel<T, decltype(kk)::value>), grid, dim3(256), 0, s, (const T*)x,
                         x_bstride, w, bias, (const T*)dout, C, L, silu, (T*)dx, dx_bstride, part);
  });
  DNA_CHECK_ARG(st == 0, "dna_causal_conv1d_bwd: kernel size %d / dtype %d unsupported (2..4; f32/bf16)", K, dtype);
  DNA_LAUNCH_CHECK("dna_causal_conv1d_bwd");
  return DNA_OK;
}
