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
// A block = 256 threads x 4 positions = 1024 positions of one (b, c) row; the K-1 halo comes
// from LDS. HBM-bound (reads x, writes out; bwd reads x, dout, writes dx).
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

extern "C" int dna_causal_conv1d_fwd(const void* x, size_t x_bstride, int dtype, const float* w,
                                     const float* bias, int B, int C, int L, int K, int silu,
                                     void* out, void* stream) {
  DNA_CHECK_ARG(x && w && out && B > 0 && C > 0 && L > 0, "dna_causal_conv1d_fwd: bad args");
  const dim3 grid((L + SEG - 1) / SEG, C, B);
  hipStream_t s = as_stream(stream);
  const int st = dispatch(dtype, K, [&](auto t, auto kk) {
    using T = decltype(t);
    hipLaunchKernelGGL((fwd_kernel<T, decltype(kk)::value>), grid, dim3(256), 0, s, (const T*)x,
                       x_bstride, w, bias, C, L, silu, (T*)out);
  });
  DNA_CHECK_ARG(st == 0, "dna_causal_conv1d_fwd: kernel size %d / dtype %d unsupported (2..4; f32/bf16)", K, dtype);
  DNA_LAUNCH_CHECK("dna_causal_conv1d_fwd");
  return DNA_OK;
}

extern "C" size_t dna_causal_conv1d_part_rows(int B, int L) { return (size_t)B * ((L + SEG - 1) / SEG); }

extern "C" int dna_causal_conv1d_bwd(const void* x, size_t x_bstride, int dtype, const float* w,
                                     const float* bias, const void* dout, int B, int C, int L,
                                     int K, int silu, void* dx, size_t dx_bstride, float* part,
                                     void* stream) {
  DNA_CHECK_ARG(x && w && dout && dx && part && B > 0 && C > 0 && L > 0,
                "dna_causal_conv1d_bwd: bad args");
  const dim3 grid((L + SEG - 1) / SEG, C, B);
  hipStream_t s = as_stream(stream);
  const int st = dispatch(dtype, K, [&](auto t, auto kk) {
    using T = decltype(t);
    hipLaunchKernelGGL((bwd_kernel<T, decltype(kk)::value>), grid, dim3(256), 0, s, (const T*)x,
                       x_bstride, w, bias, (const T*)dout, C, L, silu, (T*)dx, dx_bstride, part);
  });
  DNA_CHECK_ARG(st == 0, "dna_causal_conv1d_bwd: kernel size %d / dtype %d unsupported (2..4; f32/bf16)", K, dtype);
  DNA_LAUNCH_CHECK("dna_causal_conv1d_bwd");
  return DNA_OK;
}
