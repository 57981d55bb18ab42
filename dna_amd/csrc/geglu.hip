// GeGLU (+ dropout) of BertGatedLinearUnitMLP (bert_layers.py:292-296), fwd and bwd.
//   a = dropout( gelu_erf(g[:, :F]) * g[:, F:] ),  g = gated_layers(x) with F = intermediate_size.
// The forward also writes the backward factors fac = [d a / d g1 | d a / d g2] (common.h
// geglu_fwd_fac: dropout and 1/(1-p) folded in), optionally over g itself, so the backward is
// dg = da * fac -- the same arithmetic as the fused GEMM epilogues (csrc/gemm.hip).
// HBM-bound elementwise: 8 consecutive outputs per thread (16-B bf16 vectors), grid-stride,
// U rows per thread per iteration.
// Algorithmic bytes per output element: fwd 2*s (read g1, g2) + s (write a) [+ 2*s fac];
// bwd 3*s + 2*s.
// Dropout bits: dropout_keep8 (16-bit slices of one Philox draw per 8 elements).
#include "common.h"

namespace dna {
namespace geglu {

template <typename T> struct Vec8;
template <> struct Vec8<bf16> {
  bf16x8 v;
  __device__ __forceinline__ void load(const bf16* p) { v = *reinterpret_cast<const bf16x8*>(p); }
  __device__ __forceinline__ float operator[](int i) const { return (float)v[i]; }
  __device__ __forceinline__ static void store(bf16* p, const float (&f)[8]) {
    bf16x8 o;
#pragma unroll
    for (int i = 0; i < 8; ++i) o[i] = (bf16)f[i];
    *reinterpret_cast<bf16x8*>(p) = o;
  }
};
template <> struct Vec8<float> {
  f32x4 a, b;
  __device__ __forceinline__ void load(const float* p) {
    a = *reinterpret_cast<const f32x4*>(p);
    b = *reinterpret_cast<const f32x4*>(p + 4);
  }
  __device__ __forceinline__ float operator[](int i) const { return i < 4 ? a[i] : b[i - 4]; }
  __device__ __forceinline__ static void store(float* p, const float (&f)[8]) {
    *reinterpret_cast<f32x4*>(p) = f32x4{f[0], f[1], f[2], f[3]};
    *reinterpret_cast<f32x4*>(p + 4) = f32x4{f[4], f[5], f[6], f[7]};
  }
};

__device__ __forceinline__ uint32_t keep8(uint64_t seed, uint64_t off, uint64_t elem, uint32_t th16) {
  return dropout_keep8(seed, off, elem >> 3, th16);  // elem is a multiple of 8
}

// U rows per iteration: every load of the U rows is issued before any arithmetic, so a wave
// keeps U*2 (fwd) / U*3 (bwd) 16-B vectors per lane in flight instead of 2 / 3 (the U=1 kernels
// reached only 66 % of HBM bandwidth at the bench shape).
template <typename T, int U>
__global__ __launch_bounds__(128) void fwd_kernel(const T* g, int rows, int F,
                                                  float p, uint32_t th, float ks, uint64_t seed,
                                                  uint64_t off, T* __restrict__ a, T* fac) {
  // fac may alias g (each thread reads its g1 / g2 vectors before writing the same places)
  // 2-D launch: blockIdx.y walks row groups, x covers one row's F/8 vectors (no 64-bit div/mod)
  const int f8 = F / 8;
  for (int r0 = blockIdx.y * U; r0 < rows; r0 += gridDim.y * U)
  for (int v = blockIdx.x * blockDim.x + threadIdx.x; v < f8; v += gridDim.x * blockDim.x) {
    const size_t c = (size_t)v * 8;
    Vec8<T> g1[U], g2[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int r = min(r0 + u, rows - 1);  // tail rows re-read the last row, never stored
      g1[u].load(g + (size_t)r * 2 * F + c);
      g2[u].load(g + (size_t)r * 2 * F + F + c);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int r = r0 + u;
      if (U > 1 && r >= rows) break;
      const size_t e = (size_t)r * F + c;
      float o[8], f1[8], f2[8];
      uint32_t keep = p > 0.f ? keep8(seed, off, e, th) : 0xFFu;
#pragma unroll
      for (int j = 0; j < 8; ++j) geglu_fwd_fac(g1[u][j], g2[u][j], (keep >> j) & 1, ks, o[j], f1[j], f2[j]);
      Vec8<T>::store(a + e, o);
      if (fac) {
        Vec8<T>::store(fac + (size_t)r * 2 * F + c, f1);
        Vec8<T>::store(fac + (size_t)r * 2 * F + F + c, f2);
      }
    }
  }
}

template <typename T, int U>
__global__ __launch_bounds__(128) void bwd_kernel(const T* __restrict__ da, const T* __restrict__ g,
                                                  int rows, int F, T* __restrict__ dg) {
  // g = the forward's factors fac: dg = [da * fac1 | da * fac2]
  const int f8 = F / 8;
  for (int r0 = blockIdx.y * U; r0 < rows; r0 += gridDim.y * U)
  for (int v = blockIdx.x * blockDim.x + threadIdx.x; v < f8; v += gridDim.x * blockDim.x) {
    const size_t c = (size_t)v * 8;
    Vec8<T> g1[U], g2[U], d[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int r = min(r0 + u, rows - 1);
      g1[u].load(g + (size_t)r * 2 * F + c);
      g2[u].load(g + (size_t)r * 2 * F + F + c);
      d[u].load(da + (size_t)r * F + c);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int r = r0 + u;
      if (U > 1 && r >= rows) break;
      float o1[8], o2[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        o1[j] = d[u][j] * g1[u][j];
        o2[j] = d[u][j] * g2[u][j];
      }
      Vec8<T>::store(dg + (size_t)r * 2 * F + c, o1);
      Vec8<T>::store(dg + (size_t)r * 2 * F + F + c, o2);
    }
  }
}

// Rows per iteration (bf16 bench path; DNA_GEGLU_UNROLL=1/2/4 for A/B runs).
inline int unroll_rows(int rows) {
  static const int env = getenv("DNA_GEGLU_UNROLL") ? atoi(getenv("DNA_GEGLU_UNROLL")) : 0;
  int u = env == 1 || env == 2 || env == 4 ? env : 2;
  while (u > 1 && rows < 2048 * u) u /= 2;  // small launches keep one row per block
  return u;
}

inline dim3 grid_for(int rows, int F, int u = 1) {
  const int bx = (F / 8 + 127) / 128;  // 3072/8 = 384 vectors -> 3 blocks of 128 per row
  const int groups = (rows + u - 1) / u;
  const int by = groups < 8192 ? (groups ? groups : 1) : 8192;
  return dim3(bx, by);
}

}  // namespace geglu
}  // namespace dna

using namespace dna;

extern "C" int dna_geglu_fwd(const void* g, int dtype, int rows, int inter, float p_drop,
                             uint64_t seed, uint64_t offset, void* a, void* fac, void* stream) {
  DNA_CHECK_ARG(g && a, "dna_geglu_fwd: null pointer");
  DNA_CHECK_ARG(inter % 8 == 0 && rows >= 0, "dna_geglu_fwd: intermediate %% 8 != 0");
  DNA_CHECK_ARG(p_drop >= 0.f && p_drop < 1.f, "dna_geglu_fwd: bad p");
  if (rows == 0) return DNA_OK;
  hipStream_t s = as_stream(stream);
  const uint32_t th = dropout_threshold16(p_drop);
  const float ks = 1.f / (1.f - p_drop);
  const int u = dtype == DNA_BF16 ? geglu::unroll_rows(rows) : 1;
  const dim3 grid = geglu::grid_for(rows, inter, u);
  if (dtype == DNA_BF16 && u == 4)
    hipLaunchKernelGGL((geglu::fwd_kernel<bf16, 4>), grid, dim3(128), 0, s, (const bf16*)g,
                       rows, inter, p_drop, th, ks, seed, offset, (bf16*)a, (bf16*)fac);
  else if (dtype == DNA_BF16 && u == 2)
    hipLaunchKernelGGL((geglu::fwd_kernel<bf16, 2>), grid, dim3(128), 0, s, (const bf16*)g,
                       rows, inter, p_drop, th, ks, seed, offset, (bf16*)a, (bf16*)fac);
  else if (dtype == DNA_BF16)
    hipLaunchKernelGGL((geglu::fwd_kernel<bf16, 1>), grid, dim3(128), 0, s, (const bf16*)g,
                       rows, inter, p_drop, th, ks, seed, offset, (bf16*)a, (bf16*)fac);
  else if (dtype == DNA_F32)
    hipLaunchKernelGGL((geglu::fwd_kernel<float, 1>), grid, dim3(128), 0, s, (const float*)g,
                       rows, inter, p_drop, th, ks, seed, offset, (float*)a, (float*)fac);
  else
    DNA_CHECK_ARG(false, "dna_geglu_fwd: bad dtype");
  DNA_LAUNCH_CHECK("dna_geglu_fwd");
  return DNA_OK;
}

extern "C" int dna_geglu_bwd(const void* da, const void* fac, int dtype, int rows, int inter,
                             void* dg, void* stream) {
  DNA_CHECK_ARG(da && fac && dg, "dna_geglu_bwd: null pointer");
  DNA_CHECK_ARG(inter % 8 == 0 && rows >= 0, "dna_geglu_bwd: intermediate %% 8 != 0");
  if (rows == 0) return DNA_OK;
  hipStream_t s = as_stream(stream);
  const void* g = fac;
  const int u = dtype == DNA_BF16 ? geglu::unroll_rows(rows) : 1;
  const dim3 grid = geglu::grid_for(rows, inter, u);
  if (dtype == DNA_BF16 && u == 4)
    hipLaunchKernelGGL((geglu::bwd_kernel<bf16, 4>), grid, dim3(128), 0, s, (const bf16*)da,
                       (const bf16*)g, rows, inter, (bf16*)dg);
  else if (dtype == DNA_BF16 && u == 2)
    hipLaunchKernelGGL((geglu::bwd_kernel<bf16, 2>), grid, dim3(128), 0, s, (const bf16*)da,
                       (const bf16*)g, rows, inter, (bf16*)dg);
  else if (dtype == DNA_BF16)
    hipLaunchKernelGGL((geglu::bwd_kernel<bf16, 1>), grid, dim3(128), 0, s, (const bf16*)da,
                       (const bf16*)g, rows, inter, (bf16*)dg);
  else if (dtype == DNA_F32)
    hipLaunchKernelGGL((geglu::bwd_kernel<float, 1>), grid, dim3(128), 0, s, (const float*)da,
                       (const float*)g, rows, inter, (float*)dg);
  else
    DNA_CHECK_ARG(false, "dna_geglu_bwd: bad dtype");
  DNA_LAUNCH_CHECK("dna_geglu_bwd");
  return DNA_OK;
}
