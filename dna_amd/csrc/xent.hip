// Masked-LM cross entropy over the compact [M, V] logits of the masked rows.
// Reference: model-internal CE (bert_layers.py:820-824) and task loss bert_cross_entropy
// (src/tasks/metrics.py:268-273), computed under autocast in fp32 on bf16 logits.
// One wave per row (V = 4096 -> 64 values per lane); fwd keeps the row LSE for bwd.
#include "common.h"

namespace dna {
namespace xent {

template <typename T>
__device__ __forceinline__ float ld(const T* p, int i) { return to_f32(p[i]); }

template <typename T>
__global__ __launch_bounds__(256) void fwd_kernel(const T* __restrict__ logits,
                                                  const int64_t* __restrict__ target, int rows,
                                                  int V, float* __restrict__ loss,
                                                  float* __restrict__ lse) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const T* x = logits + (size_t)row * V;
  float m = -INFINITY;
  for (int i = lane; i < V; i += 64) m = fmaxf(m, ld(x, i));
  m = wave_max(m);
  float s = 0.f;
  for (int i = lane; i < V; i += 64) s += __expf(ld(x, i) - m);
  s = wave_sum(s);
  if (lane == 0) {
    const float l = m + __logf(s);
    long t = (long)target[row];
    const float xt = (t >= 0 && t < V) ? ld(x, (int)t) : 0.f;
    lse[row] = l;
    loss[row] = l - xt;
  }
}

template <typename T>
__global__ __launch_bounds__(256) void bwd_kernel(const T* __restrict__ logits,
                                                  const int64_t* __restrict__ target,
                                                  const float* __restrict__ lse,
                                                  const float* __restrict__ dloss, float scale,
                                                  int rows, int V, T* __restrict__ dlogits) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const T* x = logits + (size_t)row * V;
  T* dx = dlogits + (size_t)row * V;
  const float g = dloss[0] * scale, l = lse[row];
  const long t = (long)target[row];
  for (int i = lane; i < V; i += 64) {
    float p = __expf(ld(x, i) - l);
    dx[i] = from_f32<T>((p - (i == t ? 1.f : 0.f)) * g);
  }
}

// bf16, V = 512 * NV: each lane holds NV 16-B vectors of the row in registers, so the row is read
// once (max and exp-sum from registers) with wide loads; the per-row loop above issues 2-B loads
// and reads the row twice
template <int NV>
__global__ __launch_bounds__(256) void fwd_vec_kernel(const bf16* __restrict__ logits,
                                                      const int64_t* __restrict__ target, int rows,
                                                      float* __restrict__ loss,
                                                      float* __restrict__ lse) {
  constexpr int V = 512 * NV;
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const bf16* x = logits + (size_t)row * V;
  bf16x8 v[NV];
#pragma unroll
  for (int j = 0; j < NV; ++j) v[j] = *reinterpret_cast<const bf16x8*>(x + (j * 64 + lane) * 8);
  float m = -INFINITY;
#pragma unroll
  for (int j = 0; j < NV; ++j)
#pragma unroll
    for (int e = 0; e < 8; ++e) m = fmaxf(m, (float)v[j][e]);
  m = wave_max(m);
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < NV; ++j)
#pragma unroll
    for (int e = 0; e < 8; ++e) s += __expf((float)v[j][e] - m);
  s = wave_sum(s);
  if (lane == 0) {
    const float l = m + __logf(s);
    const long t = (long)target[row];
    const float xt = (t >= 0 && t < V) ? (float)x[t] : 0.f;
    lse[row] = l;
    loss[row] = l - xt;
  }
}

template <int NV>
__global__ __launch_bounds__(256) void bwd_vec_kernel(const bf16* __restrict__ logits,
                                                      const int64_t* __restrict__ target,
                                                      const float* __restrict__ lse,
                                                      const float* __restrict__ dloss, float scale,
                                                      int rows, bf16* __restrict__ dlogits) {
  constexpr int V = 512 * NV;
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const bf16* x = logits + (size_t)row * V;
  bf16* dx = dlogits + (size_t)row * V;
  const float g = dloss[0] * scale, l = lse[row];
  const long t = (long)target[row];
  bf16x8 v[NV];
#pragma unroll
  for (int j = 0; j < NV; ++j) v[j] = *reinterpret_cast<const bf16x8*>(x + (j * 64 + lane) * 8);
#pragma unroll
  for (int j = 0; j < NV; ++j) {
    const int i0 = (j * 64 + lane) * 8;
    bf16x8 o;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float p = __expf((float)v[j][e] - l);
      o[e] = (bf16)((p - (i0 + e == t ? 1.f : 0.f)) * g);
    }
    *reinterpret_cast<bf16x8*>(dx + i0) = o;
  }
}

}  // namespace xent
}  // namespace dna

using namespace dna;

extern "C" int dna_xent_fwd(const void* logits, int dtype, const int64_t* target, int rows,
                            int vocab, float* row_loss, float* row_lse, void* stream) {
  DNA_CHECK_ARG(logits && target && row_loss && row_lse, "dna_xent_fwd: null pointer");
  if (rows == 0) return DNA_OK;
  dim3 grid((rows + 3) / 4);
  hipStream_t s = as_stream(stream);
  const bool aligned = ((uintptr_t)logits & 15) == 0;
  if (dtype == DNA_BF16 && aligned && vocab == 4096)
    hipLaunchKernelGGL(xent::fwd_vec_kernel<8>, grid, dim3(256), 0, s, (const bf16*)logits, target,
                       rows, row_loss, row_lse);
  else if (dtype == DNA_BF16)
    hipLaunchKernelGGL(xent::fwd_kernel<bf16>, grid, dim3(256), 0, s, (const bf16*)logits, target,
                       rows, vocab, row_loss, row_lse);
  else if (dtype == DNA_F32)
    hipLaunchKernelGGL(xent::fwd_kernel<float>, grid, dim3(256), 0, s, (const float*)logits,
                       target, rows, vocab, row_loss, row_lse);
  else
    DNA_CHECK_ARG(false, "dna_xent_fwd: bad dtype");
  DNA_LAUNCH_CHECK("dna_xent_fwd");
  return DNA_OK;
}

extern "C" int dna_xent_bwd(const void* logits, int dtype, const int64_t* target,
                            const float* row_lse, const float* dloss, float scale, int rows,
                            int vocab, void* dlogits, void* stream) {
  DNA_CHECK_ARG(logits && target && row_lse && dloss && dlogits, "dna_xent_bwd: null pointer");
  if (rows == 0) return DNA_OK;
  dim3 grid((rows + 3) / 4);
  hipStream_t s = as_stream(stream);
  const bool aligned = (((uintptr_t)logits | (uintptr_t)dlogits) & 15) == 0;
  if (dtype == DNA_BF16 && aligned && vocab == 4096)
    hipLaunchKernelGGL(xent::bwd_vec_kernel<8>, grid, dim3(256), 0, s, (const bf16*)logits, target,
                       row_lse, dloss, scale, rows, (bf16*)dlogits);
  else if (dtype == DNA_BF16)
    hipLaunchKernelGGL(xent::bwd_kernel<bf16>, grid, dim3(256), 0, s, (const bf16*)logits, target,
                       row_lse, dloss, scale, rows, vocab, (bf16*)dlogits);
  else if (dtype == DNA_F32)
    hipLaunchKernelGGL(xent::bwd_kernel<float>, grid, dim3(256), 0, s, (const float*)logits,
                       target, row_lse, dloss, scale, rows, vocab, (float*)dlogits);
  else
    DNA_CHECK_ARG(false, "dna_xent_bwd: bad dtype");
  DNA_LAUNCH_CHECK("dna_xent_bwd");
  return DNA_OK;
}
