// Flat-buffer optimizer step: global grad L2 norm + clip (Lightning gradient_clip_val=1.0 ->
// torch.nn.utils.clip_grad_norm_) fused into torch-AdamW (train.py:462-542), one launch each.
// All 117,074,176 DNABERT-2 parameters live in ONE fp32 buffer (grads, exp_avg, exp_avg_sq
// likewise), so the whole optimizer is two grid-stride kernels instead of 141-tensor foreach
// loops; the clip coefficient is read from device memory (no host sync).
// HBM-bound: AdamW moves 4 (g) + 3*4 (p, m, v read) + 3*4 (write) [+2 bf16 copy] B/param.
#include "common.h"

namespace dna {
namespace opt {

constexpr int SUMSQ_BLOCKS = 1024;

__global__ __launch_bounds__(256) void sumsq_partial(const float* __restrict__ x, size_t n,
                                                     float* __restrict__ part) {
  __shared__ float red[4];
  float s = 0.f;
  const size_t n4 = n / 4;
  const f32x4* x4 = reinterpret_cast<const f32x4*>(x);
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n4;
       i += (size_t)gridDim.x * blockDim.x) {
    f32x4 v = x4[i];
    s += v[0] * v[0] + v[1] * v[1] + v[2] * v[2] + v[3] * v[3];
  }
  for (size_t i = n4 * 4 + blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n;
       i += (size_t)gridDim.x * blockDim.x)
    s += x[i] * x[i];
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) part[blockIdx.x] = red[0] + red[1] + red[2] + red[3];
}

__global__ __launch_bounds__(256) void sumsq_final(const float* __restrict__ part, int n,
                                                   float* __restrict__ out) {
  __shared__ float red[4];
  float s = 0.f;
  for (int i = threadIdx.x; i < n; i += 256) s += part[i];
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) out[0] = red[0] + red[1] + red[2] + red[3];
}

struct AdamArgs {
  float* p; const float* g; float* m; float* v; bf16* pb; size_t n;
  float lr, b1, b2, eps, wd, bc1, bc2_sqrt; const float* sumsq; float max_norm, gscale;
};

__device__ __forceinline__ void adam1(float& p, float g, float& m, float& v, const AdamArgs& a,
                                      float coef) {
  g *= coef;
  p *= 1.f - a.lr * a.wd;
  m = m + (1.f - a.b1) * (g - m);            // exp_avg.lerp_(grad, 1 - beta1)
  v = v * a.b2 + (1.f - a.b2) * g * g;       // exp_avg_sq.mul_(b2).addcmul_(g, g, 1 - b2)
  const float denom = sqrtf(v) / a.bc2_sqrt + a.eps;
  p = p - (a.lr / a.bc1) * (m / denom);
}

__global__ __launch_bounds__(256) void adamw_kernel(AdamArgs a) {
  float coef = a.gscale;
  if (a.sumsq) {
    const float norm = sqrtf(a.sumsq[0]) * a.gscale;
    coef *= fminf(1.f, a.max_norm / (norm + 1e-6f));
  }
  const size_t n4 = a.n / 4;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n4;
       i += (size_t)gridDim.x * blockDim.x) {
    f32x4 p = reinterpret_cast<f32x4*>(a.p)[i];
    f32x4 g = reinterpret_cast<const f32x4*>(a.g)[i];
    f32x4 m = reinterpret_cast<f32x4*>(a.m)[i];
    f32x4 v = reinterpret_cast<f32x4*>(a.v)[i];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float pj = p[j], mj = m[j], vj = v[j];
      adam1(pj, g[j], mj, vj, a, coef);
      p[j] = pj; m[j] = mj; v[j] = vj;
    }
    reinterpret_cast<f32x4*>(a.p)[i] = p;
    reinterpret_cast<f32x4*>(a.m)[i] = m;
    reinterpret_cast<f32x4*>(a.v)[i] = v;
    if (a.pb)
      reinterpret_cast<bf16x4*>(a.pb)[i] = bf16x4{(bf16)p[0], (bf16)p[1], (bf16)p[2], (bf16)p[3]};
  }
  for (size_t i = n4 * 4 + blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < a.n;
       i += (size_t)gridDim.x * blockDim.x) {
    adam1(a.p[i], a.g[i], a.m[i], a.v[i], a, coef);
    if (a.pb) a.pb[i] = (bf16)a.p[i];
  }
}

}  // namespace opt
}  // namespace dna

using namespace dna;

extern "C" size_t dna_sumsq_workspace(size_t n) {
  (void)n;
  return opt::SUMSQ_BLOCKS * sizeof(float);
}

extern "C" int dna_sumsq(const float* x, size_t n, float* out, void* workspace,
                         size_t workspace_bytes, void* stream) {
  DNA_CHECK_ARG(x && out && workspace, "dna_sumsq: null pointer");
  DNA_CHECK_ARG(workspace_bytes >= dna_sumsq_workspace(n), "dna_sumsq: workspace too small");
  DNA_CHECK_ARG(((uintptr_t)x & 15) == 0, "dna_sumsq: x must be 16-byte aligned");
  hipStream_t s = as_stream(stream);
  size_t blocks = (n / 4 + 255) / 256;
  int nb = (int)(blocks < opt::SUMSQ_BLOCKS ? (blocks ? blocks : 1) : opt::SUMSQ_BLOCKS);
  hipLaunchKernelGGL(opt::sumsq_partial, dim3(nb), dim3(256), 0, s, x, n, (float*)workspace);
  hipLaunchKernelGGL(opt::sumsq_final, dim3(1), dim3(256), 0, s, (const float*)workspace, nb, out);
  DNA_LAUNCH_CHECK("dna_sumsq");
  return DNA_OK;
}

extern "C" int dna_adamw_step(float* param, const float* grad, float* exp_avg,
                              float* exp_avg_sq, void* param_bf16, size_t n, float lr,
                              float beta1, float beta2, float eps, float weight_decay, int step,
                              const float* grad_sumsq, float max_grad_norm, float grad_scale,
                              void* stream) {
  DNA_CHECK_ARG(param && grad && exp_avg && exp_avg_sq, "dna_adamw_step: null pointer");
  DNA_CHECK_ARG(step >= 1, "dna_adamw_step: step must be >= 1");
  DNA_CHECK_ARG((((uintptr_t)param | (uintptr_t)grad | (uintptr_t)exp_avg |
                  (uintptr_t)exp_avg_sq) & 15) == 0 &&
                    (((uintptr_t)param_bf16) & 7) == 0,
                "dna_adamw_step: buffers must be 16-byte aligned (bf16 copy 8-byte)");
  opt::AdamArgs a{param, grad, exp_avg, exp_avg_sq, (bf16*)param_bf16, n, lr, beta1, beta2, eps,
                  weight_decay, (float)(1.0 - pow((double)beta1, step)),
                  (float)sqrt(1.0 - pow((double)beta2, step)), grad_sumsq, max_grad_norm,
                  grad_scale};
  size_t blocks = (n / 4 + 255) / 256;
  int nb = (int)(blocks < 8192 ? (blocks ? blocks : 1) : 8192);
  hipLaunchKernelGGL(opt::adamw_kernel, dim3(nb), dim3(256), 0, as_stream(stream), a);
  DNA_LAUNCH_CHECK("dna_adamw_step");
  return DNA_OK;
}
