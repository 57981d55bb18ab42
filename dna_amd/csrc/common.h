// Shared device/host helpers for the dna_amd HIP library (gfx950 / CDNA4 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "dna_amd.h"

namespace dna {

// ---------------------------------------------------------------------------------------- errors
// Thread-local last-error string behind dna_last_error() (include/dna_amd.h).
void set_error(const char* fmt, ...);

#define DNA_CHECK_ARG(cond, ...)                   \
  do {                                             \
    if (!(cond)) {                                 \
      ::dna::set_error(__VA_ARGS__);               \
      return DNA_ERR_INVALID;                      \
    }                                              \
  } while (0)

#define DNA_LAUNCH_CHECK(name)                                                   \
  do {                                                                           \
    hipError_t e_ = hipGetLastError();                                           \
    if (e_ != hipSuccess) {                                                      \
      ::dna::set_error("%s: launch failed: %s", name, hipGetErrorString(e_));    \
      return DNA_ERR_HIP;                                                        \
    }                                                                            \
  } while (0)

// ---------------------------------------------------------------------------------------- types
typedef __bf16 bf16;
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
typedef __attribute__((ext_vector_type(16))) float f32x16;
typedef __attribute__((ext_vector_type(4))) float f32x4;

__device__ __forceinline__ float to_f32(float x) { return x; }
__device__ __forceinline__ float to_f32(bf16 x) { return (float)x; }
template <typename T> __device__ __forceinline__ T from_f32(float x);
template <> __device__ __forceinline__ float from_f32<float>(float x) { return x; }
template <> __device__ __forceinline__ bf16 from_f32<bf16>(float x) { return (bf16)x; }

// ---------------------------------------------------------------------------------------- RNG
// Philox4x32-10 (Salmon et al., SC'11): counter-based, so the backward pass regenerates the
// forward dropout mask from (seed, offset, element index) instead of storing it.
// Timing-only diagnostic builds (scripts/build_variant.sh with DNA_AMD_FILE_FLAGS): DNA_DBG_EPI
// bit 0 replaces erf by the identity, DNA_PHILOX_ROUNDS changes the round count. Never set in
// the product build (results change).
#ifndef DNA_DBG_EPI
#define DNA_DBG_EPI 0
#endif
#ifndef DNA_PHILOX_ROUNDS
#define DNA_PHILOX_ROUNDS 10
#endif
struct Philox {
  template <int R = DNA_PHILOX_ROUNDS>
  __device__ __forceinline__ static uint4 gen(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3,
                                              uint32_t k0, uint32_t k1) {
    // each round's two 32x32 -> 64-bit products as one 64-bit multiply apiece (the pair
    // v_mul_hi_u32 + v_mul_lo_u32 per product otherwise; same bits either way)
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const uint64_t p0 = (uint64_t)0xD2511F53u * c0, p1 = (uint64_t)0xCD9E8D57u * c2;
      const uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
      const uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
      uint32_t n0 = hi1 ^ c1 ^ k0, n2 = hi0 ^ c3 ^ k1;
      c0 = n0; c1 = lo1; c2 = n2; c3 = lo0;
      k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
    }
    return make_uint4(c0, c1, c2, c3);
  }
};

// Keep-mask for 4 consecutive elements starting at element index `idx4 * 4`.
// An element is kept when its 32-bit uniform is >= p * 2^32.
__device__ __forceinline__ uint32_t dropout_keep4(uint64_t seed, uint64_t offset, uint64_t idx4,
                                                  uint32_t thresh) {
  uint64_t c = idx4 + offset;
  uint4 r = Philox::gen((uint32_t)c, (uint32_t)(c >> 32), 0x5EEDu, 0u, (uint32_t)seed,
                        (uint32_t)(seed >> 32));
  return (r.x >= thresh ? 1u : 0u) | (r.y >= thresh ? 2u : 0u) | (r.z >= thresh ? 4u : 0u) |
         (r.w >= thresh ? 8u : 0u);
}

// Keep-mask for 8 consecutive elements starting at element index `idx8 * 8`: one Philox call,
// element j uses the 16-bit half j of the 128-bit draw and is kept when it is >= p * 2^16
// (keep probability quantised to 1/65536: p = 0.1 -> 0.099991). Half the Philox work of
// two dropout_keep4 calls. Philox4x32 with 7 rounds: Salmon et al. (SC'11) find 7 rounds of
// Philox4x32 pass TestU01's BigCrush (10 is Random123's default safety margin); the draws sit in
// the GeGLU GEMM epilogue's VALU budget (geglu_epi_ab.py: 10 -> 7 rounds -0.03 ms per launch).
// The draw itself: element j of the group keeps iff its 16-bit half (r[j / 2] >> 16 * (j & 1)) &
// 0xFFFF is >= thresh16 (dropout_kept8).
__device__ __forceinline__ uint4 dropout_draw8(uint64_t seed, uint64_t offset, uint64_t idx8) {
  const uint64_t c = idx8 + offset;
  return Philox::gen<7>((uint32_t)c, (uint32_t)(c >> 32), 0x5EED8u, 0u, (uint32_t)seed,
                        (uint32_t)(seed >> 32));
}
__device__ __forceinline__ bool dropout_kept8(const uint4& r, int j, uint32_t thresh16) {
  const uint32_t w = j < 2 ? r.x : j < 4 ? r.y : j < 6 ? r.z : r.w;
  return ((j & 1) ? (w >> 16) : (w & 0xFFFFu)) >= thresh16;
}
__device__ __forceinline__ uint32_t dropout_keep8(uint64_t seed, uint64_t offset, uint64_t idx8,
                                                  uint32_t thresh16) {
  const uint4 r = dropout_draw8(seed, offset, idx8);
  const uint32_t w[4] = {r.x, r.y, r.z, r.w};
  uint32_t m = 0;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    m |= ((w[j] & 0xFFFFu) >= thresh16 ? 1u : 0u) << (2 * j);
    m |= ((w[j] >> 16) >= thresh16 ? 1u : 0u) << (2 * j + 1);
  }
  return m;
}

__host__ __device__ __forceinline__ uint32_t dropout_threshold16(float p) {
  return (uint32_t)((double)p * 65536.0);  // p < 1 -> <= 65535
}

__host__ __device__ __forceinline__ uint32_t dropout_threshold(float p) {
  double t = (double)p * 4294967296.0;
  return t >= 4294967295.0 ? 0xFFFFFFFFu : (uint32_t)t;
}

// ---------------------------------------------------------------------------------------- math
// erf(z), branchless (Abramowitz & Stegun 7.1.26: |error| < 1.5e-7 in exact arithmetic,
// < 6e-7 evaluated in fp32), with e = exp(-z^2) as a by-product: one v_rcp, one v_exp, 5 FMAs.
// The OCML erff it replaces branches on |z| per element (divergent, both paths run) and was the
// largest VALU cost of the GeGLU kernels. GELU from it: |error| < 5e-7 on [-10, 10] (checked
// against math.erf), below bf16 resolution of every tensor it feeds.
__device__ __forceinline__ float erf_fast(float z, float& e) {
  if constexpr (DNA_DBG_EPI & 1) {
    e = z;
    return z;
  }
  const float az = fabsf(z);
  const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f, az, 1.f));
  float p = fmaf(1.061405429f, t, -1.453152027f);
  p = fmaf(p, t, 1.421413741f);
  p = fmaf(p, t, -0.284496736f);
  p = fmaf(p, t, 0.254829592f);
  p *= t;
  // z * z, not |z| * |z| (same bits): no abs modifier, so the compiler pairs it into v_pk_mul
  e = __builtin_amdgcn_exp2f(z * z * -1.4426950408889634f);
  return copysignf(fmaf(-p, e, 1.f), z);
}
__device__ __forceinline__ float gelu_erf(float x) {
  float e;
  return 0.5f * x * (1.0f + erf_fast(x * 0.70710678118654752f, e));
}
// GELU(x) and its derivative Phi(x) + x phi(x), sharing one erf / exp
__device__ __forceinline__ void gelu_erf_and_grad(float x, float& g, float& dg) {
  float e;
  const float cdf = fmaf(0.5f, erf_fast(x * 0.70710678118654752f, e), 0.5f);  // one v_pk_fma
  g = x * cdf;
  dg = fmaf(x * 0.3989422804014327f, e, cdf);  // e = exp(-x^2 / 2)
}
// GeGLU forward and its backward factors (bert_layers.py:292-296), for h1 = g[:, :F], h2 =
// g[:, F:] (the bf16-rounded gated_layers outputs), the element's dropout keep bit and
// ks = 1 / (1 - p) (p = 0: kept, ks = 1):
//   s    = kept ? ks : 0
//   fac2 = gelu(h1) s                    (= d a / d h2)
//   a    = fac2 h2
//   fac1 = gelu'(h1) s h2                (= d a / d h1)
// The forward stores fac = [fac1 | fac2] where g would have gone (same bytes), so the backward is
// dg = da * fac: no erf and no keep-bit draws there (csrc/gemm.hip, csrc/geglu.hip).
__device__ __forceinline__ void geglu_fwd_fac(float h1, float h2, bool kept, float ks, float& a,
                                              float& f1, float& f2) {
  float ge, dge;
  gelu_erf_and_grad(h1, ge, dge);
  const float s = kept ? ks : 0.f;
  f2 = ge * s;
  a = f2 * h2;
  f1 = dge * s * h2;
}

// tanh(u) = 1 - 2 / (exp(2u) + 1): one v_exp + one v_rcp, branch-free (OCML tanhf branches on
// |u| -- divergent, both paths run -- and was most of EPI_GELU_BWD's epilogue); |error| < 2e-7
// absolute, saturating to +-1 for large |u| (exp -> inf / 0)
__device__ __forceinline__ float tanh_fast(float u) {
  return 1.f - 2.f * __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(u * 2.8853900817779268f));
}
// the tanh-approximation GELU 0.5 x (1 + tanh(u)), u = k (x + 0.044715 x^3), k = sqrt(2/pi),
// as x / (1 + exp(-2u)) (the same function; no cancellation in 1 + tanh(u) for u << 0, where
// torch's fp32 form rounds to 0 and this one keeps the tiny tail): one v_exp + one v_rcp
__device__ __forceinline__ float gelu_tanh(float x) {
  const float kBeta = 0.7978845608028654f, kKappa = 0.044715f;
  const float x_cube = x * x * x;
  const float inner = kBeta * (x + kKappa * x_cube);
  return x * __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(inner * -2.8853900817779268f));
}
// d/dx of gelu_tanh, in the operation order of torch's GeluBackward (approximate="tanh")
__device__ __forceinline__ float gelu_tanh_grad(float x) {
  const float kBeta = 0.7978845608028654f, kKappa = 0.044715f;
  const float x_sq = x * x, x_cube = x_sq * x;
  const float inner = kBeta * (x + kKappa * x_cube);
  const float t = tanh_fast(inner);
  const float left = 0.5f * x, right = 1.f + t;
  const float left_derivative = 0.5f * right;
  const float right_derivative = left * (1.f - t * t) * kBeta * (1.f + 3.f * kKappa * x_sq);
  return left_derivative + right_derivative;
}
__device__ __forceinline__ float gelu_erf_grad(float x) {
  float g, dg;
  gelu_erf_and_grad(x, g, dg);
  return dg;
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

}  // namespace dna
