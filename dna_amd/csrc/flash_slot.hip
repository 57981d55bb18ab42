// The flash_attn_qkvpacked_func kernel slot with the reference's full signature
// (src/models/sequence/flash_attn_triton.py:1077-1130, called at bert_layers.py:188/192 as
// flash_attn_qkvpacked_func(qkv, bias)): softmax(q k^T * scale + bias) v over packed
// qkv [b, S, 3, H, D] (bf16 or fp16), with
//   bias  none | "vector" [., ., 1, S] | "matrix" [., ., S, S], fp32 or the qkv dtype, any of its
//         batch / head dims broadcast (stride 0), streamed tile by tile (never materialised here);
//   causal  key > query masked (flash_attn_triton.py:212-214);
//   scale   qk * scale + bias, then softmax (:215-223); default 1/sqrt(D).
// Outputs out [b, S, H, D] and lse [b, H, ceil(S/128)*128] (natural log, as the Triton kernel).
// Backward returns dqkv only (the reference asserts no bias gradient, :1109-1110): delta =
// rowsum(dO*O), then a dK/dV kernel (keys on the workgroup, query tiles streamed) and a dQ kernel
// (queries on the workgroup, key tiles streamed), both recomputing P from the LSE -- no atomics,
// deterministic.
//
// This is the generic slot; DNABERT-2's own forward uses the ALiBi/pad fast path of
// attention.hip, which never reads an [b,H,S,S] bias. Layout per workgroup: 4 waves x 16 rows
// (queries or keys) = 64 rows; the streamed dimension in tiles of 64 through LDS (rows padded to
// 2D+16 bytes: row reads by 16 lanes of consecutive rows are conflict-free); MFMA
// v_mfma_f32_16x16x32_{bf16,f16}; P / dS pass from the accumulator layout to an A operand
// through a per-wave LDS image; the column-direction operands (V, dO, Q, K) come from
// ds_read_b64_tr_b16 transposed reads of the row-major tiles. A matrix bias is staged through LDS
// one 64 x 64 tile per (query block, key block) with 16-B loads (stage_bias).
#include <stdlib.h>

#include "common.h"

namespace dna {
namespace fa {

typedef _Float16 f16;
typedef __attribute__((ext_vector_type(8))) _Float16 f16x8;
typedef __attribute__((ext_vector_type(4))) short s16x4;
typedef __attribute__((ext_vector_type(8))) short s16x8;
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

constexpr int NT = 256;  // 4 waves
constexpr int BR = 64;   // rows per workgroup (16 per wave) and rows per streamed tile
constexpr float LOG2E = 1.4426950408889634f;

template <typename T> struct Mf;
template <> struct Mf<bf16> {
  using v8 = bf16x8;
  static __device__ __forceinline__ f32x4 mma(v8 a, v8 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
  }
  static __device__ __forceinline__ unsigned short bits(float x) {
    return __builtin_bit_cast(unsigned short, (bf16)x);
  }
  static __device__ __forceinline__ float val(unsigned short u) {
    return (float)__builtin_bit_cast(bf16, u);
  }
};
template <> struct Mf<f16> {
  using v8 = f16x8;
  static __device__ __forceinline__ f32x4 mma(v8 a, v8 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
  }
  static __device__ __forceinline__ unsigned short bits(float x) {
    return __builtin_bit_cast(unsigned short, (f16)x);
  }
  static __device__ __forceinline__ float val(unsigned short u) {
    return (float)__builtin_bit_cast(f16, u);
  }
};

struct Args {
  const unsigned short* qkv;  // [b, S, 3, H, D]
  const void* bias;           // null | [b?, H?, 1|S, S] with element strides sb, sh, sq
  long long sb, sh, sq;
  int bias_f32;               // 1: fp32 bias, 0: qkv dtype
  const unsigned short* out;  // [b, S, H, D] (forward output; read by the backward)
  const unsigned short* dout; // [b, S, H, D]
  unsigned short* o;          // forward: out;  backward: dqkv [b, S, 3, H, D]
  float* lse;                 // [b, H, Sr]
  float* delta;               // [b, H, Sr] (backward)
  int B, S, H, Sr, causal;
  float scale;
};

// padded row stride (bytes) of a [64][D] 16-bit tile image
template <int D> __host__ __device__ constexpr int rs() { return 2 * D + 16; }
constexpr int PRS = 2 * BR + 16;  // [16][64] P / dS image row stride

// rows r0..r0+63 of a [rows][D] operand (row stride ld elements, rows >= nrows -> 0) into LDS
template <int D>
__device__ __forceinline__ void load_tile(char* lds, const unsigned short* g, long long ld, int r0,
                                          int nrows, int tid) {
  constexpr int CPR = D / 8;
#pragma unroll
  for (int c = tid; c < BR * CPR; c += NT) {
    const int r = c / CPR, ch = c - r * CPR;
    uint4 v = make_uint4(0u, 0u, 0u, 0u);
    if (r0 + r < nrows) v = *reinterpret_cast<const uint4*>(g + (long long)(r0 + r) * ld + ch * 8);
    *reinterpret_cast<uint4*>(lds + r * rs<D>() + ch * 16) = v;
  }
}

// 8 consecutive elements of one row (an MFMA operand in row form)
template <typename V8>
__device__ __forceinline__ V8 row8(const char* lds, int stride, int row, int col) {
  return *reinterpret_cast<const V8*>(lds + row * stride + col * 2);
}

// column c0 + (lane&15) of rows kbase + 8*(lane>>4) + 0..7 (an MFMA B operand read from a
// row-major tile): two ds_read_b64_tr_b16, each delivering one 4-row x 16-column block
template <typename V8>
__device__ __forceinline__ V8 col8(const char* lds, int stride, int kbase, int c0, int lane) {
  const int i = lane & 15, g = lane >> 4;
  const char* p = lds + (kbase + 8 * g + (i >> 2)) * stride + (c0 + 4 * (i & 3)) * 2;
  const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(p));
  const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(p + 4 * stride));
  return __builtin_bit_cast(V8, s16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]});
}

// bias(q, k) (0 outside [0, S)), bias type BT: 1 vector, 2 matrix; fp32 or the qkv dtype
template <typename T, int BT>
__device__ __forceinline__ float bias_v(const Args& a, long long base, int q, int k) {
  if constexpr (BT == 0) {
    return 0.f;
  } else {
    if (q >= a.S || k >= a.S) return 0.f;
    const long long off = base + (BT >= 2 ? (long long)q * a.sq : 0) + k;
    return a.bias_f32 ? reinterpret_cast<const float*>(a.bias)[off]
                      : Mf<T>::val(reinterpret_cast<const unsigned short*>(a.bias)[off]);
  }
}

// Matrix bias staged through LDS (BT == 3: a [b?, H?, S, S] bias whose base and strides keep every
// row 16-B aligned): the 64 x 64 tile of the (query block, key block) pair is read with 16-B loads,
// converted to fp32 and kept at row stride BLD = 68 floats (rows 4 apart sit 16 banks apart, so
// every score read -- 16 consecutive columns x 4 row groups -- is conflict-free). TR stores it
// [key][query] for the dK/dV kernel, whose lanes walk queries. Out-of-range entries are 0.
constexpr int BLD = 68;
constexpr int BIAS_TILE = BR * BLD * 4;  // bytes
template <typename T, bool TR>
__device__ __forceinline__ void stage_bias(float* t, const Args& a, long long base, int q0, int k0,
                                           int tid) {
  auto put = [&](int qq, int kk, const float (&v)[8], int n) {
    if constexpr (TR) {
#pragma unroll
      for (int e = 0; e < 8; ++e)
        if (e < n) t[(kk + e) * BLD + qq] = v[e];
    } else {
      *reinterpret_cast<f32x4*>(t + qq * BLD + kk) = f32x4{v[0], v[1], v[2], v[3]};
      if (n == 8) *reinterpret_cast<f32x4*>(t + qq * BLD + kk + 4) = f32x4{v[4], v[5], v[6], v[7]};
    }
  };
  if (a.bias_f32) {
    const float* B = reinterpret_cast<const float*>(a.bias);
    for (int c = tid; c < BR * 16; c += NT) {  // 16 chunks of 4 per row
      const int qq = c >> 4, kk = (c & 15) * 4, q = q0 + qq, k = k0 + kk;
      float v[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      if (q < a.S) {
        const float* p = B + base + (long long)q * a.sq + k;
        if (k + 3 < a.S) {
          const f32x4 x = *reinterpret_cast<const f32x4*>(p);
          v[0] = x[0]; v[1] = x[1]; v[2] = x[2]; v[3] = x[3];
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] = k + e < a.S ? p[e] : 0.f;
        }
      }
      put(qq, kk, v, 4);
    }
  } else {
    const unsigned short* B = reinterpret_cast<const unsigned short*>(a.bias);
    for (int c = tid; c < BR * 8; c += NT) {  // 8 chunks of 8 per row
      const int qq = c >> 3, kk = (c & 7) * 8, q = q0 + qq, k = k0 + kk;
      float v[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      if (q < a.S) {
        const unsigned short* p = B + base + (long long)q * a.sq + k;
        if (k + 7 < a.S) {
          const uint4 x = *reinterpret_cast<const uint4*>(p);
          const unsigned short* h = reinterpret_cast<const unsigned short*>(&x);
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] = Mf<T>::val(h[e]);
        } else {
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] = k + e < a.S ? Mf<T>::val(p[e]) : 0.f;
        }
      }
      put(qq, kk, v, 8);
    }
  }
}

// reductions over the 16 lanes that share lane >> 4 (one accumulator row group)
__device__ __forceinline__ float max16(float v) {
#pragma unroll
  for (int o = 1; o < 16; o <<= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}
__device__ __forceinline__ float sum16(float v) {
#pragma unroll
  for (int o = 1; o < 16; o <<= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// ------------------------------------------------------------------------------- forward
template <typename T, int D, int BT>
__global__ __launch_bounds__(NT) void fwd_kernel(Args a) {
  using V8 = typename Mf<T>::v8;
  constexpr int KK = D / 32, NTL = D / 16;
  __shared__ __attribute__((aligned(16))) char smem[2 * BR * rs<D>() + 4 * 16 * PRS + (BT == 3 ? BIAS_TILE : 0)];
  char* Kt = smem;
  char* Vt = smem + BR * rs<D>();
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  char* Pw = smem + 2 * BR * rs<D>() + w * 16 * PRS;
  float* btile = reinterpret_cast<float*>(smem + 2 * BR * rs<D>() + 4 * 16 * PRS);
  const int bh = blockIdx.y, b = bh / a.H, h = bh - b * a.H;
  const int q0 = blockIdx.x * BR;
  const long long HD = (long long)a.H * D, ld = 3 * HD;
  const unsigned short* qg = a.qkv + (long long)b * a.S * ld + h * D;
  const long long bbase = (long long)b * a.sb + (long long)h * a.sh;
  const float sl2 = a.scale * LOG2E;

  V8 qf[KK];
  {
    const int q = q0 + w * 16 + (lane & 15);
#pragma unroll
    for (int kk = 0; kk < KK; ++kk) {
      uint4 v = make_uint4(0u, 0u, 0u, 0u);
      if (q < a.S) v = *reinterpret_cast<const uint4*>(qg + (long long)q * ld + 32 * kk + 8 * (lane >> 4));
      qf[kk] = __builtin_bit_cast(V8, v);
    }
  }
  f32x4 oacc[NTL];
#pragma unroll
  for (int t = 0; t < NTL; ++t) oacc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
  float m[4], l[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) { m[r] = -1e30f; l[r] = 0.f; }
  const int qrow = q0 + w * 16 + 4 * (lane >> 4);  // + r: this lane's accumulator rows

  const int nkt = (a.S + BR - 1) / BR;
  const int kend = a.causal ? min(nkt, q0 / BR + 1) : nkt;
  for (int kt = 0; kt < kend; ++kt) {
    const int k0 = kt * BR;
    __syncthreads();
    load_tile<D>(Kt, qg + HD, ld, k0, a.S, tid);
    load_tile<D>(Vt, qg + 2 * HD, ld, k0, a.S, tid);
    if constexpr (BT == 3) stage_bias<T, false>(btile, a, bbase, q0, k0, tid);
    __syncthreads();
    f32x4 s[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      s[j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kk = 0; kk < KK; ++kk)
        s[j] = Mf<T>::mma(qf[kk], row8<V8>(Kt, rs<D>(), 16 * j + (lane & 15), 32 * kk + 8 * (lane >> 4)), s[j]);
    }
    // s[j][r] = S[query qrow + r][key k0 + 16j + (lane & 15)]  (log2 units below)
    float mx[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) mx[r] = -1e30f;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int k = k0 + 16 * j + (lane & 15);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int q = qrow + r;
        const float bv = BT == 3 ? btile[(q - q0) * BLD + (k - k0)] : bias_v<T, BT>(a, bbase, q, k);
        float x = s[j][r] * sl2 + bv * LOG2E;
        if (k >= a.S || (a.causal && k > q)) x = -INFINITY;
        s[j][r] = x;
        mx[r] = fmaxf(mx[r], x);
      }
    }
    float alpha[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float mn = fmaxf(m[r], max16(mx[r]));
      alpha[r] = exp2f(m[r] - mn);
      m[r] = mn;
    }
    float rsum[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float p = exp2f(s[j][r] - m[r]);
        rsum[r] += p;
        *reinterpret_cast<unsigned short*>(Pw + (4 * (lane >> 4) + r) * PRS + (16 * j + (lane & 15)) * 2) =
            Mf<T>::bits(p);
      }
#pragma unroll
    for (int r = 0; r < 4; ++r) l[r] = l[r] * alpha[r] + sum16(rsum[r]);
#pragma unroll
    for (int t = 0; t < NTL; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) oacc[t][r] *= alpha[r];
    __syncthreads();  // P image complete (and K reads retired)
#pragma unroll
    for (int kk2 = 0; kk2 < 2; ++kk2) {
      const V8 pa = row8<V8>(Pw, PRS, lane & 15, 32 * kk2 + 8 * (lane >> 4));
#pragma unroll
      for (int t = 0; t < NTL; ++t) oacc[t] = Mf<T>::mma(pa, col8<V8>(Vt, rs<D>(), 32 * kk2, 16 * t, lane), oacc[t]);
    }
  }
  // epilogue: O / l through an LDS row image (16-B stores), LSE = (m + log2 l) / log2 e
  __syncthreads();
  char* Ow = smem + w * 16 * rs<D>();
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const float inv = l[r] > 0.f ? 1.f / l[r] : 0.f;
#pragma unroll
    for (int t = 0; t < NTL; ++t)
      *reinterpret_cast<unsigned short*>(Ow + (4 * (lane >> 4) + r) * rs<D>() + (16 * t + (lane & 15)) * 2) =
          Mf<T>::bits(oacc[t][r] * inv);
    const int q = qrow + r;
    if ((lane & 15) == 0 && q < a.S)
      a.lse[(long long)bh * a.Sr + q] = (m[r] + __log2f(l[r])) * 0.6931471805599453f;
  }
  __syncthreads();
  constexpr int CPR = D / 8;
  for (int c = lane; c < 16 * CPR; c += 64) {
    const int r = c / CPR, ch = c - r * CPR;
    const int q = q0 + w * 16 + r;
    if (q < a.S)
      *reinterpret_cast<uint4*>(a.o + ((long long)b * a.S + q) * HD + h * D + ch * 8) =
          *reinterpret_cast<const uint4*>(Ow + r * rs<D>() + ch * 16);
  }
}

// ------------------------------------------------------------------------------- delta
template <typename T, int D>
__global__ void delta_kernel(Args a) {
  const long long idx = (long long)blockIdx.x * blockDim.x + threadIdx.x;  // (b, s, h)
  if (idx >= (long long)a.B * a.S * a.H) return;
  const int h = (int)(idx % a.H);
  const long long bs = idx / a.H;
  const int s = (int)(bs % a.S), b = (int)(bs / a.S);
  const unsigned short* o = a.out + idx * D;
  const unsigned short* g = a.dout + idx * D;
  float acc = 0.f;
#pragma unroll
  for (int c = 0; c < D; c += 8) {
    const s16x8 ov = *reinterpret_cast<const s16x8*>(o + c), gv = *reinterpret_cast<const s16x8*>(g + c);
#pragma unroll
    for (int e = 0; e < 8; ++e) acc = fmaf(Mf<T>::val((unsigned short)ov[e]), Mf<T>::val((unsigned short)gv[e]), acc);
  }
  a.delta[((long long)b * a.H + h) * a.Sr + s] = acc;
}

// ------------------------------------------------------------------------------- dK, dV
template <typename T, int D, int BT>
__global__ __launch_bounds__(NT) void dkdv_kernel(Args a) {
  using V8 = typename Mf<T>::v8;
  constexpr int KK = D / 32, NTL = D / 16;
  __shared__ __attribute__((aligned(16))) char smem[2 * BR * rs<D>() + 8 * 16 * PRS + 2 * BR * 4 + (BT == 3 ? BIAS_TILE : 0)];
  float* btile = reinterpret_cast<float*>(smem + 2 * BR * rs<D>() + 8 * 16 * PRS + 2 * BR * 4);
  char* Qt = smem;
  char* Gt = smem + BR * rs<D>();  // dO tile
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  char* Pw = smem + 2 * BR * rs<D>() + w * 16 * PRS;
  char* Sw = smem + 2 * BR * rs<D>() + (4 + w) * 16 * PRS;
  float* lse_t = reinterpret_cast<float*>(smem + 2 * BR * rs<D>() + 8 * 16 * PRS);
  float* del_t = lse_t + BR;
  const int bh = blockIdx.y, b = bh / a.H, h = bh - b * a.H;
  const int k0 = blockIdx.x * BR;
  const long long HD = (long long)a.H * D, ld = 3 * HD;
  const unsigned short* qg = a.qkv + (long long)b * a.S * ld + h * D;
  const unsigned short* gg = a.dout + (long long)b * a.S * HD + h * D;
  const long long bbase = (long long)b * a.sb + (long long)h * a.sh;
  const float sl2 = a.scale * LOG2E;

  V8 kf[KK], vf[KK];
  {
    const int k = k0 + w * 16 + (lane & 15);
#pragma unroll
    for (int kk = 0; kk < KK; ++kk) {
      uint4 kv = make_uint4(0u, 0u, 0u, 0u), vv = kv;
      if (k < a.S) {
        kv = *reinterpret_cast<const uint4*>(qg + (long long)k * ld + HD + 32 * kk + 8 * (lane >> 4));
        vv = *reinterpret_cast<const uint4*>(qg + (long long)k * ld + 2 * HD + 32 * kk + 8 * (lane >> 4));
      }
      kf[kk] = __builtin_bit_cast(V8, kv);
      vf[kk] = __builtin_bit_cast(V8, vv);
    }
  }
  f32x4 dk[NTL], dv[NTL];
#pragma unroll
  for (int t = 0; t < NTL; ++t) { dk[t] = f32x4{0.f, 0.f, 0.f, 0.f}; dv[t] = dk[t]; }
  const int krow = k0 + w * 16 + 4 * (lane >> 4);  // + r

  const int nqt = (a.S + BR - 1) / BR;
  for (int qt = a.causal ? k0 / BR : 0; qt < nqt; ++qt) {
    const int q0 = qt * BR;
    __syncthreads();
    load_tile<D>(Qt, qg, ld, q0, a.S, tid);
    load_tile<D>(Gt, gg, HD, q0, a.S, tid);
    if constexpr (BT == 3) stage_bias<T, true>(btile, a, bbase, q0, k0, tid);
    if (tid < BR) {
      const int q = q0 + tid;
      lse_t[tid] = q < a.S ? a.lse[(long long)bh * a.Sr + q] * LOG2E : INFINITY;
      del_t[tid] = q < a.S ? a.delta[(long long)bh * a.Sr + q] : 0.f;
    }
    __syncthreads();
    f32x4 s[4], dp[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      s[j] = f32x4{0.f, 0.f, 0.f, 0.f};
      dp[j] = s[j];
#pragma unroll
      for (int kk = 0; kk < KK; ++kk) {
        const int rr = 16 * j + (lane & 15), cc = 32 * kk + 8 * (lane >> 4);
        s[j] = Mf<T>::mma(kf[kk], row8<V8>(Qt, rs<D>(), rr, cc), s[j]);
        dp[j] = Mf<T>::mma(vf[kk], row8<V8>(Gt, rs<D>(), rr, cc), dp[j]);
      }
    }
    // s[j][r] = S^T[key krow + r][query q0 + 16j + (lane&15)]
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int ql = 16 * j + (lane & 15), q = q0 + ql;
      const float lq = lse_t[ql], dq = del_t[ql];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int k = krow + r;
        const float bv = BT == 3 ? btile[(k - k0) * BLD + ql] : bias_v<T, BT>(a, bbase, q, k);
        float p = exp2f(s[j][r] * sl2 + bv * LOG2E - lq);
        if (a.causal && k > q) p = 0.f;
        const float ds = p * (dp[j][r] - dq) * a.scale;
        const int off = (4 * (lane >> 4) + r) * PRS + ql * 2;
        *reinterpret_cast<unsigned short*>(Pw + off) = Mf<T>::bits(p);
        *reinterpret_cast<unsigned short*>(Sw + off) = Mf<T>::bits(ds);
      }
    }
    __syncthreads();
#pragma unroll
    for (int kk2 = 0; kk2 < 2; ++kk2) {
      const V8 pa = row8<V8>(Pw, PRS, lane & 15, 32 * kk2 + 8 * (lane >> 4));
      const V8 sa = row8<V8>(Sw, PRS, lane & 15, 32 * kk2 + 8 * (lane >> 4));
#pragma unroll
      for (int t = 0; t < NTL; ++t) {
        dv[t] = Mf<T>::mma(pa, col8<V8>(Gt, rs<D>(), 32 * kk2, 16 * t, lane), dv[t]);
        dk[t] = Mf<T>::mma(sa, col8<V8>(Qt, rs<D>(), 32 * kk2, 16 * t, lane), dk[t]);
      }
    }
  }
  // epilogue: dK, dV rows (dqkv slots 1, 2) through LDS row images, 16-B stores
  __syncthreads();
  char* Kw = smem + w * 16 * rs<D>();
  char* Vw = smem + (4 + w) * 16 * rs<D>();
#pragma unroll
  for (int r = 0; r < 4; ++r)
#pragma unroll
    for (int t = 0; t < NTL; ++t) {
      const int off = (4 * (lane >> 4) + r) * rs<D>() + (16 * t + (lane & 15)) * 2;
      *reinterpret_cast<unsigned short*>(Kw + off) = Mf<T>::bits(dk[t][r]);
      *reinterpret_cast<unsigned short*>(Vw + off) = Mf<T>::bits(dv[t][r]);
    }
  __syncthreads();
  constexpr int CPR = D / 8;
  for (int c = lane; c < 16 * CPR; c += 64) {
    const int r = c / CPR, ch = c - r * CPR;
    const int k = k0 + w * 16 + r;
    if (k < a.S) {
      unsigned short* dst = a.o + ((long long)b * a.S + k) * ld + h * D + ch * 8;
      *reinterpret_cast<uint4*>(dst + HD) = *reinterpret_cast<const uint4*>(Kw + r * rs<D>() + ch * 16);
      *reinterpret_cast<uint4*>(dst + 2 * HD) = *reinterpret_cast<const uint4*>(Vw + r * rs<D>() + ch * 16);
    }
  }
}

// ------------------------------------------------------------------------------- dQ
template <typename T, int D, int BT>
__global__ __launch_bounds__(NT) void dq_kernel(Args a) {
  using V8 = typename Mf<T>::v8;
  constexpr int KK = D / 32, NTL = D / 16;
  __shared__ __attribute__((aligned(16))) char smem[2 * BR * rs<D>() + 4 * 16 * PRS + (BT == 3 ? BIAS_TILE : 0)];
  char* Kt = smem;
  char* Vt = smem + BR * rs<D>();
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  char* Sw = smem + 2 * BR * rs<D>() + w * 16 * PRS;
  float* btile = reinterpret_cast<float*>(smem + 2 * BR * rs<D>() + 4 * 16 * PRS);
  const int bh = blockIdx.y, b = bh / a.H, h = bh - b * a.H;
  const int q0 = blockIdx.x * BR;
  const long long HD = (long long)a.H * D, ld = 3 * HD;
  const unsigned short* qg = a.qkv + (long long)b * a.S * ld + h * D;
  const unsigned short* gg = a.dout + (long long)b * a.S * HD + h * D;
  const long long bbase = (long long)b * a.sb + (long long)h * a.sh;
  const float sl2 = a.scale * LOG2E;

  V8 qf[KK], gf[KK];
  {
    const int q = q0 + w * 16 + (lane & 15);
#pragma unroll
    for (int kk = 0; kk < KK; ++kk) {
      uint4 qv = make_uint4(0u, 0u, 0u, 0u), gv = qv;
      if (q < a.S) {
        qv = *reinterpret_cast<const uint4*>(qg + (long long)q * ld + 32 * kk + 8 * (lane >> 4));
        gv = *reinterpret_cast<const uint4*>(gg + (long long)q * HD + 32 * kk + 8 * (lane >> 4));
      }
      qf[kk] = __builtin_bit_cast(V8, qv);
      gf[kk] = __builtin_bit_cast(V8, gv);
    }
  }
  const int qrow = q0 + w * 16 + 4 * (lane >> 4);  // + r
  float lq[4], dq_[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int q = qrow + r;
    lq[r] = q < a.S ? a.lse[(long long)bh * a.Sr + q] * LOG2E : INFINITY;
    dq_[r] = q < a.S ? a.delta[(long long)bh * a.Sr + q] : 0.f;
  }
  f32x4 dq[NTL];
#pragma unroll
  for (int t = 0; t < NTL; ++t) dq[t] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nkt = (a.S + BR - 1) / BR;
  const int kend = a.causal ? min(nkt, q0 / BR + 1) : nkt;
  for (int kt = 0; kt < kend; ++kt) {
    const int k0 = kt * BR;
    __syncthreads();
    load_tile<D>(Kt, qg + HD, ld, k0, a.S, tid);
    load_tile<D>(Vt, qg + 2 * HD, ld, k0, a.S, tid);
    if constexpr (BT == 3) stage_bias<T, false>(btile, a, bbase, q0, k0, tid);
    __syncthreads();
    f32x4 s[4], dp[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      s[j] = f32x4{0.f, 0.f, 0.f, 0.f};
      dp[j] = s[j];
#pragma unroll
      for (int kk = 0; kk < KK; ++kk) {
        const int rr = 16 * j + (lane & 15), cc = 32 * kk + 8 * (lane >> 4);
        s[j] = Mf<T>::mma(qf[kk], row8<V8>(Kt, rs<D>(), rr, cc), s[j]);
        dp[j] = Mf<T>::mma(gf[kk], row8<V8>(Vt, rs<D>(), rr, cc), dp[j]);
      }
    }
    // s[j][r] = S[query qrow + r][key k0 + 16j + (lane&15)]
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int kl = 16 * j + (lane & 15), k = k0 + kl;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int q = qrow + r;
        const float bv = BT == 3 ? btile[(q - q0) * BLD + kl] : bias_v<T, BT>(a, bbase, q, k);
        float p = exp2f(s[j][r] * sl2 + bv * LOG2E - lq[r]);
        if (k >= a.S || (a.causal && k > q)) p = 0.f;
        *reinterpret_cast<unsigned short*>(Sw + (4 * (lane >> 4) + r) * PRS + kl * 2) =
            Mf<T>::bits(p * (dp[j][r] - dq_[r]) * a.scale);
      }
    }
    __syncthreads();
#pragma unroll
    for (int kk2 = 0; kk2 < 2; ++kk2) {
      const V8 sa = row8<V8>(Sw, PRS, lane & 15, 32 * kk2 + 8 * (lane >> 4));
#pragma unroll
      for (int t = 0; t < NTL; ++t) dq[t] = Mf<T>::mma(sa, col8<V8>(Kt, rs<D>(), 32 * kk2, 16 * t, lane), dq[t]);
    }
  }
  __syncthreads();
  char* Qw = smem + w * 16 * rs<D>();
#pragma unroll
  for (int r = 0; r < 4; ++r)
#pragma unroll
    for (int t = 0; t < NTL; ++t)
      *reinterpret_cast<unsigned short*>(Qw + (4 * (lane >> 4) + r) * rs<D>() + (16 * t + (lane & 15)) * 2) =
          Mf<T>::bits(dq[t][r]);
  __syncthreads();
  constexpr int CPR = D / 8;
  for (int c = lane; c < 16 * CPR; c += 64) {
    const int r = c / CPR, ch = c - r * CPR;
    const int q = q0 + w * 16 + r;
    if (q < a.S)
      *reinterpret_cast<uint4*>(a.o + ((long long)b * a.S + q) * ld + h * D + ch * 8) =
          *reinterpret_cast<const uint4*>(Qw + r * rs<D>() + ch * 16);
  }
}

// ------------------------------------------------------------------------------- dispatch
template <typename T, int D>
int run(bool bwd, const Args& a, int bias_type, hipStream_t s) {
  const dim3 grid((a.S + BR - 1) / BR, a.B * a.H);
  // a matrix bias whose rows all start 16-B aligned is staged tile by tile through LDS (BT 3);
  // DNA_FLASH_BIAS_DIRECT=1 keeps the per-score global reads (A/B)
  if (bias_type == 2) {
    const long long vec = a.bias_f32 ? 4 : 8;
    const char* e = getenv("DNA_FLASH_BIAS_DIRECT");
    if (((uintptr_t)a.bias & 15) == 0 && a.sb % vec == 0 && a.sh % vec == 0 && a.sq % vec == 0 &&
        !(e && e[0] == '1'))
      bias_type = 3;
  }
  if (!bwd) {
    if (bias_type == 0) hipLaunchKernelGGL((fwd_kernel<T, D, 0>), grid, dim3(NT), 0, s, a);
    else if (bias_type == 1) hipLaunchKernelGGL((fwd_kernel<T, D, 1>), grid, dim3(NT), 0, s, a);
    else if (bias_type == 3) hipLaunchKernelGGL((fwd_kernel<T, D, 3>), grid, dim3(NT), 0, s, a);
    else hipLaunchKernelGGL((fwd_kernel<T, D, 2>), grid, dim3(NT), 0, s, a);
    return DNA_OK;
  }
  const long long rows = (long long)a.B * a.S * a.H;
  hipLaunchKernelGGL((delta_kernel<T, D>), dim3((unsigned)((rows + 255) / 256)), dim3(256), 0, s, a);
  if (bias_type == 0) {
    hipLaunchKernelGGL((dkdv_kernel<T, D, 0>), grid, dim3(NT), 0, s, a);
    hipLaunchKernelGGL((dq_kernel<T, D, 0>), grid, dim3(NT), 0, s, a);
  } else if (bias_type == 1) {
    hipLaunchKernelGGL((dkdv_kernel<T, D, 1>), grid, dim3(NT), 0, s, a);
    hipLaunchKernelGGL((dq_kernel<T, D, 1>), grid, dim3(NT), 0, s, a);
  } else if (bias_type == 3) {
    hipLaunchKernelGGL((dkdv_kernel<T, D, 3>), grid, dim3(NT), 0, s, a);
    hipLaunchKernelGGL((dq_kernel<T, D, 3>), grid, dim3(NT), 0, s, a);
  } else {
    hipLaunchKernelGGL((dkdv_kernel<T, D, 2>), grid, dim3(NT), 0, s, a);
    hipLaunchKernelGGL((dq_kernel<T, D, 2>), grid, dim3(NT), 0, s, a);
  }
  return DNA_OK;
}

template <typename T>
int run_d(bool bwd, const Args& a, int D, int bias_type, hipStream_t s) {
  if (D == 32) return run<T, 32>(bwd, a, bias_type, s);
  if (D == 64) return run<T, 64>(bwd, a, bias_type, s);
  return run<T, 128>(bwd, a, bias_type, s);
}

static int check(const void* qkv, int dtype, const void* bias, int bias_dtype, int bias_type,
                 int batch, int seqlen, int heads, int head_dim, const char* fn) {
  DNA_CHECK_ARG(qkv, "%s: null qkv", fn);
  DNA_CHECK_ARG(batch > 0 && seqlen > 0 && heads > 0, "%s: bad shape b=%d S=%d H=%d", fn, batch,
                seqlen, heads);
  DNA_CHECK_ARG(dtype == DNA_BF16 || dtype == DNA_F16, "%s: qkv dtype must be bf16 or fp16 (got %d)",
                fn, dtype);
  if (head_dim != 32 && head_dim != 64 && head_dim != 128) {
    set_error("%s: head_dim %d unsupported (32, 64, 128)", fn, head_dim);
    return DNA_ERR_UNSUPPORTED;
  }
  DNA_CHECK_ARG(bias_type >= 0 && bias_type <= 2, "%s: bias_type %d (0 none, 1 vector, 2 matrix)", fn,
                bias_type);
  DNA_CHECK_ARG(bias_type == 0 || bias, "%s: bias_type %d with a null bias", fn, bias_type);
  DNA_CHECK_ARG(bias_type == 0 || bias_dtype == DNA_F32 || bias_dtype == dtype,
                "%s: bias dtype must be fp32 or the qkv dtype", fn);
  return DNA_OK;
}

}  // namespace fa
}  // namespace dna

using namespace dna;

extern "C" int dna_flash_lse_rows(int seqlen) { return (seqlen + 127) / 128 * 128; }

extern "C" int dna_flash_fwd(const void* qkv, int dtype, const void* bias, int bias_dtype,
                             int bias_type, long long bias_sb, long long bias_sh, long long bias_sq,
                             int batch, int seqlen, int heads, int head_dim, int causal,
                             float softmax_scale, void* out, float* lse, void* stream) {
  int st = fa::check(qkv, dtype, bias, bias_dtype, bias_type, batch, seqlen, heads, head_dim,
                     "dna_flash_fwd");
  if (st) return st;
  DNA_CHECK_ARG(out && lse, "dna_flash_fwd: null output");
  fa::Args a{};
  a.qkv = (const unsigned short*)qkv;
  a.bias = bias; a.sb = bias_sb; a.sh = bias_sh; a.sq = bias_sq; a.bias_f32 = bias_dtype == DNA_F32;
  a.o = (unsigned short*)out; a.lse = lse;
  a.B = batch; a.S = seqlen; a.H = heads; a.Sr = dna_flash_lse_rows(seqlen); a.causal = causal != 0;
  a.scale = softmax_scale;
  hipStream_t s = as_stream(stream);
  if (dtype == DNA_BF16) fa::run_d<bf16>(false, a, head_dim, bias_type, s);
  else fa::run_d<fa::f16>(false, a, head_dim, bias_type, s);
  DNA_LAUNCH_CHECK("dna_flash_fwd");
  return DNA_OK;
}

extern "C" int dna_flash_bwd(const void* qkv, int dtype, const void* bias, int bias_dtype,
                             int bias_type, long long bias_sb, long long bias_sh, long long bias_sq,
                             const void* out, const void* dout, const float* lse, int batch,
                             int seqlen, int heads, int head_dim, int causal, float softmax_scale,
                             float* delta, void* dqkv, void* stream) {
  int st = fa::check(qkv, dtype, bias, bias_dtype, bias_type, batch, seqlen, heads, head_dim,
                     "dna_flash_bwd");
  if (st) return st;
  DNA_CHECK_ARG(out && dout && lse && delta && dqkv, "dna_flash_bwd: null pointer");
  fa::Args a{};
  a.qkv = (const unsigned short*)qkv;
  a.bias = bias; a.sb = bias_sb; a.sh = bias_sh; a.sq = bias_sq; a.bias_f32 = bias_dtype == DNA_F32;
  a.out = (const unsigned short*)out; a.dout = (const unsigned short*)dout;
  a.o = (unsigned short*)dqkv; a.lse = const_cast<float*>(lse); a.delta = delta;
  a.B = batch; a.S = seqlen; a.H = heads; a.Sr = dna_flash_lse_rows(seqlen); a.causal = causal != 0;
  a.scale = softmax_scale;
  hipStream_t s = as_stream(stream);
  if (dtype == DNA_BF16) fa::run_d<bf16>(true, a, head_dim, bias_type, s);
  else fa::run_d<fa::f16>(true, a, head_dim, bias_type, s);
  DNA_LAUNCH_CHECK("dna_flash_bwd");
  return DNA_OK;
}
