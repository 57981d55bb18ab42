// HyenaDNA implicit long filter, whole: the positional MLP of HyenaFilter.filter (reference
// hyena.py:162-247: Linear(E, 64) -> Sin -> [Linear(64, 64) -> Sin] x NI -> Linear(64, C, no
// bias), one Sin module shared by every activation) with ExponentialModulation (:140-163) and the
// filter transpose the long convolution reads (:438-441), forward in one launch and backward in
// one launch plus a slice sum -- in place of ~40 small launches per layer (casts, sin / cos,
// strided GEMMs, bias sums), which took ~1 ms per layer per step at config D.
//
// The dtype flow is the one bf16 autocast gives the reference module: every Linear rounds its
// input, weight and bias to bf16 and its output to bf16 (fp32 accumulation); Sin computes
// sin(freq * y) in fp32 from the bf16 y; the modulation multiplies the bf16 h in fp32. Backward:
// dh = bf16(dk * mod), each Linear's dx in bf16, dW / db summed in fp32 and rounded to bf16 once
// (the grad of the bf16 weight copy), Sin: darg = dx * cos(freq y), dfreq += darg * y (fp32),
// dy = bf16(darg * freq). The forward's sin and every exp are the hardware forms (v_sin / v_exp
// after the range scaling, ~1e-6 absolute; each result is rounded to bf16 next, 4e-3 relative); the
// backward keeps the library sin / cos (with the hardware forms its register allocation spills
// and hipcc 7.2's AGPR-copy rewrite crashes).
//
// Layout: a block = 4 waves works on tiles of 64 positions. The 64-wide GEMMs run on
// v_mfma_f32_16x16x32_bf16 with the positions as M: a lane ends with 4 consecutive positions of
// one channel, so the transposed filter store is a 16-B fp32 store and the per-channel
// activation rows ([channel][position] tiles) are 8-B LDS writes. The weights stay in registers
// as MFMA B fragments for the block's life (persistent grid). The backward recomputes the
// forward of its tile (cheaper than storing 4 x [L, 64] activations), and keeps the weight
// gradients of all its tiles in MFMA accumulators; the per-block partials are summed by
// dna_sum_slices (deterministic).
#include "common.h"

namespace dna {
namespace hflt {

constexpr int F = 64;       // MLP width (filter_order)
constexpr int TP = 64;      // positions per tile
constexpr int NT = 256;     // 4 waves
constexpr int RS = F + 8;   // LDS row stride in bf16 of a 64-wide tile: 144 B, conflict-free b128 reads
constexpr int TILE = TP * RS;
constexpr int MAXE = 8;
constexpr int MAXNI = 4;

struct Args {
  const float* z;                 // [L][E]
  const float* w1; const float* b1;   // [F][E], [F]
  const float* wi[MAXNI];         // [F][F] each
  const float* bi[MAXNI];         // [F] each
  const float* w4;                // [C][F]
  const float* freq;              // [F]
  const float* tpos;              // [L]
  const float* delta;             // [C]
  float shift;
  int L, E, NI, C, O;
  float* k;                       // forward: [O][C / O][L]
  const float* dk;                // backward: [O][C / O][L]
  float* part;                    // backward: [gridDim.x][P]
  float* dz;                      // backward: [L][E] or null
};

// partial-gradient offsets (floats) of one block's slice
struct Off {
  int w4, wi, bi, w1, b1, fr, P;
  __host__ __device__ Off(int C, int E, int NI) {
    w4 = 0;
    wi = C * F;
    bi = wi + NI * F * F;
    w1 = bi + NI * F;
    b1 = w1 + F * E;
    fr = b1 + F;
    P = fr + F;
  }
};

__device__ __forceinline__ float rb(float x) { return (float)(bf16)x; }
// sin / cos on the hardware unit (v_sin_f32 / v_cos_f32 take revolutions): the argument reduced to
// [-0.5, 0.5] revolutions first; ~1e-6 absolute against the library forms
__device__ __forceinline__ float hsin(float x) {
  const float r = x * 0.15915494309189535f;
  return __builtin_amdgcn_sinf(r - rintf(r));
}
__device__ __forceinline__ f32x4 mfma(bf16x8 a, bf16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
// 8 consecutive fp32 (16-B aligned) as a bf16 MFMA fragment
__device__ __forceinline__ bf16x8 frag8(const float* p) {
  const f32x4 x = *reinterpret_cast<const f32x4*>(p), y = *reinterpret_cast<const f32x4*>(p + 4);
  return bf16x8{(bf16)x[0], (bf16)x[1], (bf16)x[2], (bf16)x[3], (bf16)y[0], (bf16)y[1], (bf16)y[2], (bf16)y[3]};
}
// 8 fp32 at stride `st` as a bf16 fragment (a weight column)
__device__ __forceinline__ bf16x8 frag8s(const float* p, int st) {
  bf16x8 r;
#pragma unroll
  for (int q = 0; q < 8; ++q) r[q] = (bf16)p[q * st];
  return r;
}
__device__ __forceinline__ bf16x8 lds8(const bf16* p) { return *reinterpret_cast<const bf16x8*>(p); }
__device__ __forceinline__ void st4(bf16* p, float a, float b, float c, float d) {
  *reinterpret_cast<bf16x4*>(p) = bf16x4{(bf16)a, (bf16)b, (bf16)c, (bf16)d};
}
__device__ __forceinline__ float lane_sum4(float v) {  // over lanes l, l^16, l^32, l^48
  v += __shfl_xor(v, 16);
  v += __shfl_xor(v, 32);
  return v;
}

// Linear(E, F) + Sin on the VALU for a tile: lane -> position, wave -> channels 16 w .. +15 (the
// [j][pos] row writes of a wave are then 128 contiguous bytes: no LDS bank conflicts). Writes y (bf16 values, pre-sin) to ytile[j][pos] if given, the bf16 sin output to
// xrow[pos][j] and, if given, xcol[j][pos]. zt[pos][e]: the tile's rounded features.
__device__ __forceinline__ void first_layer(const float* w1s, const float* b1s, const float* frs,
                                           const float* zt, int E, bf16* xrow, bf16* xcol, bf16* ytile) {
  const int tid = threadIdx.x, pos = tid & 63, cg = (tid >> 6) * 16;
  float zz[MAXE];
#pragma unroll
  for (int e = 0; e < MAXE; ++e) zz[e] = e < E ? zt[pos * MAXE + e] : 0.f;
  bf16x8 o[2];
#pragma unroll
  for (int jj = 0; jj < 16; ++jj) {
    const int j = cg + jj;
    float acc = 0.f;
#pragma unroll
    for (int e = 0; e < MAXE; ++e)
      if (e < E) acc = fmaf(zz[e], w1s[j * MAXE + e], acc);
    const float y = rb(acc + b1s[j]);
    const float s = hsin(frs[j] * y);
    o[jj >> 3][jj & 7] = (bf16)s;
    if (xcol) xcol[j * RS + pos] = (bf16)s;
    if (ytile) ytile[j * RS + pos] = (bf16)y;
  }
  *reinterpret_cast<bf16x8*>(xrow + pos * RS + cg) = o[0];
  *reinterpret_cast<bf16x8*>(xrow + pos * RS + cg + 8) = o[1];
}

// stage the tile's positional features (bf16-rounded) and, once, the rounded L1 weights
__device__ __forceinline__ void stage_z(const Args& a, int p0, float* zt) {
  for (int e = threadIdx.x; e < TP * MAXE; e += NT) {
    const int pos = e / MAXE, c = e - pos * MAXE;
    zt[e] = (c < a.E) ? rb(a.z[(size_t)(p0 + pos) * a.E + c]) : 0.f;
  }
}
__device__ __forceinline__ void stage_w1(const Args& a, float* w1s, float* b1s, float* frs) {
  for (int e = threadIdx.x; e < F * MAXE; e += NT) {
    const int j = e / MAXE, c = e - j * MAXE;
    w1s[e] = c < a.E ? rb(a.w1[j * a.E + c]) : 0.f;
  }
  for (int e = threadIdx.x; e < F; e += NT) {
    b1s[e] = rb(a.b1[e]);
    frs[e] = a.freq[e];
  }
}

// C = 64 * CTW (each wave owns CTW 16-channel column tiles of the output layer), NI inner layers
template <int CTW, int NI>
__global__ __launch_bounds__(NT) void fwd_kernel(Args a) {
  __shared__ __attribute__((aligned(16))) bf16 xs[2][TILE];
  __shared__ __attribute__((aligned(16))) float zt[TP * MAXE];
  __shared__ float w1s[F * MAXE], b1s[F], frs[F];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int l16 = lane & 15, lg = lane >> 4;
  stage_w1(a, w1s, b1s, frs);
  // inner layers: wave w computes output channels 16 w + [0, 16)
  bf16x8 wib[NI > 0 ? NI : 1][2];
  float bib[NI > 0 ? NI : 1];
#pragma unroll
  for (int li = 0; li < NI; ++li) {
    {
      const float* row = a.wi[li] + (16 * w + l16) * F + 8 * lg;
      wib[li][0] = frag8(row);
      wib[li][1] = frag8(row + 32);
      bib[li] = rb(a.bi[li][16 * w + l16]);
    }
  }
  const float fr = a.freq[16 * w + l16];
  // output layer: wave w owns channels w * 16 CTW + 16 ct + [0, 16)
  bf16x8 w4b[CTW][2];
  float ad[CTW];
#pragma unroll
  for (int ct = 0; ct < CTW; ++ct) {
    const int c = w * 16 * CTW + ct * 16 + l16;
    w4b[ct][0] = frag8(a.w4 + (size_t)c * F + 8 * lg);
    w4b[ct][1] = frag8(a.w4 + (size_t)c * F + 32 + 8 * lg);
    ad[ct] = fabsf(a.delta[c]);
  }
  const int V = a.C / a.O;
  const int ntiles = a.L / TP;
  for (int tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const int p0 = tile * TP;
    stage_z(a, p0, zt);
    __syncthreads();
    first_layer(w1s, b1s, frs, zt, a.E, xs[0], nullptr, nullptr);
    __syncthreads();
    for (int li = 0; li < NI; ++li) {
      const bf16* src = xs[li & 1];
      bf16* dst = xs[(li + 1) & 1];
      bf16x8 wb0 = wib[0][0], wb1 = wib[0][1];
      float bb = bib[0];
#pragma unroll
      for (int q = 1; q < NI; ++q)
        if (li == q) { wb0 = wib[q][0]; wb1 = wib[q][1]; bb = bib[q]; }
#pragma unroll
      for (int ms = 0; ms < 4; ++ms) {
        const bf16* ar = src + (ms * 16 + l16) * RS + 8 * lg;
        f32x4 acc = mfma(lds8(ar), wb0, f32x4{0.f, 0.f, 0.f, 0.f});
        acc = mfma(lds8(ar + 32), wb1, acc);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float y = rb(acc[i] + bb);
          dst[(ms * 16 + 4 * lg + i) * RS + 16 * w + l16] = (bf16)hsin(fr * y);
        }
      }
      __syncthreads();
    }
    const bf16* src = xs[NI & 1];
#pragma unroll
    for (int ms = 0; ms < 4; ++ms) {
      const bf16* ar = src + (ms * 16 + l16) * RS + 8 * lg;
      const bf16x8 a0 = lds8(ar), a1 = lds8(ar + 32);
      const int pos = p0 + ms * 16 + 4 * lg;
      const f32x4 tv = *reinterpret_cast<const f32x4*>(a.tpos + pos);
#pragma unroll
      for (int ct = 0; ct < CTW; ++ct) {
        f32x4 acc = mfma(a0, w4b[ct][0], f32x4{0.f, 0.f, 0.f, 0.f});
        acc = mfma(a1, w4b[ct][1], acc);
        const int c = w * 16 * CTW + ct * 16 + l16;
        f32x4 o;
#pragma unroll
        for (int i = 0; i < 4; ++i) o[i] = rb(acc[i]) * (__expf(-tv[i] * ad[ct]) + a.shift);
        *reinterpret_cast<f32x4*>(a.k + ((size_t)(c % a.O) * V + c / a.O) * a.L + pos) = o;
      }
    }
    __syncthreads();  // xs[0] / zt are rewritten by the next tile
  }
}

// Backward. Dynamic LDS (bf16 tiles of TILE elements unless noted):
//   xa[2]            forward recompute, [pos][k] rows (MFMA A operands)
//   xT[NI + 1]       inputs of the inner layers and of the output layer, [k][pos] rows (dW B)
//   yv[NI + 1]       pre-sin values of L1 and the inner layers, [j][pos] rows
//   dhc, dhp         one 64-channel chunk of dh as [c][pos] (dW4 A) and [pos][c] (dX4 A); dhp's
//                    8-column chunks XOR-swizzled by 2 * (pos / 16 % 4): the staging threads of a
//                    wave write 4 rows 16 apart (the same banks) at once -- 4-way conflicts else
//   dyt, dyp         dy of the current layer as [j][pos] (dW A) and [pos][j] (dX A)
//   zt (fp32)        the tile's features
template <int CTW, int NI>
__global__ __launch_bounds__(NT) void bwd_kernel(Args a) {
  extern __shared__ __attribute__((aligned(16))) bf16 smem[];
  bf16* xa0 = smem;
  bf16* xa1 = xa0 + TILE;
  bf16* xT = xa1 + TILE;
  bf16* yv = xT + (NI + 1) * TILE;
  bf16* dhc = yv + (NI + 1) * TILE;
  bf16* dhp = dhc + TILE;
  bf16* dyt = dhp + TILE;
  bf16* dyp = dyt + TILE;
  float* zt = reinterpret_cast<float*>(dyp + TILE);
  __shared__ float w1s[F * MAXE], b1s[F], frs[F];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int l16 = lane & 15, lg = lane >> 4;
  const int E = a.E;
  stage_w1(a, w1s, b1s, frs);
  const Off off(a.C, E, NI);
  // forward fragments (inner layers, wave w -> output channels 16 w + l16) and the transposed
  // ones for dX = dY . W (wave w -> input channels 16 w + l16: a weight column)
  bf16x8 wib[NI > 0 ? NI : 1][2], wit[NI > 0 ? NI : 1][2];
  float bib[NI > 0 ? NI : 1];
#pragma unroll
  for (int li = 0; li < NI; ++li) {
    {
      const float* row = a.wi[li] + (16 * w + l16) * F + 8 * lg;
      wib[li][0] = frag8(row);
      wib[li][1] = frag8(row + 32);
      bib[li] = rb(a.bi[li][16 * w + l16]);
      const float* col = a.wi[li] + (8 * lg) * F + 16 * w + l16;
      wit[li][0] = frag8s(col, F);
      wit[li][1] = frag8s(col + 32 * F, F);
    }
  }
  const float fr = a.freq[16 * w + l16];
  // dX4 = dh . W4: B[k = c][n = j] = W4[c][j], wave w -> j = 16 w + l16, per 64-channel chunk
  constexpr int NCH = CTW;  // C / 64 chunks
  bf16x8 w4t[NCH][2];
#pragma unroll
  for (int cc = 0; cc < NCH; ++cc) {
    const float* col = a.w4 + (size_t)(cc * 64 + 8 * lg) * F + 16 * w + l16;
    w4t[cc][0] = frag8s(col, F);
    w4t[cc][1] = frag8s(col + 32 * F, F);
  }
  float ad[NCH];  // |delta| of the channel this thread stages per chunk: c = cc * 64 + tid / 4
#pragma unroll
  for (int cc = 0; cc < NCH; ++cc) ad[cc] = fabsf(a.delta[cc * 64 + (tid >> 2)]);
  // gradient accumulators: dW4 chunk cc, rows (c) 16 w + 4 lg + i, column tile nt (j = 16 nt + l16)
  f32x4 gw4[NCH][4], gwi[NI > 0 ? NI : 1][4];
#pragma unroll
  for (int cc = 0; cc < NCH; ++cc)
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) gw4[cc][nt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int li = 0; li < NI; ++li)
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) gwi[li][nt] = f32x4{0.f, 0.f, 0.f, 0.f};
  float gbi[NI > 0 ? NI : 1] = {}, gb1 = 0.f, gfr = 0.f, gw1[MAXE] = {};
  const int V = a.C / a.O;
  const int ntiles = a.L / TP;
  for (int tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const int p0 = tile * TP;
    // ---- forward recompute
    stage_z(a, p0, zt);
    __syncthreads();
    first_layer(w1s, b1s, frs, zt, E, xa0, xT, yv);
    __syncthreads();
    for (int li = 0; li < NI; ++li) {
      const bf16* src = (li & 1) ? xa1 : xa0;
      bf16* dst = (li & 1) ? xa0 : xa1;
      bf16x8 wb0 = wib[0][0], wb1 = wib[0][1];
      float bb = bib[0];
#pragma unroll
      for (int q = 1; q < NI; ++q)
        if (li == q) { wb0 = wib[q][0]; wb1 = wib[q][1]; bb = bib[q]; }
      bf16* yrow = yv + (li + 1) * TILE + (16 * w + l16) * RS;
      bf16* xrow = xT + (li + 1) * TILE + (16 * w + l16) * RS;
#pragma unroll
      for (int ms = 0; ms < 4; ++ms) {
        const bf16* ar = src + (ms * 16 + l16) * RS + 8 * lg;
        f32x4 acc = mfma(lds8(ar), wb0, f32x4{0.f, 0.f, 0.f, 0.f});
        acc = mfma(lds8(ar + 32), wb1, acc);
        float y[4], s[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          y[i] = rb(acc[i] + bb);
          s[i] = hsin(fr * y[i]);  // as the forward kernel computed it
          dst[(ms * 16 + 4 * lg + i) * RS + 16 * w + l16] = (bf16)s[i];
        }
        st4(yrow + ms * 16 + 4 * lg, y[0], y[1], y[2], y[3]);
        st4(xrow + ms * 16 + 4 * lg, s[0], s[1], s[2], s[3]);
      }
      __syncthreads();
    }
    // ---- output layer + modulation: dh chunks -> dW4, dX4
    f32x4 dx[4];
#pragma unroll
    for (int ms = 0; ms < 4; ++ms) dx[ms] = f32x4{0.f, 0.f, 0.f, 0.f};
    const bf16* x4 = xT + NI * TILE;
#pragma unroll
    for (int cc = 0; cc < NCH; ++cc) {
      {  // thread -> channel cc * 64 + tid / 4, positions 16 (tid % 4) .. +15
        const int cl = tid >> 2, pg = (tid & 3) * 16, c = cc * 64 + cl;
        const float* src = a.dk + ((size_t)(c % a.O) * V + c / a.O) * a.L + p0 + pg;
        float d[16];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const f32x4 v = *reinterpret_cast<const f32x4*>(src + 4 * q);
          const f32x4 tv = *reinterpret_cast<const f32x4*>(a.tpos + p0 + pg + 4 * q);
#pragma unroll
          for (int i = 0; i < 4; ++i) d[4 * q + i] = rb(v[i] * (__expf(-tv[i] * ad[cc]) + a.shift));
        }
        bf16x8 h0, h1;
#pragma unroll
        for (int i = 0; i < 8; ++i) { h0[i] = (bf16)d[i]; h1[i] = (bf16)d[8 + i]; }
        *reinterpret_cast<bf16x8*>(dhc + cl * RS + pg) = h0;
        *reinterpret_cast<bf16x8*>(dhc + cl * RS + pg + 8) = h1;
#pragma unroll
        for (int i = 0; i < 16; ++i)
          dhp[(pg + i) * RS + (((cl >> 3) ^ (2 * ((pg >> 4) & 3))) << 3) + (cl & 7)] = (bf16)d[i];
      }
      __syncthreads();
      {  // dW4[c][j] += sum_pos dh[pos][c] x4[pos][j]: rows c = 16 w + (chunk), column tiles nt
        const bf16* ar = dhc + (16 * w + l16) * RS + 8 * lg;
        const bf16x8 a0 = lds8(ar), a1 = lds8(ar + 32);
#pragma unroll
        for (int nt = 0; nt < 4; ++nt) {
          const bf16* br = x4 + (16 * nt + l16) * RS + 8 * lg;
          gw4[cc][nt] = mfma(a0, lds8(br), gw4[cc][nt]);
          gw4[cc][nt] = mfma(a1, lds8(br + 32), gw4[cc][nt]);
        }
        // dX4[pos][j] += sum_c dh[pos][c] W4[c][j]: column tile w, row tiles ms
#pragma unroll
        for (int ms = 0; ms < 4; ++ms) {
          const bf16* pr = dhp + (ms * 16 + l16) * RS;  // row ms * 16 + l16: swizzle 2 * ms
          dx[ms] = mfma(lds8(pr + ((lg ^ (2 * ms)) << 3)), w4t[cc][0], dx[ms]);
          dx[ms] = mfma(lds8(pr + (((lg + 4) ^ (2 * ms)) << 3)), w4t[cc][1], dx[ms]);
        }
      }
      __syncthreads();
    }
    // ---- back through Sin_l and layer l, l = NI .. 0 (layer 0 = Linear(E, F))
    for (int l = NI; l >= 0; --l) {
      const bf16* yrow = yv + l * TILE + (16 * w + l16) * RS;
      float gb = 0.f;
#pragma unroll
      for (int ms = 0; ms < 4; ++ms) {
        const bf16x4 yy = *reinterpret_cast<const bf16x4*>(yrow + ms * 16 + 4 * lg);
        float dy[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float y = (float)yy[i];
          // (library cosf: v_sin / v_cos in this loop crash the ROCm 7.2 code generator)
          const float darg = rb(dx[ms][i]) * cosf(fr * y);
          gfr = fmaf(darg, y, gfr);
          dy[i] = rb(darg * fr);
          gb += dy[i];
          dyp[(ms * 16 + 4 * lg + i) * RS + 16 * w + l16] = (bf16)dy[i];
        }
        st4(dyt + (16 * w + l16) * RS + ms * 16 + 4 * lg, dy[0], dy[1], dy[2], dy[3]);
        if (l == 0) {  // dW1[j][e] += dy[pos][j] z[pos][e]
#pragma unroll
          for (int e = 0; e < MAXE; ++e)
#pragma unroll
            for (int i = 0; i < 4; ++i) gw1[e] = fmaf(dy[i], zt[(ms * 16 + 4 * lg + i) * MAXE + e], gw1[e]);
        }
      }
      if (l == 0) gb1 += gb;
#pragma unroll
      for (int q = 0; q < NI; ++q)
        if (l - 1 == q) gbi[q] += gb;
      __syncthreads();
      if (l == 0) {
        if (a.dz) {  // dz[pos][e] = bf16(sum_j dy[pos][j] W1[j][e])
          for (int e2 = tid; e2 < TP * E; e2 += NT) {
            const int pos = e2 / E, e = e2 - pos * E;
            float s = 0.f;
            for (int j = 0; j < F; ++j) s = fmaf((float)dyp[pos * RS + j], w1s[j * MAXE + e], s);
            a.dz[(size_t)(p0 + pos) * E + e] = rb(s);
          }
        }
        break;
      }
      const int li = l - 1;
      {  // dW_li[j][i] += sum_pos dy[pos][j] x_li[pos][i]; dX_li[pos][i] = sum_j dy[pos][j] W_li[j][i]
        const bf16* ar = dyt + (16 * w + l16) * RS + 8 * lg;
        const bf16x8 a0 = lds8(ar), a1 = lds8(ar + 32);
        const bf16* xin = xT + li * TILE;
#pragma unroll
        for (int q = 0; q < NI; ++q) {
          if (li == q) {
#pragma unroll
            for (int nt = 0; nt < 4; ++nt) {
              const bf16* br = xin + (16 * nt + l16) * RS + 8 * lg;
              gwi[q][nt] = mfma(a0, lds8(br), gwi[q][nt]);
              gwi[q][nt] = mfma(a1, lds8(br + 32), gwi[q][nt]);
            }
#pragma unroll
            for (int ms = 0; ms < 4; ++ms) {
              const bf16* pr = dyp + (ms * 16 + l16) * RS + 8 * lg;
              dx[ms] = mfma(lds8(pr), wit[q][0], f32x4{0.f, 0.f, 0.f, 0.f});
              dx[ms] = mfma(lds8(pr + 32), wit[q][1], dx[ms]);
            }
          }
        }
      }
      __syncthreads();
    }
    __syncthreads();
  }
  // ---- per-block partials
  float* P = a.part + (size_t)blockIdx.x * off.P;
#pragma unroll
  for (int cc = 0; cc < NCH; ++cc)
#pragma unroll
    for (int nt = 0; nt < 4; ++nt)
#pragma unroll
      for (int i = 0; i < 4; ++i)
        P[off.w4 + (cc * 64 + 16 * w + 4 * lg + i) * F + 16 * nt + l16] = gw4[cc][nt][i];
#pragma unroll
  for (int li = 0; li < NI; ++li)
    #pragma unroll
      for (int nt = 0; nt < 4; ++nt)
#pragma unroll
        for (int i = 0; i < 4; ++i)
          P[off.wi + li * F * F + (16 * w + 4 * lg + i) * F + 16 * nt + l16] = gwi[li][nt][i];
  const int j = 16 * w + l16;
#pragma unroll
  for (int li = 0; li < NI; ++li) {
    const float s = lane_sum4(gbi[li]);
    if (li < NI && lg == 0) P[off.bi + li * F + j] = s;
  }
  const float sb1 = lane_sum4(gb1), sfr = lane_sum4(gfr);
  if (lg == 0) {
    P[off.b1 + j] = sb1;
    P[off.fr + j] = sfr;
  }
#pragma unroll
  for (int e = 0; e < MAXE; ++e) {
    const float s = lane_sum4(gw1[e]);
    if (e < E && lg == 0) P[off.w1 + j * E + e] = s;
  }
}

// out[i] = sum over the G block slices of part[g][i] (fixed order), rounded to bf16 for i < nround
// (the weight / bias gradients: the grad of autocast's bf16 copies), fp32 past it (freq)
__global__ __launch_bounds__(256) void finish_kernel(const float* __restrict__ part, int G, int P, int nround,
                                                     float* __restrict__ out) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= P) return;
  float s[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};  // 8 slices in flight, fixed order
  int g = 0;
  for (; g + 8 <= G; g += 8)
#pragma unroll
    for (int q = 0; q < 8; ++q) s[q] += part[(size_t)(g + q) * P + i];
  for (; g < G; ++g) s[0] += part[(size_t)g * P + i];
  const float t = ((s[0] + s[1]) + (s[2] + s[3])) + ((s[4] + s[5]) + (s[6] + s[7]));
  out[i] = i < nround ? rb(t) : t;
}

inline size_t bwd_lds(int NI) { return (size_t)(2 + 2 * (NI + 1) + 4) * TILE * 2 + TP * MAXE * 4; }

template <typename Fn>
int by_ctw(int C, Fn&& fn) {
  switch (C / 64) {
    case 1: fn(std::integral_constant<int, 1>()); return 0;
    case 2: fn(std::integral_constant<int, 2>()); return 0;
    case 4: fn(std::integral_constant<int, 4>()); return 0;
    case 8: fn(std::integral_constant<int, 8>()); return 0;
    default: return -1;
  }
}

inline int grid_for(int L) {
  int dev = 0, n = 256;
  if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    n = 256;
  const int tiles = L / TP;
  return tiles < n ? tiles : n;
}

inline bool fill(Args& a, const float* z, const float* w1, const float* b1, const float* const* wi,
                 const float* const* bi, int NI, const float* w4, const float* freq, const float* tpos,
                 const float* delta, float shift, int L, int E, int C, int O) {
  if (!z || !w1 || !b1 || !w4 || !freq || !tpos || !delta || NI < 0 || NI > MAXNI || E < 1 || E > MAXE ||
      L <= 0 || L % TP != 0 || C % 64 != 0 || O <= 0 || C % O != 0)
    return false;
  a.z = z; a.w1 = w1; a.b1 = b1; a.w4 = w4; a.freq = freq; a.tpos = tpos; a.delta = delta;
  a.shift = shift; a.L = L; a.E = E; a.NI = NI; a.C = C; a.O = O;
  for (int i = 0; i < MAXNI; ++i) {
    a.wi[i] = i < NI ? wi[i] : nullptr;
    a.bi[i] = i < NI ? bi[i] : nullptr;
    if (i < NI && (!wi[i] || !bi[i])) return false;
  }
  return true;
}

}  // namespace hflt
}  // namespace dna

using namespace dna;

extern "C" int dna_hyena_filter_part_elems(int L, int E, int NI, int C) {
  if (L <= 0 || L % hflt::TP != 0) return 0;
  return hflt::grid_for(L) * hflt::Off(C, E, NI).P;
}

extern "C" int dna_hyena_filter_part_stride(int E, int NI, int C) { return hflt::Off(C, E, NI).P; }

extern "C" int dna_hyena_filter_fwd(const float* z, const float* w1, const float* b1, const float* const* wi,
                                    const float* const* bi, int NI, const float* w4, const float* freq,
                                    const float* tpos, const float* delta, float shift, int L, int E, int C,
                                    int O, float* k, void* stream) {
  hflt::Args a{};
  DNA_CHECK_ARG(k && hflt::fill(a, z, w1, b1, wi, bi, NI, w4, freq, tpos, delta, shift, L, E, C, O),
                "dna_hyena_filter_fwd: bad args (L %% 64, C in {64,128,256,512}, E <= 8, NI <= 4)");
  a.k = k;
  const int G = L / hflt::TP;  // one tile per block: the forward is latency-bound, not weight-load-bound
  hipStream_t s = as_stream(stream);
  DNA_CHECK_ARG(NI == 2, "dna_hyena_filter_fwd: NI = %d (built for the reference's 2 inner layers)", NI);
  const int rc = hflt::by_ctw(C, [&](auto ctw) {
    hipLaunchKernelGGL((hflt::fwd_kernel<decltype(ctw)::value, 2>), dim3(G), dim3(hflt::NT), 0, s, a);
  });
  DNA_CHECK_ARG(rc == 0, "dna_hyena_filter_fwd: C = %d not in {64, 128, 256, 512}", C);
  DNA_LAUNCH_CHECK("dna_hyena_filter_fwd");
  return DNA_OK;
}

extern "C" int dna_hyena_filter_bwd(const float* z, const float* w1, const float* b1, const float* const* wi,
                                    const float* const* bi, int NI, const float* w4, const float* freq,
                                    const float* tpos, const float* delta, float shift, int L, int E, int C,
                                    int O, const float* dk, float* part, float* dz, void* stream) {
  hflt::Args a{};
  DNA_CHECK_ARG(dk && part && hflt::fill(a, z, w1, b1, wi, bi, NI, w4, freq, tpos, delta, shift, L, E, C, O),
                "dna_hyena_filter_bwd: bad args (L %% 64, C in {64,128,256,512}, E <= 8, NI <= 4)");
  a.dk = dk; a.part = part; a.dz = dz;
  const int G = hflt::grid_for(L);
  const size_t lds = hflt::bwd_lds(NI);
  hipStream_t s = as_stream(stream);
  DNA_CHECK_ARG(NI == 2, "dna_hyena_filter_bwd: NI = %d (built for the reference's 2 inner layers)", NI);
  const int rc = hflt::by_ctw(C, [&](auto ctw) {
    auto kern = hflt::bwd_kernel<decltype(ctw)::value, 2>;
    (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipLaunchKernelGGL(kern, dim3(G), dim3(hflt::NT), lds, s, a);
  });
  DNA_CHECK_ARG(rc == 0, "dna_hyena_filter_bwd: C = %d not in {64, 128, 256, 512}", C);
  DNA_LAUNCH_CHECK("dna_hyena_filter_bwd");
  return DNA_OK;
}

extern "C" int dna_hyena_filter_finish(const float* part, int G, int P, int nround, float* out, void* stream) {
  DNA_CHECK_ARG(part && out && G > 0 && P > 0 && nround >= 0 && nround <= P, "dna_hyena_filter_finish: bad args");
  hipLaunchKernelGGL(hflt::finish_kernel, dim3((P + 255) / 256), dim3(256), 0, as_stream(stream), part, G, P,
                     nround, out);
  DNA_LAUNCH_CHECK("dna_hyena_filter_finish");
  return DNA_OK;
}
