// FFT long convolution of the HyenaDNA filter (reference src/models/sequence/hyena.py:60-92,
// called from HyenaFilter.forward :253-280), forward and backward, gfx950.
//
//   y[r, t] = sum_{j<L} k[d, j] * u~[r, (t - j) mod N] + bias[d] * u[r, t],  t < L,  N = 2L
// for rows r = (b, d) of u [B, D, L]; u~ is u zero-padded to N (causal: at offset 0,
// bidirectional: at offset pad_before = L/2 -- the reference's F.pad then rfft(n=2L)).
//
// Layout and passes. N = M1 * M2 (M2 = 512 for N >= 1024, M1 <= 512). Two rows with the same
// filter (batches b, b+1 of channel d) are packed into ONE complex sequence z = u~_b + i u~_{b+1};
// since the filter is real, IFFT(Z * K) = (u~_b * k) + i (u~_{b+1} * k) -- no separation step.
// With n = n1*M2 + n2 and k = k1 + M1*k2 (four-step / Bailey):
//   A  column pass: for each column n2, FFT-M1 over n1 (LDS-staged, 8192/M1 columns per block so
//      the global reads/writes are row segments of 32 columns at M1 = 256), times W_N^(n2*k1)
//      -> T[k1][n2]
//   B  row pass:    for each row k1, FFT-M2 over n2 -> spectrum Z[k1 + M1*k2], times the filter
//      spectrum (stored in the same [k1][k2] order, 1/N folded in), inverse FFT-M2 -> T'[k1][n2]
//   C  column pass: times W_N^-(n2*k1), inverse FFT-M1 over k1 -> z[n1*M2 + n2]; writes rows
//      b, b+1 (real, imaginary part) for t < L. The bias term bias*u is a filter tap at
//      (N - pad_before) mod N folded into the filter spectrum, so no epilogue read of u.
// FFTs are autosort Stockham passes in LDS with radix-8/4/2 register butterflies (16 points per
// thread per pass) and an LDS twiddle table W_M^m; the inter-pass twiddles W_N^(n2*k1) come
// from a two-level LDS table (W_N^(m & 511) * W_N^(512*(m >> 9))), all built with sincospi of
// exactly representable arguments.
// Backward: du runs the same three passes on dy (offset 0) with conj(K) and reads the output at
// offset pad_before; dk = Re IFFT(sum_pairs conj(Z_u) Z_dy) / N (the packed pair's cross terms are
// purely imaginary after the inverse transform), j < L; dbias = sum_{b,t} dy u.
// All arithmetic fp32; inputs/outputs fp32 or bf16 (u, y, dy, du), filters and grads fp32.
#include <math.h>

#include <mutex>
#include <type_traits>
#include <vector>

#include "common.h"

namespace dna {
namespace fftc {

typedef float2 cf;

__device__ __forceinline__ cf cadd(cf a, cf b) { return make_float2(a.x + b.x, a.y + b.y); }
__device__ __forceinline__ cf csub(cf a, cf b) { return make_float2(a.x - b.x, a.y - b.y); }
__device__ __forceinline__ cf cmul(cf a, cf b) {
  return make_float2(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x);
}
__device__ __forceinline__ cf cconj(cf a) { return make_float2(a.x, -a.y); }

// W_{2^18}^j = exp(-2 pi i j / 2^18), j < 2^18: computed on the host in double precision and
// rounded once (ensure_twiddles, first use per device). Every table a block builds (W_M, the
// two-level W_N, the bias-tap phases) is a strided read of it (L2/MALL-resident, 2 MB) instead
// of an OCML sincospif per entry (~40 VALU each, ~1000 per block).
constexpr int LOG_TW = 18;
__device__ cf g_w18[1 << LOG_TW];

// exp(-2 pi i m / N) for integer m in [0, N), N = 2^logN <= 2^18.
__device__ __forceinline__ cf twiddle(uint32_t m, int logN) { return g_w18[m << (LOG_TW - logN)]; }

// ------------------------------------------------------------------ register butterflies
// multiply by W_4^1 = -i (forward) / +i (inverse)
template <bool INV> __device__ __forceinline__ cf mul_w4(cf a) {
  return INV ? make_float2(-a.y, a.x) : make_float2(a.y, -a.x);
}
// multiply by W_8^1 = (1 -/+ i)/sqrt(2)
template <bool INV> __device__ __forceinline__ cf mul_w8(cf a) {
  const float r = 0.70710678118654752f;
  return INV ? make_float2((a.x - a.y) * r, (a.x + a.y) * r) : make_float2((a.x + a.y) * r, (a.y - a.x) * r);
}
template <bool INV> __device__ __forceinline__ void dft2(cf* x) {
  const cf t = x[0];
  x[0] = cadd(t, x[1]);
  x[1] = csub(t, x[1]);
}
template <bool INV> __device__ __forceinline__ void dft4(cf* x) {
  const cf a0 = cadd(x[0], x[2]), a1 = csub(x[0], x[2]);
  const cf a2 = cadd(x[1], x[3]), a3 = mul_w4<INV>(csub(x[1], x[3]));
  x[0] = cadd(a0, a2);
  x[2] = csub(a0, a2);
  x[1] = cadd(a1, a3);
  x[3] = csub(a1, a3);
}
template <bool INV> __device__ __forceinline__ void dft8(cf* x) {
  cf e[4] = {x[0], x[2], x[4], x[6]}, o[4] = {x[1], x[3], x[5], x[7]};
  dft4<INV>(e);
  dft4<INV>(o);
  o[1] = mul_w8<INV>(o[1]);
  o[2] = mul_w4<INV>(o[2]);
  o[3] = mul_w4<INV>(mul_w8<INV>(o[3]));
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    x[k] = cadd(e[k], o[k]);
    x[k + 4] = csub(e[k], o[k]);
  }
}
// x * W_16^m (forward: exp(-2 pi i m / 16); INV: conjugate), m in 1..9
template <bool INV, int m> __device__ __forceinline__ cf mul_w16(cf a) {
  constexpr float c1 = 0.92387953251128674f, s1 = 0.38268343236508977f;
  if constexpr (m == 2) return mul_w8<INV>(a);
  else if constexpr (m == 4) return mul_w4<INV>(a);
  else if constexpr (m == 6) return mul_w4<INV>(mul_w8<INV>(a));
  else {
    // W_16^1 = (c1, -s1), W_16^3 = (s1, -c1), W_16^9 = (-c1, s1)
    constexpr float wr = m == 1 ? c1 : m == 3 ? s1 : -c1;
    constexpr float wi0 = m == 1 ? -s1 : m == 3 ? -c1 : s1;
    const float wi = INV ? -wi0 : wi0;
    return make_float2(a.x * wr - a.y * wi, a.x * wi + a.y * wr);
  }
}
// 16-point DFT in registers, natural order in and out: radix 4 x 4, n = na + 4 nb,
// k = ka + 4 kb: X[ka + 4 kb] = sum_na W_4^(na kb) W_16^(na ka) DFT4_nb(x[na + 4 nb])[ka]
template <bool INV> __device__ __forceinline__ void dft16(cf* x) {
  cf a[4][4];
#pragma unroll
  for (int na = 0; na < 4; ++na) {
    cf t[4] = {x[na], x[na + 4], x[na + 8], x[na + 12]};
    dft4<INV>(t);
#pragma unroll
    for (int ka = 0; ka < 4; ++ka) a[na][ka] = t[ka];
  }
  a[1][1] = mul_w16<INV, 1>(a[1][1]);
  a[1][2] = mul_w16<INV, 2>(a[1][2]);
  a[1][3] = mul_w16<INV, 3>(a[1][3]);
  a[2][1] = mul_w16<INV, 2>(a[2][1]);
  a[2][2] = mul_w16<INV, 4>(a[2][2]);
  a[2][3] = mul_w16<INV, 6>(a[2][3]);
  a[3][1] = mul_w16<INV, 3>(a[3][1]);
  a[3][2] = mul_w16<INV, 6>(a[3][2]);
  a[3][3] = mul_w16<INV, 9>(a[3][3]);
#pragma unroll
  for (int ka = 0; ka < 4; ++ka) {
    cf t[4] = {a[0][ka], a[1][ka], a[2][ka], a[3][ka]};
    dft4<INV>(t);
#pragma unroll
    for (int kb = 0; kb < 4; ++kb) x[ka + 4 * kb] = t[kb];
  }
}
template <int R, bool INV> __device__ __forceinline__ void dft(cf* x) {
  if constexpr (R == 8) dft8<INV>(x);
  else if constexpr (R == 4) dft4<INV>(x);
  else dft2<INV>(x);
}

// ------------------------------------------------------------------ LDS Stockham FFT
// A block transforms G sequences of length M = 2^logM held in LDS at buf[g*S + i], with
// G*M = PTS points (PTS/NTH = 16 per thread per pass, whatever the radix). Autosort Stockham
// (Govindaraju et al. 2008): natural order in and out, in place (each pass reads its 16
// points into registers, barrier, writes them, barrier). Twiddles from the LDS table
// twM[m] = W_M^m (m < M). Unscaled; INV conjugates all twiddles.
#ifndef FFT_LOG_PTS
#define FFT_LOG_PTS 13
#endif
constexpr int LOG_PTS = FFT_LOG_PTS;  // points per block: 8192 (512 threads) or 4096 (256)
constexpr int PTS = 1 << LOG_PTS;
constexpr int NTH = PTS / 16;
constexpr int PPT = PTS / NTH;  // points per thread per pass
// 8 waves per block, 2 blocks per CU (LDS ~78 KB each): 4 waves per SIMD, <= 128 VGPRs.
#define FFT_BOUNDS __launch_bounds__(NTH, 4)  // HIP: 2nd argument = min waves per SIMD

// LDS address of point i of sequence g: one pad slot every 16 points (the stride-R writes of
// the first Stockham passes then spread over all banks) and a caller-chosen sequence stride S.
__device__ __forceinline__ int lds_at(int g, int i, int S) { return g * S + i + (i >> 4); }
// sequence stride for length M: padded length (+1 for column buffers, whose transposing
// global<->LDS copies walk across sequences)
__host__ __device__ __forceinline__ int seq_stride(int logM, bool col) {
  return (1 << logM) + ((1 << logM) >> 4) + (col ? 1 : 0);
}

template <int R, int LOGR, bool INV, int NT = NTH>  // NT threads, PPT points each
__device__ __forceinline__ void stockham_pass(cf* buf, int G, int logM, int S, int logNs, const cf* twM) {
  constexpr int IPT = PPT / R;  // butterflies per thread
  const int M = 1 << logM;
  const int lognbf = logM - LOGR;
  const int items = G << lognbf;
  const int Ns = 1 << logNs;
  const int logtstep = logM - logNs - LOGR;
  cf x[IPT][R];
#pragma unroll
  for (int it = 0; it < IPT; ++it) {
    const int w = threadIdx.x + it * NT;
    if (w < items) {
      const int g = w >> lognbf, j = w & ((1 << lognbf) - 1);
      const int k = j & (Ns - 1);
#pragma unroll
      for (int r = 0; r < R; ++r) {
        cf v = buf[lds_at(g, j + (r << lognbf), S)];
        if (r > 0 && logNs > 0) {
          cf t = twM[((r * k) << logtstep) & (M - 1)];
          if (INV) t.y = -t.y;
          v = cmul(v, t);
        }
        x[it][r] = v;
      }
      dft<R, INV>(x[it]);
    }
  }
  __syncthreads();
#pragma unroll
  for (int it = 0; it < IPT; ++it) {
    const int w = threadIdx.x + it * NT;
    if (w < items) {
      const int g = w >> lognbf, j = w & ((1 << lognbf) - 1);
      const int k = j & (Ns - 1);
      const int base = ((j - k) << LOGR) + k;
#pragma unroll
      for (int r = 0; r < R; ++r) buf[lds_at(g, base + (r << logNs), S)] = x[it][r];
    }
  }
  __syncthreads();
}

template <bool INV, int NT = NTH>
__device__ __forceinline__ void fft_lds(cf* buf, int G, int logM, int S, const cf* twM) {
  int logNs = 0, left = logM;
  while (left >= 3) {
    stockham_pass<8, 3, INV, NT>(buf, G, logM, S, logNs, twM);
    logNs += 3;
    left -= 3;
  }
  if (left == 2) stockham_pass<4, 2, INV, NT>(buf, G, logM, S, logNs, twM);
  else if (left == 1) stockham_pass<2, 1, INV, NT>(buf, G, logM, S, logNs, twM);
}

// LDS twiddle table tw[m] = W_M^m, m < M.
__device__ __forceinline__ void make_table(cf* tw, int logM) {
  const int M = 1 << logM;
  for (int m = threadIdx.x; m < M; m += blockDim.x) tw[m] = twiddle(m, logM);
}

// Two-level table for W_N^m, m < N <= 2^18: lo[m & (2^lb - 1)] * hi[m >> lb], lb = logN/2.
struct BigTwiddle {
  cf* lo;  // [2^lb]
  cf* hi;  // [2^(logN - lb)]
  int lb;
  __device__ __forceinline__ void init(int logN) {
    lb = logN >> 1;
    hi = lo + (1 << lb);
    const uint32_t mask = (1u << logN) - 1;
    for (int m = threadIdx.x; m < (1 << lb); m += blockDim.x) lo[m] = twiddle((uint32_t)m, logN);
    for (int m = threadIdx.x; m < (1 << (logN - lb)); m += blockDim.x)
      hi[m] = twiddle(((uint32_t)m << lb) & mask, logN);
  }
  __device__ __forceinline__ cf operator()(uint32_t m) const {
    return cmul(lo[m & ((1u << lb) - 1)], hi[m >> lb]);
  }
};
__host__ __device__ __forceinline__ int big_twiddle_elems(int logN) {
  return (1 << (logN >> 1)) + (1 << (logN - (logN >> 1)));
}

// W_N^(n2 (a + 16 b)), b = 4 q + r < 16, as tq[q] * sr[r]: tq[q] = W_N^(n2 (a + 64 q)) and
// sr[r] = W_N^(16 n2 r) are exact table values (7 lookups), so every twiddle of the radix-16
// column passes is at most two roundings from exact (a 15-step recurrence lost ~1e-6 relative,
// which the 8-layer config-D model amplified past its logits tolerance)
__device__ __forceinline__ void big16(const BigTwiddle& bt, uint32_t n2, uint32_t a, uint32_t mask,
                                      cf (&tq)[4], cf (&sr)[4]) {
#pragma unroll
  for (int q = 0; q < 4; ++q) tq[q] = bt((n2 * (a + 64u * q)) & mask);
  sr[0] = make_float2(1.f, 0.f);
#pragma unroll
  for (int r = 1; r < 4; ++r) sr[r] = bt((n2 * 16u * r) & mask);
}

template <typename T> __device__ __forceinline__ float ld(const T* p, size_t i) { return to_f32(p[i]); }

// Row pairing: pair p (channel-major so consecutive pairs share a filter) of a [B][D][L] tensor.
struct Pairing {
  int B, D, BP;  // BP = ceil(B/2) pairs per channel
  __device__ __forceinline__ void rows(int p, int& d, int& ra, int& rb) const {
    d = p / BP;
    const int bp = p - d * BP;
    ra = (2 * bp) * D + d;
    rb = (2 * bp + 1 < B) ? ra + D : -1;
  }
};

struct Geo {
  int L, logN, logM1, logM2;  // N = 2L = M1 * M2
};
// Kernels are instantiated for fixed transform sizes (LN = log2 N > 0) next to a generic one
// (LN = 0): with the geometry a compile-time constant every LDS address of the Stockham passes
// (sequence, stride, pad slot, twiddle index) folds into immediate offsets instead of per-point
// shift / mask arithmetic with run-time amounts.
template <int LN>
__device__ __forceinline__ Geo fixed(Geo g) {
  if constexpr (LN > 0) {
    g.logN = LN;
    g.logM2 = LN - 1 < 9 ? LN - 1 : 9;
    g.logM1 = LN - g.logM2;
  }
  return g;
}

// Column passes: G = PTS / M1 columns per block (16 at M1 = 512), column stride M1 + 1 (the
// transposing global<->LDS copies then spread over the banks). Row pass: G = PTS / M2 rows.
__host__ __device__ __forceinline__ int log_col_group(const Geo& g) {
  return (LOG_PTS - g.logM1) < g.logM2 ? (LOG_PTS - g.logM1) : g.logM2;  // log2(min(PTS/M1, M2))
}
__host__ __device__ __forceinline__ int log_row_group(const Geo& g) {
  return (LOG_PTS - g.logM2) < g.logM1 ? (LOG_PTS - g.logM2) : g.logM1;      // log2(min(PTS/M2, M1))
}

// ---------------------------------------------------------------- A: column FFT over n1
// src rows [.][L] (dtype T); z[n] = x_a[n - off] + i x_b[n - off] (zero outside [0, L)).
template <typename T, int LN>
__global__ FFT_BOUNDS void col_fwd_kernel(const T* __restrict__ x, Pairing pr, Geo g_,
                                                      int off, cf* __restrict__ ws) {
  const Geo g = fixed<LN>(g_);
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int M1 = 1 << g.logM1, M2 = 1 << g.logM2;
  const int lcw = log_col_group(g), cw = 1 << lcw;
  const int S = seq_stride(g.logM1, true);
  cf* buf = reinterpret_cast<cf*>(smem);  // [cw][S] padded
  cf* tw = buf + cw * S;                   // [M1]
  BigTwiddle bt{tw + M1};
  const int n20 = blockIdx.x * cw;
  const int p = blockIdx.y;
  int d, ra, rb;
  pr.rows(p, d, ra, rb);
  make_table(tw, g.logM1);
  bt.init(g.logN);
  const T* xa = x + (size_t)ra * g.L;
  const T* xb = rb >= 0 ? x + (size_t)rb * g.L : nullptr;
  // 16-B loads: VE consecutive columns of one n1 row of both rows of the pair per load (a chunk
  // never straddles the [0, L) edge when cw, off and L are multiples of VE)
  constexpr int VE = 16 / sizeof(T);
  typedef typename std::conditional<sizeof(T) == 2, bf16x8, f32x4>::type V16;
  if (LN > 0 && cw % VE == 0 && off % VE == 0 && g.L % VE == 0 && cw * M1 == PTS &&
      ((uintptr_t)x & 15) == 0) {
    constexpr int NP = PPT / VE;  // (n1, chunk) pairs per thread
    const int cpr = cw / VE;
    V16 va[NP], vb[NP];
#pragma unroll
    for (int it = 0; it < NP; ++it) {
      const int q = threadIdx.x + it * NTH;
      const int cc = q % cpr, n1 = q / cpr;
      const int i = n1 * M2 + n20 + cc * VE - off;
#pragma unroll
      for (int j = 0; j < VE; ++j) { va[it][j] = T(0.f); vb[it][j] = T(0.f); }
      if (i >= 0 && i < g.L) {
        va[it] = *reinterpret_cast<const V16*>(xa + i);
        if (xb) vb[it] = *reinterpret_cast<const V16*>(xb + i);
      }
    }
#pragma unroll
    for (int it = 0; it < NP; ++it) {
      const int q = threadIdx.x + it * NTH;
      const int cc = q % cpr, n1 = q / cpr;
#pragma unroll
      for (int j = 0; j < VE; ++j)
        buf[lds_at(cc * VE + j, n1, S)] = make_float2(to_f32((T)va[it][j]), to_f32((T)vb[it][j]));
    }
  } else {
    // all PPT loads in flight before the LDS stores (a plain strided loop serialises them)
    cf v[PPT];
#pragma unroll
    for (int it = 0; it < PPT; ++it) {
      const int e = threadIdx.x + it * NTH;
      const int n1 = e >> lcw, c = e & (cw - 1);
      const int i = n1 * M2 + n20 + c - off;
      v[it] = make_float2(0.f, 0.f);
      if (e < cw * M1 && i >= 0 && i < g.L) {
        v[it].x = ld(xa, i);
        if (xb) v[it].y = ld(xb, i);
      }
    }
#pragma unroll
    for (int it = 0; it < PPT; ++it) {
      const int e = threadIdx.x + it * NTH;
      const int n1 = e >> lcw, c = e & (cw - 1);
      if (e < cw * M1) buf[lds_at(c, n1, S)] = v[it];
    }
  }
  __syncthreads();
  const uint32_t mask = (1u << g.logN) - 1;
  if constexpr (LN == 17) {
    // N = 2^17: the 256-point column FFT as two register radix-16 steps (one LDS exchange
    // instead of three Stockham passes; the W_256 twiddles are wave-uniform table reads),
    // n1 = j + 16 r, k1 = ka + 16 kb. Thread (c, j): 16 points of column c at stride 16 ->
    // DFT16 over r, times W_256^(j ka), back to the same slots; thread (c, ka): the 16
    // contiguous slots 16 ka + j -> DFT16 over j = X[ka + 16 kb]; times W_N^(n2 k1) by
    // recurrence over kb; stored straight from registers (32 columns = 256-B row segments).
    static_assert(NTH == 512 && PTS == 8192, "radix-16 column pass geometry");
    const int c = threadIdx.x & 31, j = threadIdx.x >> 5;
    cf* col = buf + c * S;
    cf v[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) v[r] = col[j + 17 * r];  // lds_at(c, j + 16 r, S)
    dft16<false>(v);
#pragma unroll
    for (int ka = 1; ka < 16; ++ka) v[ka] = cmul(v[ka], tw[(j * ka) & 255]);
#pragma unroll
    for (int ka = 0; ka < 16; ++ka) col[j + 17 * ka] = v[ka];
    __syncthreads();
    const int ka = j;
#pragma unroll
    for (int jj = 0; jj < 16; ++jj) v[jj] = col[17 * ka + jj];  // lds_at(c, jj + 16 ka, S)
    dft16<false>(v);
    const uint32_t n2 = (uint32_t)(n20 + c);
    cf tq[4], sr[4];
    big16(bt, n2, (uint32_t)ka, mask, tq, sr);
    cf* out = ws + ((size_t)p << g.logN) + n2;
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int kb = 4 * q + r;
        out[(size_t)(ka + 16 * kb) * M2] = cmul(v[kb], r == 0 ? tq[q] : cmul(tq[q], sr[r]));
      }
    return;
  }
  fft_lds<false>(buf, cw, g.logM1, S, tw);
  cf* out = ws + ((size_t)p << g.logN);
  for (int e = threadIdx.x; e < cw * M1; e += NTH) {
    const int k1 = e >> lcw, c = e & (cw - 1);
    const int n2 = n20 + c;
    out[(size_t)k1 * M2 + n2] = cmul(buf[lds_at(c, k1, S)], bt(((uint32_t)n2 * (uint32_t)k1) & mask));
  }
}

// ---------------------------------------------------------------- B: row FFT over n2
enum RowMode { ROW_SPEC = 0, ROW_MUL = 1, ROW_MULCONJ = 2, ROW_INV = 3, ROW_INV_MULCONJ = 4 };
// ROW_SPEC: FFT, store the spectrum (natural k2). ROW_MUL(CONJ): FFT, times (conj) kspec[d],
// inverse FFT, store. ROW_INV: input is a spectrum (natural k2): inverse FFT, store.
// ROW_INV_MULCONJ: input is a spectrum: times conj kspec[d], inverse FFT, store.
template <int MODE, int LN>
__global__ FFT_BOUNDS void row_kernel(cf* __restrict__ ws, const cf* __restrict__ kspec,
                                      Pairing pr, Geo g_, cf* __restrict__ zsave) {
  const Geo g = fixed<LN>(g_);
  constexpr bool FWD = MODE == ROW_SPEC || MODE == ROW_MUL || MODE == ROW_MULCONJ;
  constexpr bool MUL = MODE == ROW_MUL || MODE == ROW_MULCONJ || MODE == ROW_INV_MULCONJ;
  constexpr bool CONJK = MODE == ROW_MULCONJ || MODE == ROW_INV_MULCONJ;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int M2 = 1 << g.logM2;
  const int lrw = log_row_group(g), rw = 1 << lrw;
  const int S = seq_stride(g.logM2, false);
  cf* buf = reinterpret_cast<cf*>(smem);  // [rw][S] padded
  cf* tw = buf + rw * S;
  const int k10 = blockIdx.x * rw;
  const int p = blockIdx.y;
  make_table(tw, g.logM2);
  cf* base = ws + ((size_t)p << g.logN) + (size_t)k10 * M2;
  {
    cf v[PPT];
#pragma unroll
    for (int it = 0; it < PPT; ++it) {
      const int e = threadIdx.x + it * NTH;
      if (e < rw * M2) v[it] = base[e];
    }
#pragma unroll
    for (int it = 0; it < PPT; ++it) {
      const int e = threadIdx.x + it * NTH;
      if (e < rw * M2) buf[lds_at(e >> g.logM2, e & (M2 - 1), S)] = v[it];
    }
  }
  __syncthreads();
  if (FWD) fft_lds<false>(buf, rw, g.logM2, S, tw);
  if (MODE == ROW_SPEC) {
    for (int e = threadIdx.x; e < rw * M2; e += NTH) base[e] = buf[lds_at(e >> g.logM2, e & (M2 - 1), S)];
    return;
  }
  if (MODE == ROW_MUL && zsave) {  // keep the input spectrum for the backward's dk (no barrier needed)
    cf* zs = zsave + ((size_t)p << g.logN) + (size_t)k10 * M2;
    for (int e = threadIdx.x; e < rw * M2; e += NTH) zs[e] = buf[lds_at(e >> g.logM2, e & (M2 - 1), S)];
  }
  if (MUL) {
    int d = p;
    if (pr.BP > 0) {
      int ra, rb;
      pr.rows(p, d, ra, rb);
    }
    const cf* ks = kspec + ((size_t)d << g.logN) + (size_t)k10 * M2;
#pragma unroll 1
    for (int c0 = 0; c0 < PPT; c0 += 8) {  // 8 spectrum loads in flight (register budget)
      cf kv[8];
#pragma unroll
      for (int it = 0; it < 8; ++it) {
        const int e = threadIdx.x + (c0 + it) * NTH;
        if (e < rw * M2) kv[it] = ks[e];
      }
#pragma unroll
      for (int it = 0; it < 8; ++it) {
        const int e = threadIdx.x + (c0 + it) * NTH;
        const int a = lds_at(e >> g.logM2, e & (M2 - 1), S);
        if (e < rw * M2) buf[a] = cmul(buf[a], CONJK ? cconj(kv[it]) : kv[it]);
      }
    }
    __syncthreads();
  }
  fft_lds<true>(buf, rw, g.logM2, S, tw);
  for (int e = threadIdx.x; e < rw * M2; e += NTH) base[e] = buf[lds_at(e >> g.logM2, e & (M2 - 1), S)];
}

// ---------------------------------------------------------------- B, backward: both gradients
// One row block of channel d, the channel's BP pairs in turn: FFT-M2 of the dy column output ->
// Z_dy, then (DU) Z_dy * conj(K_d), inverse FFT-M2, stored in place (the du column pass reads it),
// and (DK) conj(Z_u) * Z_dy summed over the pairs in registers (each thread owns the same PPT
// points every pair), inverse FFT-M2 of the sum -> pk[d]. Replaces ROW_SPEC + the dk spectrum
// pass + ROW_INV + ROW_INV_MULCONJ: Z_dy never goes to memory, the products see the same fp32
// values in the same order (bit-identical to the four-pass form).
// 256-thread blocks (8 rows of 512 at N = 2^17): the PPT-point sum stays in registers (32 VGPRs
// beside the Stockham pass's 32) without spilling, 3 waves per SIMD.
constexpr int RB_NT = 256, RB_LOG_PTS = LOG_PTS - 1;
__host__ __device__ __forceinline__ int log_rowbwd_group(const Geo& g) {
  return (RB_LOG_PTS - g.logM2) < g.logM1 ? (RB_LOG_PTS - g.logM2) : g.logM1;
}
template <int LN, bool DK, bool DU, int MINB = 3>
__global__ __launch_bounds__(RB_NT, MINB) void row_bwd_kernel(cf* __restrict__ zy, const cf* __restrict__ zu,
                                                           const cf* __restrict__ kspec, int BP, Geo g_,
                                                           cf* __restrict__ pk) {
  const Geo g = fixed<LN>(g_);
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int M2 = 1 << g.logM2;
  const int lrw = log_rowbwd_group(g), rw = 1 << lrw;
  const int S = seq_stride(g.logM2, false);
  cf* buf = reinterpret_cast<cf*>(smem);  // [rw][S] padded
  cf* tw = buf + rw * S;
  const int k10 = blockIdx.x * rw;
  const int d = blockIdx.y;
  const size_t roff = (size_t)k10 * M2;
  make_table(tw, g.logM2);
  static_assert(PPT == 16, "row_bwd_kernel: acc[] in two halves of 8");
  cf acc[PPT];
#pragma unroll
  for (int it = 0; it < PPT; ++it) acc[it] = make_float2(0.f, 0.f);
  const cf* ks = kspec + ((size_t)d << g.logN) + roff;
  for (int bp = 0; bp < BP; ++bp) {
    const int p = d * BP + bp;
    cf* base = zy + ((size_t)p << g.logN) + roff;
    {
      cf v[PPT];
#pragma unroll
      for (int it = 0; it < PPT; ++it) {
        const int e = threadIdx.x + it * RB_NT;
        if (e < rw * M2) v[it] = base[e];
      }
      if (bp > 0) __syncthreads();  // the previous pair's reads / stores of buf are done
#pragma unroll
      for (int it = 0; it < PPT; ++it) {
        const int e = threadIdx.x + it * RB_NT;
        if (e < rw * M2) buf[lds_at(e >> g.logM2, e & (M2 - 1), S)] = v[it];
      }
    }
    __syncthreads();
    fft_lds<false, RB_NT>(buf, rw, g.logM2, S, tw);
    const cf* zup = zu + ((size_t)p << g.logN) + roff;
#pragma unroll 1
    for (int c0 = 0; c0 < PPT; c0 += 8) {  // 8 spectrum loads per operand in flight
      cf uv[8], kv[8];
#pragma unroll
      for (int it = 0; it < 8; ++it) {
        const int e = threadIdx.x + (c0 + it) * RB_NT;
        if (e < rw * M2) {
          if (DK) uv[it] = zup[e];
          if (DU) kv[it] = ks[e];
        }
      }
#pragma unroll
      for (int it = 0; it < 8; ++it) {
        const int e = threadIdx.x + (c0 + it) * RB_NT;
        const int a = lds_at(e >> g.logM2, e & (M2 - 1), S);
        if (e < rw * M2) {
          const cf z = buf[a];
          // (static indices in both arms: a run-time acc[c0 + it] put acc in scratch memory)
          if (DK) {
            if (c0 == 0) acc[it] = cadd(acc[it], cmul(cconj(uv[it]), z));
            else acc[8 + it] = cadd(acc[8 + it], cmul(cconj(uv[it]), z));
          }
          if (DU) buf[a] = cmul(z, cconj(kv[it]));
        }
      }
    }
    if (DU) {
      __syncthreads();
      fft_lds<true, RB_NT>(buf, rw, g.logM2, S, tw);
      for (int e = threadIdx.x; e < rw * M2; e += RB_NT) base[e] = buf[lds_at(e >> g.logM2, e & (M2 - 1), S)];
    }
  }
  if (DK) {
    __syncthreads();  // the last pair's reads / stores of buf are done
#pragma unroll
    for (int it = 0; it < PPT; ++it) {
      const int e = threadIdx.x + it * RB_NT;
      if (e < rw * M2) buf[lds_at(e >> g.logM2, e & (M2 - 1), S)] = acc[it];
    }
    __syncthreads();
    fft_lds<true, RB_NT>(buf, rw, g.logM2, S, tw);
    cf* out = pk + ((size_t)d << g.logN) + roff;
    for (int e = threadIdx.x; e < rw * M2; e += RB_NT) out[e] = buf[lds_at(e >> g.logM2, e & (M2 - 1), S)];
  }
}

// ---------------------------------------------------------------- C: inverse column FFT over k1
enum OutMode { OUT_PAIR = 0, OUT_REAL = 1 };
// OUT_PAIR: rows ra/rb of y get Re/Im at i = n - off for i in [0, L).
// OUT_REAL: row p (= channel) of outf gets Re * scale at i = n for i < L.
template <typename T, int MODE, int LN>
__global__ FFT_BOUNDS void col_inv_kernel(const cf* __restrict__ ws, Pairing pr, Geo g_, int off,
                                          T* __restrict__ y, float* __restrict__ outf, float scale) {
  const Geo g = fixed<LN>(g_);
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int M1 = 1 << g.logM1, M2 = 1 << g.logM2;
  const int lcw = log_col_group(g), cw = 1 << lcw;
  const int S = seq_stride(g.logM1, true);
  cf* buf = reinterpret_cast<cf*>(smem);
  cf* tw = buf + cw * S;
  BigTwiddle bt{tw + M1};
  const int n20 = blockIdx.x * cw;
  const int p = blockIdx.y;
  make_table(tw, g.logM1);
  bt.init(g.logN);
  // the tables' barrier comes after this block's column loads are issued (both from L2 / HBM:
  // a barrier in between serialised the two latencies, ~16 us of the 100-us pass at config D)
  const cf* src = ws + ((size_t)p << g.logN);
  const uint32_t mask = (1u << g.logN) - 1;
  if constexpr (LN == 17) {
    // radix-16 form of the inverse 256-point column FFT (see col_fwd_kernel), k1 = ma + 16 mb,
    // n1 = la + 16 lb: thread (c, ma) loads its 16 rows k1 of column n2 straight into registers
    // (256-B row segments per wave), times conj W_N^(n2 k1) by recurrence, inverse DFT16 over
    // mb, times conj W_256^(ma la), to LDS slots ma + 16 la; thread (c, la): slots 16 la + ma ->
    // inverse DFT16 over ma = z[n1 = la + 16 lb], stored to lds_at(c, n1) for the output copy.
    static_assert(NTH == 512 && PTS == 8192, "radix-16 column pass geometry");
    const int c = threadIdx.x & 31, ma = threadIdx.x >> 5;
    const uint32_t n2 = (uint32_t)(n20 + c);
    cf* col = buf + c * S;
    cf v[16];
#pragma unroll
    for (int mb = 0; mb < 16; ++mb) v[mb] = src[(size_t)(ma + 16 * mb) * M2 + n2];
    __syncthreads();  // twiddle tables
    cf tq[4], sr[4];
    big16(bt, n2, (uint32_t)ma, mask, tq, sr);
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int mb = 4 * q + r;
        v[mb] = cmul(v[mb], cconj(r == 0 ? tq[q] : cmul(tq[q], sr[r])));
      }
    dft16<true>(v);
#pragma unroll
    for (int la = 1; la < 16; ++la) v[la] = cmul(v[la], cconj(tw[(ma * la) & 255]));
#pragma unroll
    for (int la = 0; la < 16; ++la) col[ma + 17 * la] = v[la];  // lds_at(c, ma + 16 la, S)
    __syncthreads();
    const int la = ma;
#pragma unroll
    for (int mm = 0; mm < 16; ++mm) v[mm] = col[17 * la + mm];  // lds_at(c, mm + 16 la, S)
    dft16<true>(v);
    __syncthreads();
#pragma unroll
    for (int lb = 0; lb < 16; ++lb) col[la + 17 * lb] = v[lb];  // lds_at(c, la + 16 lb, S)
  } else {
  {
    cf v[PPT];
#pragma unroll
    for (int it = 0; it < PPT; ++it) {
      const int e = threadIdx.x + it * NTH;
      const int k1 = e >> lcw, c = e & (cw - 1);
      if (e < cw * M1) v[it] = src[(size_t)k1 * M2 + n20 + c];
    }
    __syncthreads();  // twiddle tables
#pragma unroll
    for (int it = 0; it < PPT; ++it) {
      const int e = threadIdx.x + it * NTH;
      const int k1 = e >> lcw, c = e & (cw - 1);
      const int n2 = n20 + c;
      if (e < cw * M1) buf[lds_at(c, k1, S)] = cmul(v[it], cconj(bt(((uint32_t)n2 * (uint32_t)k1) & mask)));
    }
  }
  __syncthreads();
  fft_lds<true>(buf, cw, g.logM1, S, tw);
  }
  __syncthreads();
  if (MODE == OUT_PAIR) {
    int d, ra, rb;
    pr.rows(p, d, ra, rb);
    T* ya = y + (size_t)ra * g.L;
    T* yb = rb >= 0 ? y + (size_t)rb * g.L : nullptr;
    constexpr int VE = 16 / sizeof(T);
    typedef typename std::conditional<sizeof(T) == 2, bf16x8, f32x4>::type V16;
    if (LN > 0 && cw % VE == 0 && off % VE == 0 && g.L % VE == 0 && ((uintptr_t)y & 15) == 0) {
      // 16-B stores: VE consecutive columns of one n1 row (a chunk never straddles [0, L))
      const int cpr = cw / VE;
      for (int q = threadIdx.x; q < M1 * cpr; q += NTH) {
        const int cc = q % cpr, n1 = q / cpr;
        const int i = n1 * M2 + n20 + cc * VE - off;
        if (i < 0 || i >= g.L) continue;
        V16 va, vb;
#pragma unroll
        for (int j = 0; j < VE; ++j) {
          const cf v = buf[lds_at(cc * VE + j, n1, S)];
          va[j] = from_f32<T>(v.x);
          vb[j] = from_f32<T>(v.y);
        }
        *reinterpret_cast<V16*>(ya + i) = va;
        if (yb) *reinterpret_cast<V16*>(yb + i) = vb;
      }
      return;
    }
    for (int e = threadIdx.x; e < cw * M1; e += NTH) {
      const int n1 = e >> lcw, c = e & (cw - 1);
      const int i = n1 * M2 + n20 + c - off;
      if (i < 0 || i >= g.L) continue;
      const cf v = buf[lds_at(c, n1, S)];
      ya[i] = from_f32<T>(v.x);
      if (yb) yb[i] = from_f32<T>(v.y);
    }
  } else {
    if (LN > 0 && cw % 4 == 0 && g.L % 4 == 0 && ((uintptr_t)outf & 15) == 0) {
      const int cpr = cw / 4;  // 16-B stores of 4 consecutive columns
      for (int q = threadIdx.x; q < M1 * cpr; q += NTH) {
        const int cc = q % cpr, n1 = q / cpr;
        const int i = n1 * M2 + n20 + cc * 4;
        if (i >= g.L) continue;
        f32x4 o;
#pragma unroll
        for (int j = 0; j < 4; ++j) o[j] = buf[lds_at(cc * 4 + j, n1, S)].x * scale;
        *reinterpret_cast<f32x4*>(outf + (size_t)p * g.L + i) = o;
      }
      return;
    }
    for (int e = threadIdx.x; e < cw * M1; e += NTH) {
      const int n1 = e >> lcw, c = e & (cw - 1);
      const int i = n1 * M2 + n20 + c;
      if (i >= g.L) continue;
      outf[(size_t)p * g.L + i] = buf[lds_at(c, n1, S)].x * scale;
    }
  }
}

// ---------------------------------------------------------------- B for the filter: row FFT +
// separation in one pass. The separation of Z = FFT(k_{2q} + i k_{2q+1}) (below) pairs bin f
// with N - f, which for f = k1 + M1 k2 lies in row (M1 - k1) mod M1, column M2 - 1 - k2 (k1 != 0)
// or row 0, column (M2 - k2) mod M2 (k1 == 0). A block therefore transforms row pairs
// {j, M1 - j} (j in [j0, j0 + rw/2); j = 0 pairs row 0 with row M1/2, both self-mirrored), so
// every bin's mirror is in its LDS and the spectrum goes straight to kspec: no spectrum round
// trip through HBM and no separate pass (ROW_SPEC + separate_kernel read and wrote 3 N-point
// complex arrays per pair more).
template <int LN>
__global__ FFT_BOUNDS void row_sep_kernel(const cf* __restrict__ ws, const float* __restrict__ bias,
                                          int D, int pad, Geo g_, cf* __restrict__ kspec) {
  const Geo g = fixed<LN>(g_);
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int M1 = 1 << g.logM1, M2 = 1 << g.logM2;
  const int lrw = log_row_group(g), rw = 1 << lrw, h = rw >> 1;
  const int S = seq_stride(g.logM2, false);
  cf* buf = reinterpret_cast<cf*>(smem);  // [rw][S] padded
  cf* tw = buf + rw * S;
  const int j0 = blockIdx.x * h;
  const int q = blockIdx.y;
  auto row_of = [&](int slot) {
    if (slot < h) return j0 + slot;
    const int j = j0 + slot - h;
    return j == 0 ? M1 / 2 : M1 - j;
  };
  make_table(tw, g.logM2);
  const cf* base = ws + ((size_t)q << g.logN);
  {
    cf v[PPT];
#pragma unroll
    for (int it = 0; it < PPT; ++it) {
      const int e = threadIdx.x + it * NTH;
      if (e < rw * M2) v[it] = base[((size_t)row_of(e >> g.logM2) << g.logM2) + (e & (M2 - 1))];
    }
#pragma unroll
    for (int it = 0; it < PPT; ++it) {
      const int e = threadIdx.x + it * NTH;
      if (e < rw * M2) buf[lds_at(e >> g.logM2, e & (M2 - 1), S)] = v[it];
    }
  }
  __syncthreads();
  fft_lds<false>(buf, rw, g.logM2, S, tw);
  const int logN = g.logN;
  const uint32_t mask = (1u << logN) - 1;
  const float sc = 0.5f / (float)(1u << logN);
  const float ba = bias ? bias[2 * q] / (float)(1u << logN) : 0.f;
  const bool has_b = 2 * q + 1 < D;
  const float bb = (bias && has_b) ? bias[2 * q + 1] / (float)(1u << logN) : 0.f;
  cf* ka = kspec + ((size_t)(2 * q) << logN);
  cf* kb = kspec + ((size_t)(2 * q + 1) << logN);
  for (int e = threadIdx.x; e < rw * M2; e += NTH) {
    const int slot = e >> g.logM2, k2 = e & (M2 - 1);
    const int k1 = row_of(slot);
    const int j = j0 + (slot < h ? slot : slot - h);
    const int ms = (j == 0) ? slot : (slot < h ? slot + h : slot - h);
    const int k2m = k1 == 0 ? ((M2 - k2) & (M2 - 1)) : (M2 - 1 - k2);
    const cf a = buf[lds_at(slot, k2, S)], b = cconj(buf[lds_at(ms, k2m, S)]);
    cf sh = make_float2(1.f, 0.f);
    if (pad) {
      const uint32_t f = (uint32_t)k1 + ((uint32_t)k2 << g.logM1);
      sh = cconj(twiddle((f * (uint32_t)pad) & mask, logN));
    }
    const size_t pos = ((size_t)k1 << g.logM2) + k2;
    ka[pos] = make_float2((a.x + b.x) * sc + ba * sh.x, (a.y + b.y) * sc + ba * sh.y);
    if (has_b) {
      const cf dlt = csub(a, b);  // (a - b) / (2i) = (-i/2)(a - b)
      kb[pos] = make_float2(dlt.y * sc + bb * sh.x, -dlt.x * sc + bb * sh.y);
    }
  }
}

// ---------------------------------------------------------------- filter spectrum separation
// Z = FFT(k_{2q} + i k_{2q+1}) in [k1][k2] order -> kspec rows 2q, 2q+1 (scaled 1/N):
//   K_a[f] = (Z[f] + conj Z[N-f]) / 2,   K_b[f] = (Z[f] - conj Z[N-f]) / (2i)
// plus the bias folded in as a filter tap: bias * u[t] = bias * u~[(t + pad) mod N] is tap
// (N - pad) mod N of the circular convolution, i.e. + bias * W_N^(-f * pad) in the spectrum.
__global__ __launch_bounds__(256) void separate_kernel(const cf* __restrict__ ws, const float* __restrict__ bias,
                                                       int D, int pad, Geo g, cf* __restrict__ kspec) {
  const int M1 = 1 << g.logM1, M2 = 1 << g.logM2;
  const int logN = g.logM1 + g.logM2;
  const size_t N = (size_t)1 << logN;
  const uint32_t mask = (uint32_t)N - 1;
  const int q = blockIdx.y;
  const float s = 0.5f / (float)N;
  const float ba = bias ? bias[2 * q] / (float)N : 0.f;
  const float bb = (bias && 2 * q + 1 < D) ? bias[2 * q + 1] / (float)N : 0.f;
  const cf* z = ws + ((size_t)q << logN);
  for (size_t pos = (size_t)blockIdx.x * 256 + threadIdx.x; pos < N; pos += (size_t)gridDim.x * 256) {
    const int k1 = (int)(pos >> g.logM2), k2 = (int)(pos & (M2 - 1));
    const int k1m = k1 == 0 ? 0 : M1 - k1;
    const int k2m = k1 == 0 ? ((M2 - k2) & (M2 - 1)) : (M2 - 1 - k2);
    const cf a = z[pos], b = cconj(z[((size_t)k1m << g.logM2) + k2m]);
    cf sh = make_float2(1.f, 0.f);
    if (pad) {
      const uint32_t f = (uint32_t)k1 + ((uint32_t)k2 << g.logM1);
      sh = cconj(twiddle((f * (uint32_t)pad) & mask, logN));
    }
    kspec[((size_t)(2 * q) << logN) + pos] =
        make_float2((a.x + b.x) * s + ba * sh.x, (a.y + b.y) * s + ba * sh.y);
    if (2 * q + 1 < D) {
      // (a - b) / (2i) = (-i/2)(a - b)
      const cf dlt = csub(a, b);
      kspec[((size_t)(2 * q + 1) << logN) + pos] =
          make_float2(dlt.y * s + bb * sh.x, -dlt.x * s + bb * sh.y);
    }
  }
}

// ---------------------------------------------------------------- dk spectrum: sum over pairs
// P[d][pos] = sum_bp conj(Zu[p(d,bp)][pos]) * Zy[p(d,bp)][pos]   (pairs are channel-major)
__global__ __launch_bounds__(NTH) void dkspec_kernel(const cf* __restrict__ zu, const cf* __restrict__ zy,
                                                     int BP, int logN, cf* __restrict__ P) {
  const size_t N = (size_t)1 << logN;
  const int d = blockIdx.y;
  for (size_t pos = (size_t)blockIdx.x * NTH + threadIdx.x; pos < N; pos += (size_t)gridDim.x * NTH) {
    cf acc = make_float2(0.f, 0.f);
    for (int bp = 0; bp < BP; ++bp) {
      const size_t o = ((size_t)(d * BP + bp) << logN) + pos;
      acc = cadd(acc, cmul(cconj(zu[o]), zy[o]));
    }
    P[((size_t)d << logN) + pos] = acc;
  }
}

// dbias[d] = sum_{b,t} dy[b,d,t] u[b,d,t]: blockIdx.x = channel, blockIdx.y = one of DB_CHUNKS
// slices of the (b, t) range -> partials[d][chunk]; dbias_final sums them in fixed order.
constexpr int DB_CHUNKS = 32;
template <typename T>
__global__ __launch_bounds__(NTH) void dbias_kernel(const T* __restrict__ dy, const T* __restrict__ u,
                                                    int B, int D, int L, float* __restrict__ part) {
  __shared__ float red[NTH / 64];
  const int d = blockIdx.x, ch = blockIdx.y;
  const size_t tot = (size_t)B * L;
  constexpr int VE = 16 / sizeof(T);
  // 16-B path: chunk bounds on multiples of VE, so a VE-run never crosses a row (L % VE == 0)
  const bool vec = L % VE == 0 && (((uintptr_t)dy | (uintptr_t)u) & 15) == 0;
  size_t per = (tot + DB_CHUNKS - 1) / DB_CHUNKS;
  if (vec) per = (per + VE - 1) / VE * VE;
  const size_t beg = min(tot, ch * per), end = min(tot, beg + per);
  float s = 0.f;
  typedef typename std::conditional<sizeof(T) == 2, bf16x8, f32x4>::type V16;
  if (vec) {
    for (size_t q = beg + (size_t)threadIdx.x * VE; q < end; q += (size_t)2 * NTH * VE) {
      V16 a[2], b[2];
#pragma unroll
      for (int u2 = 0; u2 < 2; ++u2) {
        const size_t qq = q + (size_t)u2 * NTH * VE;
        if (qq < end) {
          const size_t o = ((qq / L) * D + d) * (size_t)L + qq % L;
          a[u2] = *reinterpret_cast<const V16*>(dy + o);
          b[u2] = *reinterpret_cast<const V16*>(u + o);
        } else {
#pragma unroll
          for (int j = 0; j < VE; ++j) { a[u2][j] = T(0.f); b[u2][j] = T(0.f); }
        }
      }
#pragma unroll
      for (int u2 = 0; u2 < 2; ++u2)
#pragma unroll
        for (int j = 0; j < VE; ++j) s += to_f32((T)a[u2][j]) * to_f32((T)b[u2][j]);
    }
  } else
  for (size_t q = beg + threadIdx.x; q < end; q += 4 * NTH) {
    float a[4], b[4];
#pragma unroll
    for (int u4 = 0; u4 < 4; ++u4) {
      const size_t qq = q + (size_t)u4 * NTH;
      a[u4] = b[u4] = 0.f;
      if (qq < end) {
        const size_t o = ((qq / L) * D + d) * (size_t)L + qq % L;
        a[u4] = to_f32(dy[o]);
        b[u4] = to_f32(u[o]);
      }
    }
#pragma unroll
    for (int u4 = 0; u4 < 4; ++u4) s += a[u4] * b[u4];
  }
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    float t = 0.f;
    for (int w = 0; w < NTH / 64; ++w) t += red[w];
    part[d * DB_CHUNKS + ch] = t;
  }
}

__global__ void dbias_final(const float* __restrict__ part, int D, float* __restrict__ dbias) {
  const int d = blockIdx.x * blockDim.x + threadIdx.x;
  if (d >= D) return;
  float t = 0.f;
  for (int c = 0; c < DB_CHUNKS; ++c) t += part[d * DB_CHUNKS + c];
  dbias[d] = t;
}

inline bool geometry(int L, Geo& g) {
  if (L < 64 || (L & (L - 1))) return false;
  int logN = 0;
  while ((1 << logN) < 2 * L) ++logN;
  if (logN > 18) return false;
  g.L = L;
  g.logN = logN;
  g.logM2 = logN - 1 < 9 ? logN - 1 : 9;  // N = 2^17 -> 256 x 512
  g.logM1 = logN - g.logM2;
  return true;
}

inline size_t col_lds(const Geo& g) {
  return ((size_t)(1 << log_col_group(g)) * seq_stride(g.logM1, true) + (1u << g.logM1) +
          big_twiddle_elems(g.logN)) * sizeof(cf);
}
inline size_t row_lds(const Geo& g) {
  return ((size_t)(1 << log_row_group(g)) * seq_stride(g.logM2, false) + (1u << g.logM2)) * sizeof(cf);
}
inline dim3 col_grid(const Geo& g, int P) { return dim3(1 << (g.logM2 - log_col_group(g)), P); }
inline dim3 row_grid(const Geo& g, int P) { return dim3(1 << (g.logM1 - log_row_group(g)), P); }

template <typename Kern>
inline void allow_lds(Kern k, size_t bytes) {
  if (bytes > 65536) (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
}

// instantiated sizes: N = 2^16 .. 2^18 (L = 32,768 .. 131,072: HyenaDNA's long configs, config D
// at 2^17); every other size runs the generic kernels. DNA_FFT_GENERIC=1 forces those (A/B).
inline int fixed_ln(const Geo& g) {
  static const bool generic = getenv("DNA_FFT_GENERIC") && atoi(getenv("DNA_FFT_GENERIC")) == 1;
  return (!generic && g.logN >= 16 && g.logN <= 18) ? g.logN : 0;
}
#define DNA_FFT_DISPATCH(LAUNCH)      \
  switch (fixed_ln(g)) {              \
    case 16: LAUNCH(16); break;       \
    case 17: LAUNCH(17); break;       \
    case 18: LAUNCH(18); break;       \
    default: LAUNCH(0); break;        \
  }

template <typename T>
int launch_col_fwd(const void* x, Pairing pr, const Geo& g, int off, cf* ws, int P, hipStream_t s) {
#define L_(LN)                                                                                    \
  {                                                                                               \
    auto k = col_fwd_kernel<T, LN>;                                                               \
    allow_lds(k, col_lds(g));                                                                     \
    hipLaunchKernelGGL(k, col_grid(g, P), dim3(NTH), col_lds(g), s, (const T*)x, pr, g, off, ws); \
  }
  DNA_FFT_DISPATCH(L_)
#undef L_
  return DNA_OK;
}

template <int MODE>
void launch_row(cf* ws, const cf* kspec, Pairing pr, const Geo& g, int P, hipStream_t s,
                cf* zsave = nullptr) {
#define L_(LN)                                                                                  \
  {                                                                                             \
    auto k = row_kernel<MODE, LN>;                                                              \
    allow_lds(k, row_lds(g));                                                                   \
    hipLaunchKernelGGL(k, row_grid(g, P), dim3(NTH), row_lds(g), s, ws, kspec, pr, g, zsave); \
  }
  DNA_FFT_DISPATCH(L_)
#undef L_
}

template <bool DK, bool DU>
void launch_row_bwd(cf* zy, const cf* zu, const cf* kspec, int BP, int D, const Geo& g, cf* pk,
                    hipStream_t s) {
  // DNA_FFT_RB_BLOCKS=4 / 2 (A/B): four blocks per CU (128 VGPRs, spills) or two (256 VGPRs)
  // instead of three
  static const int rbb = getenv("DNA_FFT_RB_BLOCKS") ? atoi(getenv("DNA_FFT_RB_BLOCKS")) : 3;
#define L_(LN)                                                                                   \
  {                                                                                              \
    auto k = (DK && DU && rbb == 4)   ? row_bwd_kernel<LN, DK, DU, 4>                            \
             : (DK && DU && rbb == 2) ? row_bwd_kernel<LN, DK, DU, 2>                            \
                                      : row_bwd_kernel<LN, DK, DU>;                              \
    const size_t lds = ((size_t)(1 << log_rowbwd_group(g)) * seq_stride(g.logM2, false) +        \
                        (1u << g.logM2)) * sizeof(cf);                                           \
    allow_lds(k, lds);                                                                           \
    hipLaunchKernelGGL(k, dim3(1 << (g.logM1 - log_rowbwd_group(g)), D), dim3(RB_NT), lds, s, zy, \
                       zu, kspec, BP, g, pk);                                                    \
  }
  DNA_FFT_DISPATCH(L_)
#undef L_
}

template <typename T, int MODE>
void launch_col_inv(const cf* ws, Pairing pr, const Geo& g, int off, void* y, float* outf, float scale,
                    int P, hipStream_t s) {
#define L_(LN)                                                                                                  \
  {                                                                                                             \
    auto k = col_inv_kernel<T, MODE, LN>;                                                                       \
    allow_lds(k, col_lds(g));                                                                                   \
    hipLaunchKernelGGL(k, col_grid(g, P), dim3(NTH), col_lds(g), s, ws, pr, g, off, (T*)y, outf, scale);        \
  }
  DNA_FFT_DISPATCH(L_)
#undef L_
}

inline int pad_before(int L, int bidirectional) {
  if (!bidirectional) return 0;
  const int padded = L + 2 * (L / 2);
  return padded / 2 - L / 2;
}

}  // namespace fftc
}  // namespace dna

using namespace dna;
using namespace dna::fftc;

// Upload g_w18 once per device (immutable afterwards). Synchronous: nothing can be using the
// table before its first upload on that device.
static int ensure_twiddles() {
  static std::mutex mu;
  static bool done[64] = {};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) {
    set_error("fftconv: hipGetDevice failed");
    return DNA_ERR_HIP;
  }
  std::lock_guard<std::mutex> lock(mu);
  if (done[dev]) return DNA_OK;
  std::vector<cf> h((size_t)1 << LOG_TW);
  const double step = -2.0 * M_PI / (double)((size_t)1 << LOG_TW);
  for (size_t j = 0; j < h.size(); ++j) h[j] = make_float2((float)cos(step * (double)j), (float)sin(step * (double)j));
  if (hipMemcpyToSymbol(HIP_SYMBOL(g_w18), h.data(), h.size() * sizeof(cf)) != hipSuccess) {
    set_error("fftconv: twiddle table upload failed");
    return DNA_ERR_HIP;
  }
  done[dev] = true;
  return DNA_OK;
}

extern "C" size_t dna_fftconv_workspace(int B, int D, int L) {
  Geo g;
  if (B <= 0 || D <= 0 || !geometry(L, g)) return 0;
  const size_t N = (size_t)1 << g.logN;
  const size_t P = (size_t)((B + 1) / 2) * D;
  // forward: P spectra; backward: 2P spectra (u and dy) + D accumulated dk spectra
  return (2 * P + (size_t)D + (size_t)(D + 1) / 2) * N * sizeof(cf);
}

extern "C" size_t dna_fftconv_kspec_elems(int L) {
  Geo g;
  if (!geometry(L, g)) return 0;
  return (size_t)2 << g.logN;  // floats per channel (complex N)
}

extern "C" int dna_fftconv_filter(const float* k, const float* bias, int D, int L, int bidirectional,
                                  void* kspec, void* ws, size_t ws_bytes, void* stream) {
  Geo g;
  DNA_CHECK_ARG(k && kspec && ws, "dna_fftconv_filter: null pointer");
  DNA_CHECK_ARG(D > 0 && geometry(L, g), "dna_fftconv_filter: L=%d must be a power of 2 in [64, 131072]", L);
  const size_t N = (size_t)1 << g.logN;
  const int Q = (D + 1) / 2;
  DNA_CHECK_ARG(ws_bytes >= (size_t)Q * N * sizeof(cf), "dna_fftconv_filter: workspace too small");
  if (int st = ensure_twiddles()) return st;
  hipStream_t s = as_stream(stream);
  Pairing pr{D, 1, Q};  // channels paired (2q, 2q+1)
  cf* w = (cf*)ws;
  launch_col_fwd<float>(k, pr, g, 0, w, Q, s);
  const int pad = pad_before(L, bidirectional);
  static const bool unfused = getenv("DNA_FFT_FILTER_SEPARATE") && atoi(getenv("DNA_FFT_FILTER_SEPARATE")) == 1;
  if (unfused) {  // the unfused ROW_SPEC + separate form (A/B)
    launch_row<ROW_SPEC>(w, nullptr, pr, g, Q, s);
    const int bx = (int)((N + 255) / 256) < 1024 ? (int)((N + 255) / 256) : 1024;
    hipLaunchKernelGGL(separate_kernel, dim3(bx, Q), dim3(256), 0, s, (const cf*)w, bias, D, pad,
                       g, (cf*)kspec);
  } else {
#define L_(LN)                                                                                 \
    {                                                                                          \
      auto kk = row_sep_kernel<LN>;                                                            \
      allow_lds(kk, row_lds(g));                                                               \
      hipLaunchKernelGGL(kk, dim3(1 << (g.logM1 - log_row_group(g)), Q), dim3(NTH), row_lds(g), \
                         s, (const cf*)w, bias, D, pad, g, (cf*)kspec);                        \
    }
    DNA_FFT_DISPATCH(L_)
#undef L_
  }
  DNA_LAUNCH_CHECK("dna_fftconv_filter");
  return DNA_OK;
}

extern "C" int dna_fftconv_fwd(const void* u, int dtype, const void* kspec, int B, int D, int L,
                               int bidirectional, void* y, void* uspec, void* ws, size_t ws_bytes,
                               void* stream) {
  Geo g;
  DNA_CHECK_ARG(u && kspec && y && ws, "dna_fftconv_fwd: null pointer");
  DNA_CHECK_ARG(B > 0 && D > 0 && geometry(L, g), "dna_fftconv_fwd: L=%d must be a power of 2 in [64, 131072]", L);
  const size_t N = (size_t)1 << g.logN;
  const int BP = (B + 1) / 2, P = BP * D;
  DNA_CHECK_ARG(ws_bytes >= (size_t)P * N * sizeof(cf), "dna_fftconv_fwd: workspace too small");
  if (int st = ensure_twiddles()) return st;
  hipStream_t s = as_stream(stream);
  Pairing pr{B, D, BP};
  cf* w = (cf*)ws;
  const int pb = pad_before(L, bidirectional);
  if (dtype == DNA_BF16) {
    launch_col_fwd<bf16>(u, pr, g, pb, w, P, s);
    launch_row<ROW_MUL>(w, (const cf*)kspec, pr, g, P, s, (cf*)uspec);
    launch_col_inv<bf16, OUT_PAIR>(w, pr, g, 0, y, nullptr, 1.f, P, s);
  } else if (dtype == DNA_F32) {
    launch_col_fwd<float>(u, pr, g, pb, w, P, s);
    launch_row<ROW_MUL>(w, (const cf*)kspec, pr, g, P, s, (cf*)uspec);
    launch_col_inv<float, OUT_PAIR>(w, pr, g, 0, y, nullptr, 1.f, P, s);
  } else {
    DNA_CHECK_ARG(false, "dna_fftconv_fwd: bad dtype");
  }
  DNA_LAUNCH_CHECK("dna_fftconv_fwd");
  return DNA_OK;
}

template <typename T>
static void bwd_impl(const void* dy, const void* u, const cf* kspec, const cf* uspec, int B, int D,
                     const Geo& g, int pb, void* du, float* dk, float* dbias, cf* ws, hipStream_t s) {
  const size_t N = (size_t)1 << g.logN;
  const int BP = (B + 1) / 2, P = BP * D;
  Pairing pr{B, D, BP};
  cf* zu = ws;
  cf* zy = ws + (size_t)P * N;
  cf* pk = ws + (size_t)2 * P * N;
  // spectra of u~ and of dy (padded at the end)
  if (dk && !uspec) {
    launch_col_fwd<T>(u, pr, g, pb, zu, P, s);
    launch_row<ROW_SPEC>(zu, nullptr, pr, g, P, s);
  }
  const cf* zuc = uspec ? uspec : zu;
  launch_col_fwd<T>(dy, pr, g, 0, zy, P, s);
  static const bool split = getenv("DNA_FFT_BWD_SPLIT") && atoi(getenv("DNA_FFT_BWD_SPLIT")) == 1;
  Pairing one{D, 1, 0};  // BP = 0: row index is the channel
  if (!split) {
    // one row pass for both gradients (row_bwd_kernel): zy -> du column input in place, pk
    if (dk && du) launch_row_bwd<true, true>(zy, zuc, kspec, BP, D, g, pk, s);
    else if (dk) launch_row_bwd<true, false>(zy, zuc, kspec, BP, D, g, pk, s);
    else if (du) launch_row_bwd<false, true>(zy, zuc, kspec, BP, D, g, pk, s);
    if (dk) launch_col_inv<float, OUT_REAL>(pk, one, g, 0, nullptr, dk, 1.f / (float)N, D, s);
    if (du) launch_col_inv<T, OUT_PAIR>(zy, pr, g, pb, du, nullptr, 1.f, P, s);
  } else {  // DNA_FFT_BWD_SPLIT=1 (A/B): the four-pass form
    launch_row<ROW_SPEC>(zy, nullptr, pr, g, P, s);
    if (dk) {
      const int bx = (int)((N + NTH - 1) / NTH) < 512 ? (int)((N + NTH - 1) / NTH) : 512;
      hipLaunchKernelGGL(dkspec_kernel, dim3(bx, D), dim3(NTH), 0, s, zuc, (const cf*)zy, BP,
                         g.logN, pk);
      launch_row<ROW_INV>(pk, nullptr, one, g, D, s);
      launch_col_inv<float, OUT_REAL>(pk, one, g, 0, nullptr, dk, 1.f / (float)N, D, s);
    }
    if (du) {
      // du~ = IFFT(DY * conj(K')) with the bias tap in K'; du = du~[pb : pb + L]  (zy consumed in place)
      launch_row<ROW_INV_MULCONJ>(zy, kspec, pr, g, P, s);
      launch_col_inv<T, OUT_PAIR>(zy, pr, g, pb, du, nullptr, 1.f, P, s);
    }
  }
  if (dbias) {
    // partials live after the dk spectra in the workspace
    float* part = reinterpret_cast<float*>(ws + (2 * (size_t)P + D) * N);
    hipLaunchKernelGGL(dbias_kernel<T>, dim3(D, DB_CHUNKS), dim3(NTH), 0, s, (const T*)dy, (const T*)u, B,
                       D, g.L, part);
    hipLaunchKernelGGL(dbias_final, dim3((D + 255) / 256), dim3(256), 0, s, (const float*)part, D, dbias);
  }
}

extern "C" int dna_fftconv_bwd(const void* dy, const void* u, int dtype, const void* kspec,
                               const void* uspec, int B, int D, int L, int bidirectional, void* du,
                               float* dk, float* dbias, void* ws, size_t ws_bytes, void* stream) {
  Geo g;
  DNA_CHECK_ARG(dy && u && kspec && ws, "dna_fftconv_bwd: null pointer");
  DNA_CHECK_ARG(B > 0 && D > 0 && geometry(L, g), "dna_fftconv_bwd: L=%d must be a power of 2 in [64, 131072]", L);
  const size_t N = (size_t)1 << g.logN;
  const size_t P = (size_t)((B + 1) / 2) * D;
  DNA_CHECK_ARG(ws_bytes >= (2 * P + (size_t)D) * N * sizeof(cf) + (size_t)D * DB_CHUNKS * sizeof(float),
                "dna_fftconv_bwd: workspace too small");
  if (int st = ensure_twiddles()) return st;
  const int pb = pad_before(L, bidirectional);
  hipStream_t s = as_stream(stream);
  if (dtype == DNA_BF16)
    bwd_impl<bf16>(dy, u, (const cf*)kspec, (const cf*)uspec, B, D, g, pb, du, dk, dbias, (cf*)ws, s);
  else if (dtype == DNA_F32)
    bwd_impl<float>(dy, u, (const cf*)kspec, (const cf*)uspec, B, D, g, pb, du, dk, dbias, (cf*)ws, s);
  else
    DNA_CHECK_ARG(false, "dna_fftconv_bwd: bad dtype");
  DNA_LAUNCH_CHECK("dna_fftconv_bwd");
  return DNA_OK;
}
