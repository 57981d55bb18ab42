// FFT long convolution of the HyenaDNA filter (reference src/models/sequence/hyena.py:60-92,
// called from HyenaFilter.forward :253-280), forward and backward, gfx950.
//
//   y[r, t] = sum_{j<L} k[d, j] * u~[r, (t - j) mod N] + bias[d] * u[r, t],  t < L,  N = 2L
// for rows r = (b, d) of u [B, D, L]; u~ is u zero-padded to N (causal: at offset 0,
// bidirectional: at offset pad_before = L/2 -- the reference's F.pad then rfft(n=2L)).
//
// Layout and passes. N = M1 * M2 (M2 = 256 for N >= 512, M1 <= 1024). Two rows with the same
// filter (batches b, b+1 of channel d) are packed into ONE complex sequence z = u~_b + i u~_{b+1};
// since the filter is real, IFFT(Z * K) = (u~_b * k) + i (u~_{b+1} * k) -- no separation step.
// With n = n1*M2 + n2 and k = k1 + M1*k2 (four-step / Bailey):
//   A  column pass: for each column n2, FFT-M1 over n1 (LDS-staged, CW columns per block so the
//      global reads/writes are CW*8-byte row segments), times W_N^(n2*k1) -> T[k1][n2]
//   B  row pass:    for each row k1, FFT-M2 over n2 -> spectrum Z[k1 + M1*k2], times the filter
//      spectrum (stored in the same [k1][k2] order, 1/N folded in), inverse FFT-M2 -> T'[k1][n2]
//   C  column pass: times W_N^-(n2*k1), inverse FFT-M1 over k1 -> z[n1*M2 + n2]; epilogue adds
//      bias*u and writes rows b, b+1 (real, imaginary part) for t < L.
// FFTs are radix-2 in LDS with an LDS twiddle table (W_M^m, m < M/2, from sincospi); the
// inter-pass twiddles W_N^(n2*k1) come from sincospi of an exactly-representable argument.
// Backward: du runs the same three passes on dy (offset 0) with conj(K) and reads the output at
// offset pad_before; dk = Re IFFT(sum_pairs conj(Z_u) Z_dy) / N (the packed pair's cross terms are
// purely imaginary after the inverse transform), j < L; dbias = sum_{b,t} dy u.
// All arithmetic fp32; inputs/outputs fp32 or bf16 (u, y, dy, du), filters and grads fp32.
#include <math.h>

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

// exp(-2 pi i m / N) for integer m in [0, N): the sincospi argument 2m/N is exact in fp32.
__device__ __forceinline__ cf twiddle(uint32_t m, int logN) {
  float s, c;
  sincospif(-2.0f * (float)m / (float)(1u << logN), &s, &c);
  return make_float2(c, s);
}

__device__ __forceinline__ int brev(int i, int bits) { return (int)(__brev((unsigned)i) >> (32 - bits)); }

// LDS twiddle table tw[m] = W_M^m, m < M/2.
__device__ __forceinline__ void make_table(cf* tw, int logM) {
  const int half = 1 << (logM - 1);
  for (int m = threadIdx.x; m < half; m += blockDim.x) tw[m] = twiddle(m, logM);
}

// G independent in-place radix-2 FFTs of length M = 2^logM on buf[g*stride + i].
// DIT: input in bit-reversed order, output natural. INV uses conj twiddles (unscaled).
template <bool INV>
__device__ void fft_dit(cf* buf, int G, int logM, const cf* tw, int stride) {
  const int M = 1 << logM, halfM = M >> 1;
  const int nb = G * halfM;
  for (int s = 0; s < logM; ++s) {
    const int h = 1 << s;
    const int tstep = logM - 1 - s;  // twiddle index = pos << tstep
    for (int idx = threadIdx.x; idx < nb; idx += blockDim.x) {
      const int g = idx >> (logM - 1), j = idx & (halfM - 1);
      const int pos = j & (h - 1), grp = j >> s;
      const int i0 = g * stride + (grp << (s + 1)) + pos, i1 = i0 + h;
      cf w = tw[pos << tstep];
      if (INV) w.y = -w.y;
      const cf a = buf[i0], b = cmul(buf[i1], w);
      buf[i0] = cadd(a, b);
      buf[i1] = csub(a, b);
    }
    __syncthreads();
  }
}

// DIF: input natural order, output bit-reversed.
template <bool INV>
__device__ void fft_dif(cf* buf, int G, int logM, const cf* tw, int stride) {
  const int M = 1 << logM, halfM = M >> 1;
  const int nb = G * halfM;
  for (int s = logM - 1; s >= 0; --s) {
    const int h = 1 << s;
    const int tstep = logM - 1 - s;
    for (int idx = threadIdx.x; idx < nb; idx += blockDim.x) {
      const int g = idx >> (logM - 1), j = idx & (halfM - 1);
      const int pos = j & (h - 1), grp = j >> s;
      const int i0 = g * stride + (grp << (s + 1)) + pos, i1 = i0 + h;
      cf w = tw[pos << tstep];
      if (INV) w.y = -w.y;
      const cf a = buf[i0], b = buf[i1];
      buf[i0] = cadd(a, b);
      buf[i1] = cmul(csub(a, b), w);
    }
    __syncthreads();
  }
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

constexpr int CW = 16;      // columns per block in the column passes
constexpr int NTH = 256;

// ---------------------------------------------------------------- A: column FFT over n1
// src rows [.][L] (dtype T); z[n] = x_a[n - off] + i x_b[n - off] (zero outside [0, L)).
template <typename T>
__global__ __launch_bounds__(NTH) void col_fwd_kernel(const T* __restrict__ x, Pairing pr, Geo g,
                                                      int off, cf* __restrict__ ws) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int M1 = 1 << g.logM1, M2 = 1 << g.logM2;
  const int cw = min(CW, M2);
  const int S = M1 + 1;                    // padded column stride (bank spread)
  cf* buf = reinterpret_cast<cf*>(smem);  // [cw][S]
  cf* tw = buf + cw * S;                   // [M1/2]
  const int n20 = blockIdx.x * cw;
  const int p = blockIdx.y;
  int d, ra, rb;
  pr.rows(p, d, ra, rb);
  make_table(tw, g.logM1);
  const T* xa = x + (size_t)ra * g.L;
  const T* xb = rb >= 0 ? x + (size_t)rb * g.L : nullptr;
  for (int e = threadIdx.x; e < cw * M1; e += NTH) {
    const int n1 = e / cw, c = e - n1 * cw;
    const int i = n1 * M2 + n20 + c - off;
    cf v = make_float2(0.f, 0.f);
    if (i >= 0 && i < g.L) {
      v.x = ld(xa, i);
      if (xb) v.y = ld(xb, i);
    }
    buf[c * S + brev(n1, g.logM1)] = v;
  }
  __syncthreads();
  fft_dit<false>(buf, cw, g.logM1, tw, S);
  cf* out = ws + ((size_t)p << (g.logM1 + g.logM2));
  const int logN = g.logM1 + g.logM2;
  for (int e = threadIdx.x; e < cw * M1; e += NTH) {
    const int k1 = e / cw, c = e - k1 * cw;
    const int n2 = n20 + c;
    const uint32_t m = ((uint32_t)n2 * (uint32_t)k1) & ((1u << logN) - 1);
    out[(size_t)k1 * M2 + n2] = cmul(buf[c * S + k1], twiddle(m, logN));
  }
}

// ---------------------------------------------------------------- B: row FFT over n2
enum RowMode { ROW_SPEC = 0, ROW_MUL = 1, ROW_MULCONJ = 2, ROW_INV = 3, ROW_INV_MULCONJ = 4 };
// ROW_SPEC: FFT, store the spectrum (natural k2). ROW_MUL(CONJ): FFT, times (conj) kspec[d],
// inverse FFT, store. ROW_INV: input is a spectrum (natural k2): inverse FFT, store.
// ROW_INV_MULCONJ: input is a spectrum: times conj kspec[d], inverse FFT, store.
template <int MODE>
__global__ __launch_bounds__(NTH) void row_kernel(cf* __restrict__ ws, const cf* __restrict__ kspec,
                                                  Pairing pr, Geo g) {
  constexpr bool FWD = MODE == ROW_SPEC || MODE == ROW_MUL || MODE == ROW_MULCONJ;
  constexpr bool MUL = MODE == ROW_MUL || MODE == ROW_MULCONJ || MODE == ROW_INV_MULCONJ;
  constexpr bool CONJK = MODE == ROW_MULCONJ || MODE == ROW_INV_MULCONJ;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int M1 = 1 << g.logM1, M2 = 1 << g.logM2;
  const int rw = max(1, 2048 >> g.logM2);  // rows per block
  cf* buf = reinterpret_cast<cf*>(smem);   // [rw][M2]
  cf* tw = buf + rw * M2;
  const int k10 = blockIdx.x * rw;
  const int p = blockIdx.y;
  const int nrow = min(rw, M1 - k10);
  make_table(tw, g.logM2);
  cf* base = ws + ((size_t)p << (g.logM1 + g.logM2)) + (size_t)k10 * M2;
  for (int e = threadIdx.x; e < nrow * M2; e += NTH) {
    const int r = e >> g.logM2, n = e & (M2 - 1);
    const int dst = FWD ? brev(n, g.logM2) : n;
    buf[r * M2 + dst] = base[e];
  }
  __syncthreads();
  if (FWD) fft_dit<false>(buf, nrow, g.logM2, tw, M2);
  if (MODE == ROW_SPEC) {
    for (int e = threadIdx.x; e < nrow * M2; e += NTH) base[e] = buf[e];
    return;
  }
  if (MUL) {
    int d = p;
    if (pr.BP > 0) {
      int ra, rb;
      pr.rows(p, d, ra, rb);
    }
    const cf* ks = kspec + ((size_t)d << (g.logM1 + g.logM2)) + (size_t)k10 * M2;
    for (int e = threadIdx.x; e < nrow * M2; e += NTH) {
      cf kv = ks[e];
      if (CONJK) kv = cconj(kv);
      buf[e] = cmul(buf[e], kv);
    }
    __syncthreads();
  }
  fft_dif<true>(buf, nrow, g.logM2, tw, M2);
  for (int e = threadIdx.x; e < nrow * M2; e += NTH) {
    const int r = e >> g.logM2, n = e & (M2 - 1);
    base[e] = buf[r * M2 + brev(n, g.logM2)];
  }
}

// ---------------------------------------------------------------- C: inverse column FFT over k1
enum OutMode { OUT_PAIR = 0, OUT_REAL = 1 };
// OUT_PAIR: rows ra/rb of y get Re/Im at i = n - off for i in [0, L), plus bias[d] * aux[i].
// OUT_REAL: row p (= channel) of outf gets Re * scale at i = n for i < L.
template <typename T, int MODE>
__global__ __launch_bounds__(NTH) void col_inv_kernel(const cf* __restrict__ ws, Pairing pr, Geo g,
                                                      int off, const float* __restrict__ bias,
                                                      const T* __restrict__ aux, T* __restrict__ y,
                                                      float* __restrict__ outf, float scale) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int M1 = 1 << g.logM1, M2 = 1 << g.logM2;
  const int cw = min(CW, M2);
  const int S = M1 + 1;
  cf* buf = reinterpret_cast<cf*>(smem);
  cf* tw = buf + cw * S;
  const int n20 = blockIdx.x * cw;
  const int p = blockIdx.y;
  const int logN = g.logM1 + g.logM2;
  make_table(tw, g.logM1);
  const cf* src = ws + ((size_t)p << logN);
  for (int e = threadIdx.x; e < cw * M1; e += NTH) {
    const int k1 = e / cw, c = e - k1 * cw;
    const int n2 = n20 + c;
    const uint32_t m = ((uint32_t)n2 * (uint32_t)k1) & ((1u << logN) - 1);
    buf[c * S + brev(k1, g.logM1)] = cmul(src[(size_t)k1 * M2 + n2], cconj(twiddle(m, logN)));
  }
  __syncthreads();
  fft_dit<true>(buf, cw, g.logM1, tw, S);
  if (MODE == OUT_PAIR) {
    int d, ra, rb;
    pr.rows(p, d, ra, rb);
    const float bd = bias ? bias[d] : 0.f;
    for (int e = threadIdx.x; e < cw * M1; e += NTH) {
      const int n1 = e / cw, c = e - n1 * cw;
      const int i = n1 * M2 + n20 + c - off;
      if (i < 0 || i >= g.L) continue;
      const cf v = buf[c * S + n1];
      const size_t ia = (size_t)ra * g.L + i;
      y[ia] = from_f32<T>(v.x + bd * (aux ? to_f32(aux[ia]) : 0.f));
      if (rb >= 0) {
        const size_t ib = (size_t)rb * g.L + i;
        y[ib] = from_f32<T>(v.y + bd * (aux ? to_f32(aux[ib]) : 0.f));
      }
    }
  } else {
    for (int e = threadIdx.x; e < cw * M1; e += NTH) {
      const int n1 = e / cw, c = e - n1 * cw;
      const int i = n1 * M2 + n20 + c;
      if (i >= g.L) continue;
      outf[(size_t)p * g.L + i] = buf[c * S + n1].x * scale;
    }
  }
}

// ---------------------------------------------------------------- filter spectrum separation
// Z = FFT(k_{2q} + i k_{2q+1}) in [k1][k2] order -> kspec rows 2q, 2q+1 (scaled 1/N):
//   K_a[k] = (Z[k] + conj Z[N-k]) / 2,   K_b[k] = (Z[k] - conj Z[N-k]) / (2i)
__global__ __launch_bounds__(NTH) void separate_kernel(const cf* __restrict__ ws, int D, Geo g,
                                                       cf* __restrict__ kspec) {
  const int M1 = 1 << g.logM1, M2 = 1 << g.logM2;
  const int logN = g.logM1 + g.logM2;
  const size_t N = (size_t)1 << logN;
  const int q = blockIdx.y;
  const float s = 0.5f / (float)N;
  const cf* z = ws + ((size_t)q << logN);
  for (size_t pos = (size_t)blockIdx.x * NTH + threadIdx.x; pos < N; pos += (size_t)gridDim.x * NTH) {
    const int k1 = (int)(pos >> g.logM2), k2 = (int)(pos & (M2 - 1));
    const int k1m = k1 == 0 ? 0 : M1 - k1;
    const int k2m = k1 == 0 ? ((M2 - k2) & (M2 - 1)) : (M2 - 1 - k2);
    const cf a = z[pos], b = cconj(z[((size_t)k1m << g.logM2) + k2m]);
    kspec[((size_t)(2 * q) << logN) + pos] = make_float2((a.x + b.x) * s, (a.y + b.y) * s);
    if (2 * q + 1 < D) {
      // (a - b) / (2i) = (-i/2)(a - b)
      const cf dlt = csub(a, b);
      kspec[((size_t)(2 * q + 1) << logN) + pos] = make_float2(dlt.y * s, -dlt.x * s);
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

// dbias[d] = sum_{b,t} dy[b,d,t] u[b,d,t]   (one block per channel, fixed order)
template <typename T>
__global__ __launch_bounds__(NTH) void dbias_kernel(const T* __restrict__ dy, const T* __restrict__ u,
                                                    int B, int D, int L, float* __restrict__ dbias) {
  __shared__ float red[NTH / 64];
  const int d = blockIdx.x;
  float s = 0.f;
  for (int b = 0; b < B; ++b) {
    const size_t o = ((size_t)b * D + d) * L;
    for (int t = threadIdx.x; t < L; t += NTH) s += to_f32(dy[o + t]) * to_f32(u[o + t]);
  }
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    float t = 0.f;
    for (int w = 0; w < NTH / 64; ++w) t += red[w];
    dbias[d] = t;
  }
}

inline bool geometry(int L, Geo& g) {
  if (L < 64 || (L & (L - 1))) return false;
  int logN = 0;
  while ((1 << logN) < 2 * L) ++logN;
  if (logN > 18) return false;
  g.L = L;
  g.logN = logN;
  g.logM2 = logN - 1 < 8 ? logN - 1 : 8;
  g.logM1 = logN - g.logM2;
  return true;
}

inline size_t col_lds(const Geo& g) {
  const int cw = (1 << g.logM2) < CW ? (1 << g.logM2) : CW;
  return ((size_t)cw * ((1u << g.logM1) + 1) + (1u << (g.logM1 - 1))) * sizeof(cf);
}
inline size_t row_lds(const Geo& g) {
  const int rw = (2048 >> g.logM2) > 1 ? (2048 >> g.logM2) : 1;
  return ((size_t)rw * (1u << g.logM2) + (1u << (g.logM2 - 1))) * sizeof(cf);
}
inline dim3 col_grid(const Geo& g, int P) {
  const int cw = (1 << g.logM2) < CW ? (1 << g.logM2) : CW;
  return dim3((1 << g.logM2) / cw, P);
}
inline dim3 row_grid(const Geo& g, int P) {
  const int rw = (2048 >> g.logM2) > 1 ? (2048 >> g.logM2) : 1;
  return dim3(((1 << g.logM1) + rw - 1) / rw, P);
}

template <typename Kern>
inline void allow_lds(Kern k, size_t bytes) {
  if (bytes > 65536) hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
}

template <typename T>
int launch_col_fwd(const void* x, Pairing pr, const Geo& g, int off, cf* ws, int P, hipStream_t s) {
  auto k = col_fwd_kernel<T>;
  allow_lds(k, col_lds(g));
  hipLaunchKernelGGL(k, col_grid(g, P), dim3(NTH), col_lds(g), s, (const T*)x, pr, g, off, ws);
  return DNA_OK;
}

template <int MODE>
void launch_row(cf* ws, const cf* kspec, Pairing pr, const Geo& g, int P, hipStream_t s) {
  auto k = row_kernel<MODE>;
  allow_lds(k, row_lds(g));
  hipLaunchKernelGGL(k, row_grid(g, P), dim3(NTH), row_lds(g), s, ws, kspec, pr, g);
}

template <typename T, int MODE>
void launch_col_inv(const cf* ws, Pairing pr, const Geo& g, int off, const float* bias, const void* aux,
                    void* y, float* outf, float scale, int P, hipStream_t s) {
  auto k = col_inv_kernel<T, MODE>;
  allow_lds(k, col_lds(g));
  hipLaunchKernelGGL(k, col_grid(g, P), dim3(NTH), col_lds(g), s, ws, pr, g, off, bias,
                     (const T*)aux, (T*)y, outf, scale);
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

extern "C" int dna_fftconv_filter(const float* k, int D, int L, void* kspec, void* ws,
                                  size_t ws_bytes, void* stream) {
  Geo g;
  DNA_CHECK_ARG(k && kspec && ws, "dna_fftconv_filter: null pointer");
  DNA_CHECK_ARG(D > 0 && geometry(L, g), "dna_fftconv_filter: L=%d must be a power of 2 in [64, 131072]", L);
  const size_t N = (size_t)1 << g.logN;
  const int Q = (D + 1) / 2;
  DNA_CHECK_ARG(ws_bytes >= (size_t)Q * N * sizeof(cf), "dna_fftconv_filter: workspace too small");
  hipStream_t s = as_stream(stream);
  Pairing pr{D, 1, Q};  // channels paired (2q, 2q+1)
  cf* w = (cf*)ws;
  launch_col_fwd<float>(k, pr, g, 0, w, Q, s);
  launch_row<ROW_SPEC>(w, nullptr, pr, g, Q, s);
  const int bx = (int)((N + NTH - 1) / NTH) < 1024 ? (int)((N + NTH - 1) / NTH) : 1024;
  hipLaunchKernelGGL(separate_kernel, dim3(bx, Q), dim3(NTH), 0, s, (const cf*)w, D, g, (cf*)kspec);
  DNA_LAUNCH_CHECK("dna_fftconv_filter");
  return DNA_OK;
}

extern "C" int dna_fftconv_fwd(const void* u, int dtype, const void* kspec, const float* bias,
                               int B, int D, int L, int bidirectional, void* y, void* ws,
                               size_t ws_bytes, void* stream) {
  Geo g;
  DNA_CHECK_ARG(u && kspec && y && ws, "dna_fftconv_fwd: null pointer");
  DNA_CHECK_ARG(B > 0 && D > 0 && geometry(L, g), "dna_fftconv_fwd: L=%d must be a power of 2 in [64, 131072]", L);
  const size_t N = (size_t)1 << g.logN;
  const int BP = (B + 1) / 2, P = BP * D;
  DNA_CHECK_ARG(ws_bytes >= (size_t)P * N * sizeof(cf), "dna_fftconv_fwd: workspace too small");
  hipStream_t s = as_stream(stream);
  Pairing pr{B, D, BP};
  cf* w = (cf*)ws;
  const int pb = pad_before(L, bidirectional);
  if (dtype == DNA_BF16) {
    launch_col_fwd<bf16>(u, pr, g, pb, w, P, s);
    launch_row<ROW_MUL>(w, (const cf*)kspec, pr, g, P, s);
    launch_col_inv<bf16, OUT_PAIR>(w, pr, g, 0, bias, u, y, nullptr, 1.f, P, s);
  } else if (dtype == DNA_F32) {
    launch_col_fwd<float>(u, pr, g, pb, w, P, s);
    launch_row<ROW_MUL>(w, (const cf*)kspec, pr, g, P, s);
    launch_col_inv<float, OUT_PAIR>(w, pr, g, 0, bias, u, y, nullptr, 1.f, P, s);
  } else {
    DNA_CHECK_ARG(false, "dna_fftconv_fwd: bad dtype");
  }
  DNA_LAUNCH_CHECK("dna_fftconv_fwd");
  return DNA_OK;
}

template <typename T>
static void bwd_impl(const void* dy, const void* u, const cf* kspec, const float* bias, int B, int D,
                     const Geo& g, int pb, void* du, float* dk, float* dbias, cf* ws, hipStream_t s) {
  const size_t N = (size_t)1 << g.logN;
  const int BP = (B + 1) / 2, P = BP * D;
  Pairing pr{B, D, BP};
  cf* zu = ws;
  cf* zy = ws + (size_t)P * N;
  cf* pk = ws + (size_t)2 * P * N;
  // spectra of u~ and of dy (padded at the end)
  if (dk) {
    launch_col_fwd<T>(u, pr, g, pb, zu, P, s);
    launch_row<ROW_SPEC>(zu, nullptr, pr, g, P, s);
  }
  launch_col_fwd<T>(dy, pr, g, 0, zy, P, s);
  launch_row<ROW_SPEC>(zy, nullptr, pr, g, P, s);
  if (dk) {
    const int bx = (int)((N + NTH - 1) / NTH) < 512 ? (int)((N + NTH - 1) / NTH) : 512;
    hipLaunchKernelGGL(dkspec_kernel, dim3(bx, D), dim3(NTH), 0, s, (const cf*)zu, (const cf*)zy, BP,
                       g.logN, pk);
    Pairing one{D, 1, 0};  // BP = 0: row index is the channel
    launch_row<ROW_INV>(pk, nullptr, one, g, D, s);
    launch_col_inv<float, OUT_REAL>(pk, one, g, 0, nullptr, nullptr, nullptr, dk, 1.f / (float)N, D, s);
  }
  if (du) {
    // du~ = IFFT(DY * conj(K)); du = du~[pb : pb + L] + bias * dy   (zy is consumed in place)
    launch_row<ROW_INV_MULCONJ>(zy, kspec, pr, g, P, s);
    launch_col_inv<T, OUT_PAIR>(zy, pr, g, pb, bias, dy, du, nullptr, 1.f, P, s);
  }
  if (dbias) hipLaunchKernelGGL(dbias_kernel<T>, dim3(D), dim3(NTH), 0, s, (const T*)dy, (const T*)u, B, D,
                                g.L, dbias);
}

extern "C" int dna_fftconv_bwd(const void* dy, const void* u, int dtype, const void* kspec,
                               const float* bias, int B, int D, int L, int bidirectional, void* du,
                               float* dk, float* dbias, void* ws, size_t ws_bytes, void* stream) {
  Geo g;
  DNA_CHECK_ARG(dy && u && kspec && ws, "dna_fftconv_bwd: null pointer");
  DNA_CHECK_ARG(B > 0 && D > 0 && geometry(L, g), "dna_fftconv_bwd: L=%d must be a power of 2 in [64, 131072]", L);
  const size_t N = (size_t)1 << g.logN;
  const size_t P = (size_t)((B + 1) / 2) * D;
  DNA_CHECK_ARG(ws_bytes >= (2 * P + (size_t)D) * N * sizeof(cf), "dna_fftconv_bwd: workspace too small");
  const int pb = pad_before(L, bidirectional);
  hipStream_t s = as_stream(stream);
  if (dtype == DNA_BF16)
    bwd_impl<bf16>(dy, u, (const cf*)kspec, bias, B, D, g, pb, du, dk, dbias, (cf*)ws, s);
  else if (dtype == DNA_F32)
    bwd_impl<float>(dy, u, (const cf*)kspec, bias, B, D, g, pb, du, dk, dbias, (cf*)ws, s);
  else
    DNA_CHECK_ARG(false, "dna_fftconv_bwd: bad dtype");
  DNA_LAUNCH_CHECK("dna_fftconv_bwd");
  return DNA_OK;
}
