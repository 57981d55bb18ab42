// Channel-major projection with a register-resident weight (gfx950): the Mamba in_proj forward
// of Caduceus (reference src/models/caduceus/modeling_caduceus.py:88-91 -> mamba_ssm
// Mamba.forward, `in_proj.weight @ rearrange(hidden, "b l d -> d (b l)")`):
//
//   C[z][c][l] = sum_{j < K} W[c][j] X[z][l][j] (+ bias[c]),   c < M, l < N, K <= 256
//
// At config E (M = 2E = 1024, K = d_model = 256, N = L = 131,072) the product moves 67 MB of X
// and 268 MB of C against 69 GFLOP: HBM-bound (~42 us at 8 TB/s) on a shape where the general
// tile GEMMs lose to per-tile prologues (K is only 8 k-steps of 32). Here a block owns 256
// channels: each of its 4 waves holds its 64 channels x K of W as MFMA fragments in registers
// for the block's whole life (K/2 VGPRs), and the block streams X through LDS 64 positions at a
// time -- the next tile's X is loaded into registers while the current one multiplies, so per
// tile the only global traffic is X in and C out.
//
// MFMA v_mfma_f32_16x16x32_bf16 issued swapped (D = X_frag . W_frag^T): a lane holds 4
// consecutive positions of one channel, so the output leaves as 8-B stores, 32 B per channel row
// and n-subtile (the 4 n-subtiles of a tile complete each 128-B row segment in L2).
#include <stdlib.h>

#include "common.h"

namespace dna {
namespace pcm {

constexpr int NT = 256;          // threads: 4 waves
constexpr int CB = 256;          // channels per block (64 per wave)
constexpr int NTILE = 64;        // positions per tile
constexpr int KMAX = 256;
constexpr int XS = KMAX + 8;     // LDS row stride (elements): 528 B, rows 4 banks apart

typedef __attribute__((ext_vector_type(2))) unsigned u32x2;

constexpr int OS = NTILE + 4;   // staged output row stride (elements): 136 B

template <int K, bool STAGE>
__global__ __launch_bounds__(NT, 1) void proj_cm_kernel(const bf16* __restrict__ W,
                                                        const bf16* __restrict__ X,
                                                        const float* __restrict__ bias, int M,
                                                        int N, int rev, bf16* __restrict__ C) {
  static_assert(K % 32 == 0 && K <= KMAX, "K");
  constexpr int KS = K / 32;                 // k-steps
  constexpr int CH = NTILE * K / 8 / NT;     // 16-B chunks of an X tile per thread
  __shared__ __attribute__((aligned(16))) bf16 xs[NTILE * XS];
  // STAGE: each wave's 64 x 64 output tile goes through LDS so the global stores are 16 B per
  // lane and 128 B contiguous per channel row (8 rows per instruction)
  __shared__ __attribute__((aligned(16))) bf16 os[STAGE ? 4 * 64 * OS : 1];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int i16 = lane & 15, g = lane >> 4;
  const int z = blockIdx.z;
  const int cw = blockIdx.y * CB + wave * 64;  // this wave's first channel
  const bf16* Xz = X + (size_t)z * N * K;
  bf16* Cz = C + (size_t)z * M * N;

  // W fragments: [m-subtile][k-step], lane (i16 = channel row, g = k group of 8)
  bf16x8 wf[4][KS];
#pragma unroll
  for (int ms = 0; ms < 4; ++ms) {
    const int c = cw + 16 * ms + i16;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
      wf[ms][ks] = c < M ? *reinterpret_cast<const bf16x8*>(W + (size_t)c * K + 32 * ks + 8 * g)
                         : bf16x8{};
  }
  float bz[4];
#pragma unroll
  for (int ms = 0; ms < 4; ++ms) {
    const int c = cw + 16 * ms + i16;
    bz[ms] = (bias && c < M) ? bias[c] : 0.f;
  }

  const int ntiles = (N + NTILE - 1) / NTILE;
  // X tile staging: chunk q = tid + NT * p covers row q / (K/8), 16-B column q % (K/8)
  auto load_x = [&](int tile, bf16x8 (&r)[CH]) {
#pragma unroll
    for (int p = 0; p < CH; ++p) {
      const int q = tid + NT * p;
      const int row = q / (K / 8), col = q % (K / 8);
      const int l = tile * NTILE + row;
      const int lx = rev ? N - 1 - l : l;  // rev: X read in reversed position order
      r[p] = l < N ? *reinterpret_cast<const bf16x8*>(Xz + (size_t)lx * K + 8 * col) : bf16x8{};
    }
  };
  bf16x8 xr[CH];
  int tile = blockIdx.x;
  if (tile < ntiles) load_x(tile, xr);
  for (; tile < ntiles; tile += gridDim.x) {
    __syncthreads();  // the previous tile's fragment reads are done
#pragma unroll
    for (int p = 0; p < CH; ++p) {
      const int q = tid + NT * p;
      *reinterpret_cast<bf16x8*>(xs + (q / (K / 8)) * XS + 8 * (q % (K / 8))) = xr[p];
    }
    __syncthreads();
    const int nxt = tile + gridDim.x;
    if (nxt < ntiles) load_x(nxt, xr);  // in flight while this tile multiplies
    if (cw >= M) continue;              // wave past the last channel (uniform)
    f32x4 acc[4][4];                    // [m-subtile][n-subtile]
#pragma unroll
    for (int ms = 0; ms < 4; ++ms)
#pragma unroll
      for (int ns = 0; ns < 4; ++ns) acc[ms][ns] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      bf16x8 xf[4];
#pragma unroll
      for (int ns = 0; ns < 4; ++ns)
        xf[ns] = *reinterpret_cast<const bf16x8*>(xs + (16 * ns + i16) * XS + 32 * ks + 8 * g);
#pragma unroll
      for (int ns = 0; ns < 4; ++ns)
#pragma unroll
        for (int ms = 0; ms < 4; ++ms)
          acc[ms][ns] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(xf[ns], wf[ms][ks], acc[ms][ns], 0, 0, 0);
    }
    // lane: channel cw + 16 ms + i16, positions tile*64 + 16 ns + 4 g + 0..3
    if constexpr (STAGE) {
      bf16* ow = os + wave * 64 * OS;
#pragma unroll
      for (int ms = 0; ms < 4; ++ms)
#pragma unroll
        for (int ns = 0; ns < 4; ++ns) {
          const bf16x4 h = {(bf16)(acc[ms][ns][0] + bz[ms]), (bf16)(acc[ms][ns][1] + bz[ms]),
                            (bf16)(acc[ms][ns][2] + bz[ms]), (bf16)(acc[ms][ns][3] + bz[ms])};
          *reinterpret_cast<u32x2*>(ow + (16 * ms + i16) * OS + 16 * ns + 4 * g) =
              __builtin_bit_cast(u32x2, h);
        }
      // the wave reads back only what it wrote: LDS keeps one wave's operations in order, so a
      // compiler barrier suffices (no s_barrier)
      asm volatile("" ::: "memory");
      const int l0 = tile * NTILE + 8 * (lane & 7);
#pragma unroll
      for (int it = 0; it < 8; ++it) {
        const int r = 8 * it + (lane >> 3);
        const int c = cw + r;
        const bf16x4 lo = *reinterpret_cast<const bf16x4*>(ow + r * OS + 8 * (lane & 7));
        const bf16x4 hi = *reinterpret_cast<const bf16x4*>(ow + r * OS + 8 * (lane & 7) + 4);
        if (c < M) {
          bf16* dst = Cz + (size_t)c * N + l0;
          if (l0 + 8 <= N && (N & 7) == 0) {
            *reinterpret_cast<bf16x8*>(dst) = bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
          } else {
#pragma unroll
            for (int e = 0; e < 8; ++e)
              if (l0 + e < N) dst[e] = e < 4 ? lo[e] : hi[e - 4];
          }
        }
      }
      asm volatile("" ::: "memory");
      continue;
    }
#pragma unroll
    for (int ms = 0; ms < 4; ++ms) {
      const int c = cw + 16 * ms + i16;
      if (c >= M) continue;
      bf16* row = Cz + (size_t)c * N;
#pragma unroll
      for (int ns = 0; ns < 4; ++ns) {
        const int l = tile * NTILE + 16 * ns + 4 * g;
        const bf16x4 h = {(bf16)(acc[ms][ns][0] + bz[ms]), (bf16)(acc[ms][ns][1] + bz[ms]),
                          (bf16)(acc[ms][ns][2] + bz[ms]), (bf16)(acc[ms][ns][3] + bz[ms])};
        if (l + 4 <= N && (N & 3) == 0) {
          *reinterpret_cast<u32x2*>(row + l) = __builtin_bit_cast(u32x2, h);
        } else {
#pragma unroll
          for (int r = 0; r < 4; ++r)
            if (l + r < N) row[l + r] = h[r];
        }
      }
    }
  }
}

}  // namespace pcm
}  // namespace dna

using namespace dna;
using namespace dna::pcm;

extern "C" int dna_proj_cm_bf16(const void* W, const void* X, const float* bias, int M, int N,
                                int K, int batch, int reverse, void* C, void* stream) {
  DNA_CHECK_ARG(M >= 0 && N >= 0 && batch >= 1, "dna_proj_cm_bf16: bad shape (M=%d N=%d batch=%d)",
                M, N, batch);
  if (M == 0 || N == 0) return DNA_OK;
  DNA_CHECK_ARG(W && X && C, "dna_proj_cm_bf16: null pointer");
  DNA_CHECK_ARG(K == 64 || K == 128 || K == 256,
                "dna_proj_cm_bf16: K=%d unsupported (64, 128 or 256)", K);
  DNA_CHECK_ARG(((uintptr_t)W & 15) == 0 && ((uintptr_t)X & 15) == 0 && ((uintptr_t)C & 7) == 0,
                "dna_proj_cm_bf16: W / X need 16-B, C 8-B alignment");
  DNA_CHECK_ARG(batch <= 65535, "dna_proj_cm_bf16: batch too large");
  const int ntiles = (N + NTILE - 1) / NTILE;
  const int cblocks = (M + CB - 1) / CB;
  // about 4 blocks per CU over the whole grid: each block multiplies several tiles with its
  // register-resident W slab
  int gx = (4 * 256 + cblocks * batch - 1) / (cblocks * batch);
  if (gx > ntiles) gx = ntiles;
  if (gx < 1) gx = 1;
  const dim3 grid(gx, cblocks, batch);
  hipStream_t s = as_stream(stream);
  // DNA_PROJ_CM_STAGE=0: direct 8-B stores from the accumulators (A/B)
  static const int stage_env = getenv("DNA_PROJ_CM_STAGE") ? atoi(getenv("DNA_PROJ_CM_STAGE")) : 1;
  const bool stage = stage_env != 0;
#define DNA_PCM(KK)                                                                                   \
  if (stage) hipLaunchKernelGGL((proj_cm_kernel<KK, true>), grid, dim3(NT), 0, s, (const bf16*)W,   \
                                (const bf16*)X, bias, M, N, reverse, (bf16*)C);                      \
  else hipLaunchKernelGGL((proj_cm_kernel<KK, false>), grid, dim3(NT), 0, s, (const bf16*)W,        \
                          (const bf16*)X, bias, M, N, reverse, (bf16*)C);
  switch (K) {
    case 64: DNA_PCM(64) break;
    case 128: DNA_PCM(128) break;
    default: DNA_PCM(256) break;
  }
#undef DNA_PCM
  DNA_LAUNCH_CHECK("dna_proj_cm_bf16");
  return DNA_OK;
}
