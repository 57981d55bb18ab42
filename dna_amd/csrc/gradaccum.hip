// Gradient accumulation kernels that write straight into the flat fp32 .grad buffer.
//
//  * dna_sum_slices_accum: out += sum_k parts[k] -- the split-K weight-gradient partials of a
//    [s, M, N] batched GEMM folded into the parameter's gradient in one pass (no separate reduce
//    + AccumulateGrad add; replaces autograd's accumulation for Linear weights).
//  * dna_embed_grad_segsum: d(word_embeddings) from per-token row gradients, by token id:
//    rows visited in id-sorted order, summed in registers per run of equal ids per 32-row chunk,
//    runs crossing chunks joined in chunk order (deterministic, no atomics) -- frequent BPE tokens (thousands of rows per id in a
//    65,536-token batch) no longer serialise on one row (nn.Embedding backward with
//    padding_idx=0, bert_layers.py:45-47).
#include "common.h"

namespace dna {
namespace gacc {

// accum: out += sum (gradient accumulation); else out = sum (no zero fill needed first). The
// slices are added in slice order either way (deterministic).
__global__ __launch_bounds__(256) void sum_slices_kernel(const float* __restrict__ parts, int s,
                                                         size_t n, float* __restrict__ out,
                                                         int vec, int accum) {
  const size_t n4 = vec ? n / 4 : 0;  // 16-B path when every slice starts 16-B aligned
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n4;
       i += (size_t)gridDim.x * blockDim.x) {
    f32x4 acc = accum ? reinterpret_cast<const f32x4*>(out)[i] : f32x4{0.f, 0.f, 0.f, 0.f};
    int k = 0;
    for (; k + 8 <= s; k += 8) {  // 8 slice loads in flight, added in slice order
      f32x4 v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = reinterpret_cast<const f32x4*>(parts + (size_t)(k + u) * n)[i];
#pragma unroll
      for (int u = 0; u < 8; ++u) acc += v[u];
    }
    for (; k < s; ++k) acc += reinterpret_cast<const f32x4*>(parts + (size_t)k * n)[i];
    reinterpret_cast<f32x4*>(out)[i] = acc;
  }
  for (size_t i = n4 * 4 + blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n;
       i += (size_t)gridDim.x * blockDim.x) {
    float acc = accum ? out[i] : 0.f;
    for (int k = 0; k < s; ++k) acc += parts[(size_t)k * n + i];
    out[i] = acc;
  }
}

// out[c] (+)= sum_r part[r][c], deterministic: a block = 64 columns x 16 row groups (row r goes
// to group r % 16, summed in row order with 8 loads in flight), groups combined in fixed order.
constexpr int CS_GROUPS = 16;

__global__ __launch_bounds__(64 * CS_GROUPS) void colsum_kernel(const float* __restrict__ part,
                                                                int rows, int cols, int accumulate,
                                                                float* __restrict__ out) {
  __shared__ float red[CS_GROUPS][64];
  const int c = blockIdx.x * 64 + (threadIdx.x & 63), g = threadIdx.x >> 6;
  float s = 0.f;
  int r = g;
  for (; r + 7 * CS_GROUPS < rows; r += 8 * CS_GROUPS) {
    float v[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = part[(size_t)(r + i * CS_GROUPS) * cols + c];
#pragma unroll
    for (int i = 0; i < 8; ++i) s += v[i];
  }
  for (; r < rows; r += CS_GROUPS) s += part[(size_t)r * cols + c];
  red[g][threadIdx.x & 63] = s;
  __syncthreads();
  if (g == 0) {
    float t = 0.f;
#pragma unroll
    for (int i = 0; i < CS_GROUPS; ++i) t += red[i][threadIdx.x];
    out[c] = accumulate ? out[c] + t : t;
  }
}

// Column sums of a bf16 matrix (a Linear's bias gradient sum_r dy[r][c]), stage 1: partial
// sums per chunk of CS_CHUNK rows. A block = W column groups of 8 (one 16-B load each) x 256/W
// row groups; a thread sums its rows of the chunk in row order (4 loads in flight), the row
// groups are combined through LDS in fixed order -> part[chunk][c]. Stage 2 is colsum_kernel
// over the chunks (deterministic end to end).
constexpr int CS_CHUNK = 256;
template <int W>
__global__ __launch_bounds__(256) void colsum_bf16_part_kernel(const bf16* __restrict__ x, int rows,
                                                               int cols, float* __restrict__ part) {
  constexpr int RG = 256 / W;
  __shared__ f32x4 red[RG][W][2];
  const int cg = threadIdx.x % W, rg = threadIdx.x / W;
  const int c0 = (blockIdx.x * W + cg) * 8;
  const int r0 = blockIdx.y * CS_CHUNK, r1 = min(rows, r0 + CS_CHUNK);
  f32x4 a0 = {0.f, 0.f, 0.f, 0.f}, a1 = {0.f, 0.f, 0.f, 0.f};
  int r = r0 + rg;
  for (; r + 3 * RG < r1; r += 4 * RG) {
    bf16x8 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = *reinterpret_cast<const bf16x8*>(x + (size_t)(r + u * RG) * cols + c0);
#pragma unroll
    for (int u = 0; u < 4; ++u) {
#pragma unroll
      for (int e = 0; e < 4; ++e) { a0[e] += (float)v[u][e]; a1[e] += (float)v[u][4 + e]; }
    }
  }
  for (; r < r1; r += RG) {
    const bf16x8 v = *reinterpret_cast<const bf16x8*>(x + (size_t)r * cols + c0);
#pragma unroll
    for (int e = 0; e < 4; ++e) { a0[e] += (float)v[e]; a1[e] += (float)v[4 + e]; }
  }
  red[rg][cg][0] = a0;
  red[rg][cg][1] = a1;
  __syncthreads();
  if (rg == 0) {
#pragma unroll
    for (int g = 1; g < RG; ++g) { a0 += red[g][cg][0]; a1 += red[g][cg][1]; }
    float* o = part + (size_t)blockIdx.y * cols + c0;
    *reinterpret_cast<f32x4*>(o) = a0;
    *reinterpret_cast<f32x4*>(o + 4) = a1;
  }
}

constexpr int SEG_CHUNK = 32;

// Deterministic: a run of equal ids lying inside one chunk belongs to that chunk's wave (plain
// read-modify-write of its table row). A run crossing a chunk boundary leaves one partial per
// chunk it touches in `work` (slot 0: the chunk's first run continued from the previous chunk,
// slot 1: its last run continuing into the next); segsum_join_kernel then sums those partials
// in chunk order. No atomics, so the table gradient is bit-identical run to run.
__device__ __forceinline__ bool seg_cont(const int64_t* ids, int a, int b, int rows) {
  return a >= 0 && b < rows && ids[a] == ids[b];
}

template <int NV>
__global__ __launch_bounds__(256) void segsum_kernel(const float* __restrict__ drows,
                                                     const int64_t* __restrict__ sorted_ids,
                                                     const int64_t* __restrict__ perm, int rows,
                                                     int cols, int vocab, int pad_idx,
                                                     float* __restrict__ dE,
                                                     float* __restrict__ work) {
  const int lane = threadIdx.x & 63;
  const int chunk = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int p0 = chunk * SEG_CHUNK;
  if (p0 >= rows) return;
  const int p1 = min(rows, p0 + SEG_CHUNK);
  const bool cross_start = seg_cont(sorted_ids, p0 - 1, p0, rows);
  const bool cross_end = seg_cont(sorted_ids, p1 - 1, p1, rows);
  float acc[NV];
#pragma unroll
  for (int k = 0; k < NV; ++k) acc[k] = 0.f;
  long cur = (long)sorted_ids[p0];
  bool first = true;
  auto flush = [&](long id, bool last) {
    if (id == pad_idx || id < 0 || id >= vocab) return;
    int slot = -1;
    if (first && cross_start) slot = 0;
    else if (last && cross_end) slot = 1;
    float* dst = slot < 0 ? dE + (size_t)id * cols : work + ((size_t)chunk * 2 + slot) * cols;
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      if (slot < 0) dst[k * 64 + lane] += acc[k];
      else dst[k * 64 + lane] = acc[k];
    }
  };
  // the chunk's ids and row indices are read once, one per lane, and handed out by readlane;
  // RU rows' loads are issued before their adds (same order of adds as one row at a time)
  const int n = p1 - p0;
  const int pl = p0 + min(lane & (SEG_CHUNK - 1), n - 1);
  const long my_id = (long)sorted_ids[pl];
  const int my_row = (int)perm[pl];
  constexpr int RU = NV <= 4 ? 8 : 4;
  for (int q = 0; q < n; q += RU) {
    float row[RU][NV];
#pragma unroll
    for (int u = 0; u < RU; ++u) {
      const int r = __builtin_amdgcn_readlane(my_row, min(q + u, n - 1));
      const float* src = drows + (size_t)r * cols;
#pragma unroll
      for (int k = 0; k < NV; ++k) row[u][k] = src[k * 64 + lane];
    }
#pragma unroll
    for (int u = 0; u < RU; ++u) {
      if (q + u < n) {
        const int lo = __builtin_amdgcn_readlane((int)my_id, q + u);
        const int hi = __builtin_amdgcn_readlane((int)(my_id >> 32), q + u);
        const long id = (long)(((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo);
        if (id != cur) {
          flush(cur, false);
          first = false;
#pragma unroll
          for (int k = 0; k < NV; ++k) acc[k] = 0.f;
          cur = id;
        }
#pragma unroll
        for (int k = 0; k < NV; ++k) acc[k] += row[u][k];
      }
    }
  }
  flush(cur, true);
}

constexpr int SEG_GROUP = 32;  // chunks per group of the join's second level

// A group of SEG_GROUP chunks lying wholly inside one run (the rows before and after it carry
// its id) holds only slot-0 partials of that run: one wave per such group sums them in chunk
// order into work2[group], so the join below steps over a frequent token's ~1000-chunk run
// 32 chunks at a time.
template <int NV>
__global__ __launch_bounds__(256) void segsum_group_kernel(const int64_t* __restrict__ sorted_ids,
                                                           int rows, int cols,
                                                           const float* __restrict__ work,
                                                           float* __restrict__ work2) {
  const int lane = threadIdx.x & 63;
  const int g = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int p0 = g * SEG_GROUP * SEG_CHUNK;
  const int p1 = p0 + SEG_GROUP * SEG_CHUNK;
  if (p0 == 0 || p1 >= rows || sorted_ids[p0 - 1] != sorted_ids[p1]) return;
  constexpr int GU = NV <= 4 ? SEG_GROUP : 8;  // partials in flight (registers)
  float acc[NV];
#pragma unroll
  for (int k = 0; k < NV; ++k) acc[k] = 0.f;
  for (int u0 = 0; u0 < SEG_GROUP; u0 += GU) {
    float part[GU][NV];
#pragma unroll
    for (int u = 0; u < GU; ++u)
#pragma unroll
      for (int k = 0; k < NV; ++k)
        part[u][k] = work[((size_t)(g * SEG_GROUP + u0 + u) * 2) * cols + k * 64 + lane];
#pragma unroll
    for (int u = 0; u < GU; ++u)
#pragma unroll
      for (int k = 0; k < NV; ++k) acc[k] += part[u][k];
  }
#pragma unroll
  for (int k = 0; k < NV; ++k) work2[(size_t)g * cols + k * 64 + lane] = acc[k];
}

// One wave per chunk whose last run starts inside it and crosses its end: sum the run's partials
// -- this chunk's slot 1, then the slot-0 partials of the chunks up to the next group boundary,
// the group sums of the whole groups the run covers, and the slot-0 partials of the chunks after
// them up to the run's end. The order is fixed by the ids alone, so the table gradient stays
// bit-identical run to run; every phase loads a batch of partials and run-end tests at once.
template <int NV>
__global__ __launch_bounds__(256) void segsum_join_kernel(const int64_t* __restrict__ sorted_ids,
                                                          int rows, int cols, int vocab,
                                                          int pad_idx, float* __restrict__ dE,
                                                          const float* __restrict__ work,
                                                          const float* __restrict__ work2) {
  const int lane = threadIdx.x & 63;
  const int chunk = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int p0 = chunk * SEG_CHUNK;
  if (p0 >= rows) return;
  const int p1 = min(rows, p0 + SEG_CHUNK);
  if (!seg_cont(sorted_ids, p1 - 1, p1, rows)) return;                 // last run ends here
  if (sorted_ids[p0] == sorted_ids[p1 - 1] && seg_cont(sorted_ids, p0 - 1, p0, rows))
    return;                                                              // run started earlier
  const long id = (long)sorted_ids[p1 - 1];
  if (id == pad_idx || id < 0 || id >= vocab) return;
  float acc[NV];
#pragma unroll
  for (int k = 0; k < NV; ++k) acc[k] = work[((size_t)chunk * 2 + 1) * cols + k * 64 + lane];
  constexpr int JU = NV <= 4 ? 32 : (NV <= 8 ? 16 : 8);
  const int nch = (rows + SEG_CHUNK - 1) / SEG_CHUNK;
  // slot-0 partials of chunks c, c+1, ... (at most n) while the run goes on; true once it ended
  auto singles = [&](int& c, int n) -> bool {
    while (n > 0) {
      float part[JU][NV];
      bool more[JU];
#pragma unroll
      for (int u = 0; u < JU; ++u) {
        const int cu = min(c + u, nch - 1);  // past the last chunk: a harmless re-read, never added
        const int q1 = min(rows, (cu + 1) * SEG_CHUNK);
#pragma unroll
        for (int k = 0; k < NV; ++k) part[u][k] = work[((size_t)cu * 2) * cols + k * 64 + lane];
        // branch-free run-end test (a short-circuit && put a branch and a vmcnt(0) around each)
        const long a = (long)sorted_ids[q1 - 1], b = (long)sorted_ids[min(q1, rows - 1)];
        more[u] = (a == id) & (b == id) & (q1 < rows);
      }
      bool done = false;
      int used = 0;
#pragma unroll
      for (int u = 0; u < JU; ++u) {
        if (!done && u < n) {
#pragma unroll
          for (int k = 0; k < NV; ++k) acc[k] += part[u][k];
          done = !more[u];
          used = u + 1;
        }
      }
      c += used;
      n -= used;
      if (done) return true;
    }
    return false;
  };
  int c = chunk + 1;
  if (c % SEG_GROUP && singles(c, SEG_GROUP - c % SEG_GROUP)) goto store;
  {
    // whole groups: the run covers group c / SEG_GROUP iff the row after it still carries id
    // (the run reaches the group's first row, and the ids are sorted)
    constexpr int JG = 8;
    const int ng = nch / SEG_GROUP;
    for (;;) {
      float part[JG][NV];
      bool in[JG];
#pragma unroll
      for (int u = 0; u < JG; ++u) {
        const int g = min(c / SEG_GROUP + u, max(ng - 1, 0));
        const int q1 = (c / SEG_GROUP + u + 1) * SEG_GROUP * SEG_CHUNK;
#pragma unroll
        for (int k = 0; k < NV; ++k) part[u][k] = work2[(size_t)g * cols + k * 64 + lane];
        in[u] = (q1 < rows) & ((long)sorted_ids[min(q1, rows - 1)] == id);
      }
      bool done = false;
#pragma unroll
      for (int u = 0; u < JG; ++u) {
        if (!done && in[u]) {
#pragma unroll
          for (int k = 0; k < NV; ++k) acc[k] += part[u][k];
          c += SEG_GROUP;
        } else {
          done = true;
        }
      }
      if (done) break;
    }
  }
  singles(c, nch);  // the run ends inside this group
store:
  float* dst = dE + (size_t)id * cols;
#pragma unroll
  for (int k = 0; k < NV; ++k) dst[k * 64 + lane] += acc[k];
}

}  // namespace gacc
}  // namespace dna

using namespace dna;

extern "C" int dna_sum_slices_accum(const float* parts, int s, size_t n, float* out, void* stream) {
  DNA_CHECK_ARG(parts && out && s >= 1, "dna_sum_slices_accum: bad args");
  if (n == 0) return DNA_OK;
  // 16-byte loads when the buffers and every slice are 16-B aligned; element-wise otherwise
  const int vec = (((uintptr_t)parts | (uintptr_t)out) & 15) == 0 && n % 4 == 0;
  size_t blocks = ((vec ? n / 4 : n) + 255) / 256;
  int nb = (int)(blocks < 4096 ? (blocks ? blocks : 1) : 4096);
  hipLaunchKernelGGL(gacc::sum_slices_kernel, dim3(nb), dim3(256), 0, as_stream(stream), parts, s,
                     n, out, vec, 1);
  DNA_LAUNCH_CHECK("dna_sum_slices_accum");
  return DNA_OK;
}

extern "C" int dna_sum_slices(const float* parts, int s, size_t n, float* out, void* stream) {
  DNA_CHECK_ARG(parts && out && s >= 1, "dna_sum_slices: bad args");
  if (n == 0) return DNA_OK;
  const int vec = (((uintptr_t)parts | (uintptr_t)out) & 15) == 0 && n % 4 == 0;
  size_t blocks = ((vec ? n / 4 : n) + 255) / 256;
  int nb = (int)(blocks < 4096 ? (blocks ? blocks : 1) : 4096);
  hipLaunchKernelGGL(gacc::sum_slices_kernel, dim3(nb), dim3(256), 0, as_stream(stream), parts, s,
                     n, out, vec, 0);
  DNA_LAUNCH_CHECK("dna_sum_slices");
  return DNA_OK;
}

extern "C" int dna_colsum_f32(const float* part, int rows, int cols, float* out, int accumulate,
                              void* stream) {
  DNA_CHECK_ARG(part && out && rows >= 1 && cols >= 64 && cols % 64 == 0,
                "dna_colsum_f32: bad args (rows %d, cols %d; cols %% 64 == 0 required)", rows, cols);
  hipLaunchKernelGGL(gacc::colsum_kernel, dim3(cols / 64), dim3(64 * gacc::CS_GROUPS), 0,
                     as_stream(stream), part, rows, cols, accumulate, out);
  DNA_LAUNCH_CHECK("dna_colsum_f32");
  return DNA_OK;
}

extern "C" size_t dna_colsum_bf16_workspace(int rows, int cols) {
  if (rows <= 0 || cols <= 0) return 0;
  return (size_t)((rows + gacc::CS_CHUNK - 1) / gacc::CS_CHUNK) * cols * sizeof(float);
}

extern "C" int dna_colsum_bf16(const void* x, int rows, int cols, float* out, int accumulate,
                               void* workspace, size_t workspace_bytes, void* stream) {
  DNA_CHECK_ARG(x && out && rows >= 1 && cols >= 64 && cols % 64 == 0,
                "dna_colsum_bf16: bad args (rows %d, cols %d; cols %% 64 == 0 required)", rows, cols);
  DNA_CHECK_ARG(((uintptr_t)x & 15) == 0, "dna_colsum_bf16: x must be 16-B aligned");
  DNA_CHECK_ARG(workspace && workspace_bytes >= dna_colsum_bf16_workspace(rows, cols),
                "dna_colsum_bf16: workspace too small");
  hipStream_t s = as_stream(stream);
  const int ng = cols / 8, chunks = (rows + gacc::CS_CHUNK - 1) / gacc::CS_CHUNK;
  float* part = (float*)workspace;
  if (ng % 64 == 0)
    hipLaunchKernelGGL(gacc::colsum_bf16_part_kernel<64>, dim3(ng / 64, chunks), dim3(256), 0, s,
                       (const bf16*)x, rows, cols, part);
  else if (ng % 32 == 0)
    hipLaunchKernelGGL(gacc::colsum_bf16_part_kernel<32>, dim3(ng / 32, chunks), dim3(256), 0, s,
                       (const bf16*)x, rows, cols, part);
  else
    hipLaunchKernelGGL(gacc::colsum_bf16_part_kernel<8>, dim3(ng / 8, chunks), dim3(256), 0, s,
                       (const bf16*)x, rows, cols, part);
  hipLaunchKernelGGL(gacc::colsum_kernel, dim3(cols / 64), dim3(64 * gacc::CS_GROUPS), 0, s,
                     (const float*)part, chunks, cols, accumulate, out);
  DNA_LAUNCH_CHECK("dna_colsum_bf16");
  return DNA_OK;
}

extern "C" size_t dna_embed_grad_segsum_workspace(int rows, int cols) {
  const size_t chunks = (size_t)(rows + gacc::SEG_CHUNK - 1) / gacc::SEG_CHUNK;
  // slot 0 / 1 partials per chunk, then one group sum per SEG_GROUP chunks
  return (chunks * 2 + chunks / gacc::SEG_GROUP + 1) * (size_t)cols * sizeof(float);
}

extern "C" int dna_embed_grad_segsum(const float* drows, const int64_t* sorted_ids,
                                     const int64_t* perm, int rows, int cols, int vocab,
                                     int padding_idx, float* dword_emb, float* work,
                                     size_t work_bytes, void* stream) {
  DNA_CHECK_ARG(drows && sorted_ids && perm && dword_emb, "dna_embed_grad_segsum: null pointer");
  DNA_CHECK_ARG(cols % 64 == 0 && cols <= 1024, "dna_embed_grad_segsum: cols %% 64 != 0");
  if (rows == 0) return DNA_OK;
  DNA_CHECK_ARG(work && work_bytes >= dna_embed_grad_segsum_workspace(rows, cols),
                "dna_embed_grad_segsum: workspace too small");
  const int chunks = (rows + gacc::SEG_CHUNK - 1) / gacc::SEG_CHUNK;
  dim3 grid((chunks + 3) / 4);
  hipStream_t s = as_stream(stream);
  float* work2 = work + (size_t)chunks * 2 * cols;
  switch (cols / 64) {
#define DNA_SEG_CASE(K)                                                                         \
  case K:                                                                                       \
    hipLaunchKernelGGL(gacc::segsum_kernel<K>, grid, dim3(256), 0, s, drows, sorted_ids, perm,   \
                       rows, cols, vocab, padding_idx, dword_emb, work);                         \
    if (chunks >= gacc::SEG_GROUP)                                                              \
      hipLaunchKernelGGL(gacc::segsum_group_kernel<K>, dim3((chunks / gacc::SEG_GROUP + 3) / 4), \
                         dim3(256), 0, s, sorted_ids, rows, cols, work, work2);                  \
    hipLaunchKernelGGL(gacc::segsum_join_kernel<K>, grid, dim3(256), 0, s, sorted_ids, rows,     \
                       cols, vocab, padding_idx, dword_emb, work, work2);                        \
    break;
    DNA_SEG_CASE(1) DNA_SEG_CASE(2) DNA_SEG_CASE(3) DNA_SEG_CASE(4) DNA_SEG_CASE(6)
    DNA_SEG_CASE(8) DNA_SEG_CASE(12) DNA_SEG_CASE(16)
#undef DNA_SEG_CASE
    default:
      set_error("dna_embed_grad_segsum: cols=%d unsupported", cols);
      return DNA_ERR_UNSUPPORTED;
  }
  DNA_LAUNCH_CHECK("dna_embed_grad_segsum");
  return DNA_OK;
}

// bf16 transpose dst[cols][rows] = src[rows][cols]: the transposed weight copy that lets the data
// gradient dx = dy . W run on the K-major persistent GEMM (dx = dy . (W^T)^T). 64x64 tiles through
// LDS (row stride padded by 8 elements: the transposed 8-byte reads land on distinct banks),
// 16-B loads and stores, 256 threads.
namespace dna {
namespace gacc {
__global__ __launch_bounds__(256) void transpose_bf16_kernel(const bf16* __restrict__ src, int rows,
                                                             int cols, bf16* __restrict__ dst) {
  __shared__ bf16 t[64][72];
  const int r0 = blockIdx.y * 64, c0 = blockIdx.x * 64, tid = threadIdx.x;
#pragma unroll
  for (int p = 0; p < 2; ++p) {
    const int r = p * 32 + (tid >> 3), c = (tid & 7) * 8;
    bf16x8 v = {};
    if (r0 + r < rows && c0 + c < cols) v = *reinterpret_cast<const bf16x8*>(src + (size_t)(r0 + r) * cols + c0 + c);
#pragma unroll
    for (int q = 0; q < 8; ++q) t[r][c + q] = v[q];
  }
  __syncthreads();
#pragma unroll
  for (int p = 0; p < 2; ++p) {
    const int c = p * 32 + (tid >> 3), r = (tid & 7) * 8;  // output row c (a source column)
    bf16x8 v;
#pragma unroll
    for (int q = 0; q < 8; ++q) v[q] = t[r + q][c];
    if (c0 + c < cols && r0 + r < rows) *reinterpret_cast<bf16x8*>(dst + (size_t)(c0 + c) * rows + r0 + r) = v;
  }
}

// dst[b][t][:] = src[b][L - 1 - t][:] (rows of `row16` 16-B chunks): the sequence flip of the
// bidirectional Mamba wrapper, one 16-B chunk per thread, grid-stride over all chunks
__global__ __launch_bounds__(256) void flip_rows_kernel(const uint4* __restrict__ src, int L, int row16,
                                                        size_t total, uint4* __restrict__ dst) {
  for (size_t i = blockIdx.x * (size_t)256 + threadIdx.x; i < total; i += (size_t)gridDim.x * 256) {
    const size_t row = i / row16, c = i - row * row16;
    const size_t b = row / L, t = row - b * L;
    dst[i] = src[(b * L + (L - 1 - t)) * row16 + c];
  }
}
}  // namespace gacc
}  // namespace dna

extern "C" int dna_flip_rows(const void* src, int B, int L, size_t row_bytes, void* dst, void* stream) {
  DNA_CHECK_ARG(src && dst && src != dst && B > 0 && L > 0 && row_bytes > 0 && row_bytes % 16 == 0,
                "dna_flip_rows: bad args (row_bytes %% 16 == 0, distinct buffers)");
  DNA_CHECK_ARG((((uintptr_t)src | (uintptr_t)dst) & 15) == 0, "dna_flip_rows: 16-B alignment required");
  const size_t total = (size_t)B * L * (row_bytes / 16);
  const size_t blocks = (total + 255) / 256;
  hipLaunchKernelGGL(gacc::flip_rows_kernel, dim3((unsigned)(blocks < 8192 ? blocks : 8192)), dim3(256), 0,
                     as_stream(stream), (const uint4*)src, L, (int)(row_bytes / 16), total, (uint4*)dst);
  DNA_LAUNCH_CHECK("dna_flip_rows");
  return DNA_OK;
}

extern "C" int dna_transpose_bf16(const void* src, int rows, int cols, void* dst, void* stream) {
  DNA_CHECK_ARG(src && dst && src != dst, "dna_transpose_bf16: bad pointers");
  DNA_CHECK_ARG(rows > 0 && cols > 0 && rows % 8 == 0 && cols % 8 == 0,
                "dna_transpose_bf16: rows and cols must be positive multiples of 8 (%d x %d)", rows, cols);
  dim3 grid((cols + 63) / 64, (rows + 63) / 64);
  hipLaunchKernelGGL(gacc::transpose_bf16_kernel, grid, dim3(256), 0, as_stream(stream),
                     (const bf16*)src, rows, cols, (bf16*)dst);
  DNA_LAUNCH_CHECK("dna_transpose_bf16");
  return DNA_OK;
}
