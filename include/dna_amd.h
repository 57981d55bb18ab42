/*
 * dna_amd.h -- C ABI of the MI355X-native DNABERT-2 masked-LM pretraining hot path.
 *
 * Every entry point takes plain pointers + sizes (device pointers for the kernels, host
 * pointers for the data path) and an opaque `stream` (a hipStream_t, NULL = default stream).
 * Kernels enqueue asynchronously and never allocate; scratch comes in through `workspace`.
 * Return value: DNA_OK (0) or a DNA_ERR_* code; dna_last_error() gives a thread-local message.
 * Layouts are row-major. "T" below is batch*seqlen (padded layout: pads stay in place and are
 * excluded from attention by `key_valid`, exactly as the reference's -10000 pad bias does).
 *
 * Each function names the reference interface it replaces (paths under /root/reference).
 * The Python host side (dna_amd/) binds these through ctypes; INTEGRATION.md shows the
 * binding a maintainer of the reference would add.
 */
#ifndef DNA_AMD_H
#define DNA_AMD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DNA_AMD_ABI_VERSION 1

enum dna_status {
  DNA_OK = 0,
  DNA_ERR_INVALID = 1,     /* bad shape / dtype / null pointer */
  DNA_ERR_HIP = 2,         /* HIP launch or runtime failure */
  DNA_ERR_UNSUPPORTED = 3, /* valid request this build does not implement (e.g. head_dim) */
  DNA_ERR_IO = 4,          /* file missing / unreadable / malformed */
  DNA_ERR_NOMEM = 5        /* host allocation failed or caller buffer too small */
};

enum dna_dtype { DNA_F32 = 0, DNA_BF16 = 1, DNA_F16 = 2 };
enum dna_act { DNA_ACT_NONE = 0, DNA_ACT_GELU = 1 };

int dna_abi_version(void);
const char* dna_last_error(void);

/* ------------------------------------------------------------------ attention (ALiBi + key pad)
 * Replaces the PyTorch attention path of BertUnpadSelfAttention.forward
 * (src/models/DNABERT2/bert_layers.py:160-196, active because flash_attn_qkvpacked_func is forced
 * to None at :31) and the kernel slot flash_attn_qkvpacked_func(qkv, bias)
 * (src/models/DNABERT2/flash_attn_triton.py:1077-1130) with bias = alibi + (1-mask)*-10000
 * (bert_layers.py:421-448) computed in-kernel instead of materialised as [b,H,S,S].
 *
 *   qkv      [T, 3*heads*head_dim]  (columns: t*H*D + h*D + d, t in {q,k,v}), dtype
 *   key_valid[T] uint8 (1 = real token, 0 = pad) or NULL (all valid)
 *   slopes   [heads] fp32 ALiBi slopes (bert_layers.py:378-396), device memory
 *   out      [T, heads*head_dim] dtype;  lse [batch, heads, seqlen] fp32 (natural-log LSE)
 * Supported: head_dim 64; bf16 uses MFMA tiles (seqlen % 64 == 0), fp32 any seqlen.
 */
int dna_attn_fwd(const void* qkv, const uint8_t* key_valid, const float* slopes, int batch,
                 int seqlen, int heads, int head_dim, int dtype, float softmax_scale, void* out,
                 float* lse, void* stream);

/* ------------------------------------------------------------------ generic FlashAttention slot
 * flash_attn_qkvpacked_func(qkv, bias=None, causal=False, softmax_scale=None) with the reference's
 * signature (src/models/sequence/flash_attn_triton.py:1077-1130; _flash_attn_forward :767-860,
 * _flash_attn_backward :863-1074; call site src/models/DNABERT2/bert_layers.py:188,192):
 *   qkv  [batch, seqlen, 3, heads, head_dim] contiguous, dtype DNA_BF16 or DNA_F16, head_dim
 *        32 / 64 / 128, any seqlen;
 *   bias bias_type 0 none, 1 "vector" [., ., 1, seqlen], 2 "matrix" [., ., seqlen, seqlen];
 *        element (b, h, q, k) at bias[b*bias_sb + h*bias_sh + q*bias_sq + k] (a stride of 0
 *        broadcasts that dim, as the reference's repeat does); bias_dtype DNA_F32 or the qkv dtype;
 *   out  [batch, seqlen, heads, head_dim] (qkv dtype); lse [batch, heads, dna_flash_lse_rows]
 *        fp32 natural-log LSE (the reference's seqlen_q_rounded layout).
 * softmax(q k^T * softmax_scale + bias), causal masks key > query. The backward writes dqkv
 * [batch, seqlen, 3, heads, head_dim]; delta is caller workspace [batch, heads, lse rows]. */
int dna_flash_lse_rows(int seqlen);
int dna_flash_fwd(const void* qkv, int dtype, const void* bias, int bias_dtype, int bias_type,
                  long long bias_sb, long long bias_sh, long long bias_sq, int batch, int seqlen,
                  int heads, int head_dim, int causal, float softmax_scale, void* out, float* lse,
                  void* stream);
int dna_flash_bwd(const void* qkv, int dtype, const void* bias, int bias_dtype, int bias_type,
                  long long bias_sb, long long bias_sh, long long bias_sq, const void* out,
                  const void* dout, const float* lse, int batch, int seqlen, int heads,
                  int head_dim, int causal, float softmax_scale, float* delta, void* dqkv,
                  void* stream);

/* Backward of dna_attn_fwd (replaces autograd through bert_layers.py:167-178 and
 * _flash_attn_backward, flash_attn_triton.py:941-1074). Writes dqkv [T, 3*H*D] (dtype).
 * delta_ws: fp32 workspace of batch*heads*seqlen floats (rowsum(dO*O)). */
int dna_attn_bwd(const void* qkv, const void* out, const void* dout, const float* lse,
                 const uint8_t* key_valid, const float* slopes, int batch, int seqlen, int heads,
                 int head_dim, int dtype, float softmax_scale, void* dqkv, float* delta_ws,
                 void* stream);
/* Same, and (bf16 only, dbias_part non-NULL) the column sums of dqkv -- the gradient of the
 * packed QKV projection's bias, Wqkv.bias (bert_layers.py:64, autograd's sum over tokens) -- as
 * fp32 partials: dbias_part [dna_attn_dbias_part_rows(batch, seqlen)][3*heads*head_dim], one row
 * per 128-token block, finished by dna_colsum_f32. The partials use the fp32 gradient values
 * before their bf16 rounding. */
int dna_attn_bwd_ex(const void* qkv, const void* out, const void* dout, const float* lse,
                    const uint8_t* key_valid, const float* slopes, int batch, int seqlen, int heads,
                    int head_dim, int dtype, float softmax_scale, void* dqkv, float* delta_ws,
                    float* dbias_part, void* stream);
int dna_attn_dbias_part_rows(int batch, int seqlen);

/* ------------------------------------------------------------------ fused (bias, act, dropout, residual) + LayerNorm
 * y = LN( dropout( act(x + bias) ) + residual ) over the last dim.
 * Replaces BertSelfOutput.forward (bert_layers.py:209-214: act none, residual),
 * the add+LN tail of BertGatedLinearUnitMLP.forward (:298-300: p_drop 0, residual) and
 * BertPredictionHeadTransform.forward (:524-528: act gelu, no residual, eps 1e-12).
 *   x [rows, cols] x_dtype; bias [cols] fp32 or NULL; residual [rows, cols] fp32 or NULL;
 *   y [rows, cols] fp32 or NULL; y_bf16 [rows, cols] bf16 or NULL; mean/rstd [rows] fp32.
 * Dropout mask = Philox4x32-10(seed, offset + element index / 4): regenerated in backward. */
int dna_ln_fwd(const void* x, int x_dtype, const float* bias, int act, float p_drop,
               uint64_t seed, uint64_t offset, const float* residual, const float* gamma,
               const float* beta, int rows, int cols, float eps, float* y, void* y_bf16,
               float* mean, float* rstd, void* stream);

/* Backward of dna_ln_fwd. The output gradient is dy (fp32) + dy_bf16 (bf16), either may be NULL.
 * Writes: dresidual [rows, cols] fp32 (NULL to skip), dx [rows, cols] x_dtype,
 * dgamma/dbeta/dbias [cols] fp32 (each NULL to skip; written, not accumulated).
 * workspace >= dna_ln_bwd_workspace(rows, cols) bytes. */
size_t dna_ln_bwd_workspace(int rows, int cols);
int dna_ln_bwd(const float* dy, const void* dy_bf16, const void* x, int x_dtype,
               const float* bias, int act, float p_drop, uint64_t seed, uint64_t offset,
               const float* residual, const float* gamma, const float* mean, const float* rstd,
               int rows, int cols, float* dresidual, void* dx, float* dgamma, float* dbeta,
               float* dbias, void* workspace, size_t workspace_bytes, void* stream);
/* Backward of dna_ln_fwd (act none) with x_hat recomputed from the forward's fp32 output y:
 * x_hat = (y - beta) / gamma (gamma without zero entries; mean not needed) -- reads y instead of
 * x and the residual. Same outputs and workspace as dna_ln_bwd. */
int dna_ln_bwd_from_y(const float* dy, const void* dy_bf16, const float* y, int x_dtype,
                      float p_drop, uint64_t seed, uint64_t offset, const float* gamma,
                      const float* beta, const float* rstd, int rows, int cols, float* dresidual,
                      void* dx, float* dgamma, float* dbeta, float* dbias, void* workspace,
                      size_t workspace_bytes, void* stream);
/* dna_ln_bwd_from_y adding dgamma / dbeta / dbias into the given buffers (+=) instead of writing
 * them: the parameters' fp32 gradient slices of a flat gradient buffer (dna_amd.flat), in place
 * of torch AccumulateGrad's per-parameter add (same fp32 add). */
int dna_ln_bwd_from_y_acc(const float* dy, const void* dy_bf16, const float* y, int x_dtype,
                          float p_drop, uint64_t seed, uint64_t offset, const float* gamma,
                          const float* beta, const float* rstd, int rows, int cols,
                          float* dresidual, void* dx, float* dgamma, float* dbeta, float* dbias,
                          void* workspace, size_t workspace_bytes, void* stream);

/* Pre-norm residual add + LayerNorm: sum = x + residual (fp32, written), y = LN(sum).
 * Replaces the flash_attn Block's `residual = dropout(x) + residual; norm(residual)` with
 * residual_in_fp32 (HyenaDNA's create_block, src/models/sequence/long_conv_lm.py:205-267; dropout
 * p = 0). x [rows, cols] x_dtype; residual, sum [rows, cols] fp32; y fp32 and / or y_bf16.
 * Backward: dsum = gradient of `sum` from its other consumers (NULL: none), added to the LN's
 * input gradient; writes dresidual (fp32) = dx (x_dtype) = that total, dgamma / dbeta (written).
 * rms = 1: RMSNorm instead (no mean, no beta: beta / mean / dbeta may be NULL) -- mamba_ssm's
 * Block with fused_add_norm as the Caduceus Blocks use it (modeling_caduceus.py:25-65).
 * workspace >= dna_ln_bwd_workspace(rows, cols). */
int dna_add_ln_fwd(const void* x, int x_dtype, const float* residual, const float* gamma,
                   const float* beta, int rows, int cols, float eps, int rms, float* sum, float* y,
                   void* y_bf16, float* mean, float* rstd, void* stream);
int dna_add_ln_bwd(const float* dy, const void* dy_bf16, const float* dsum, const void* x,
                   int x_dtype, const float* residual, const float* gamma, const float* mean,
                   const float* rstd, int rows, int cols, int rms, float* dresidual, void* dx,
                   float* dgamma, float* dbeta, void* workspace, size_t workspace_bytes,
                   void* stream);

/* RMSNorm y = x * rsqrt(mean(x^2) + eps) * gamma with fp32 statistics -- replaces mamba_ssm's
 * RMSNorm as the Caduceus Blocks and norm_f apply it (src/models/caduceus/modeling_caduceus.py
 * :25-65 and :214-216 build them with rms_norm=True; the fused add is left to the caller).
 * x [rows, cols] x_dtype; y fp32 and/or
 * y_bf16; rstd [rows] fp32. Backward writes dx (x_dtype) and dgamma [cols] (written, not
 * accumulated); the output gradient is dy (fp32) + dy_bf16, either may be NULL;
 * workspace >= dna_ln_bwd_workspace(rows, cols). */
int dna_rms_fwd(const void* x, int x_dtype, const float* gamma, int rows, int cols, float eps,
                float* y, void* y_bf16, float* rstd, void* stream);
int dna_rms_bwd(const float* dy, const void* dy_bf16, const void* x, int x_dtype,
                const float* gamma, const float* rstd, int rows, int cols, void* dx,
                float* dgamma, void* workspace, size_t workspace_bytes, void* stream);

/* ------------------------------------------------------------------ embeddings
 * y = dropout( LN( word_emb[ids] + type_row ) )   (BertEmbeddings.forward, bert_layers.py:62-107;
 * token_type_ids are all zero so type_row = token_type_embeddings.weight[0]).
 *   ids [rows] int64; word_emb [vocab, cols] fp32; y fp32 / y_bf16 (either may be NULL). */
int dna_embed_ln_fwd(const int64_t* ids, const float* word_emb, const float* type_row,
                     const float* gamma, const float* beta, int rows, int cols, int vocab,
                     float eps, float p_drop, uint64_t seed, uint64_t offset, float* y,
                     void* y_bf16, float* mean, float* rstd, void* stream);

/* Backward. dword_emb [vocab, cols] is ACCUMULATED into (+=, fp32 atomics; rows whose id equals
 * padding_idx are skipped -- nn.Embedding(padding_idx=0), bert_layers.py:45-47). dtype_row,
 * dgamma, dbeta [cols] are written. workspace >= dna_ln_bwd_workspace(rows, cols). */
int dna_embed_ln_bwd(const float* dy, const void* dy_bf16, const int64_t* ids,
                     const float* word_emb, const float* type_row, const float* gamma,
                     const float* mean, const float* rstd, int rows, int cols, int vocab,
                     int padding_idx, float p_drop, uint64_t seed, uint64_t offset,
                     float* dword_emb, float* dtype_row, float* dgamma, float* dbeta,
                     void* workspace, size_t workspace_bytes, void* stream);

/* Same backward, but instead of accumulating into the table it writes each token's embedding-row
 * gradient to drows [rows, cols] fp32 (for dna_embed_grad_segsum). */
int dna_embed_ln_bwd_rows(const float* dy, const void* dy_bf16, const int64_t* ids,
                          const float* word_emb, const float* type_row, const float* gamma,
                          const float* mean, const float* rstd, int rows, int cols, int vocab,
                          float p_drop, uint64_t seed, uint64_t offset, float* drows,
                          float* dtype_row, float* dgamma, float* dbeta, void* workspace,
                          size_t workspace_bytes, void* stream);

/* dword_emb[id] += sum of drows[perm[p]] over the id-sorted positions p (sorted_ids ascending,
 * perm = the argsort of ids); rows with id == padding_idx are skipped. Replaces the scatter-add
 * of nn.Embedding backward (padding_idx=0, bert_layers.py:45-47). Deterministic for a given
 * (sorted_ids, perm): runs crossing 32-row chunks are joined through `work` in chunk order
 * (work_bytes >= dna_embed_grad_segsum_workspace(rows, cols)). */
size_t dna_embed_grad_segsum_workspace(int rows, int cols);
int dna_embed_grad_segsum(const float* drows, const int64_t* sorted_ids, const int64_t* perm,
                          int rows, int cols, int vocab, int padding_idx, float* dword_emb,
                          float* work, size_t work_bytes, void* stream);

/* out[c] = sum_r part[r][c] (accumulate != 0: out[c] += ...), fp32, deterministic order;
 * cols % 64 == 0. Finishes the fused bias-gradient partials (Linear bias grads, autograd's
 * dy.sum(0)). */
int dna_colsum_f32(const float* part, int rows, int cols, float* out, int accumulate, void* stream);
/* out[c] (+)= sum_r x[r][c] for a bf16 matrix x [rows, cols] (16-B aligned, cols % 64 == 0): a
 * Linear's bias gradient from the bf16 output gradient (replaces autograd's dy.sum(0) for
 * nn.Linear under bf16 autocast). fp32 partials per 256-row chunk in workspace (>=
 * dna_colsum_bf16_workspace(rows, cols) bytes), summed in chunk order (deterministic). */
size_t dna_colsum_bf16_workspace(int rows, int cols);
int dna_colsum_bf16(const void* x, int rows, int cols, float* out, int accumulate, void* workspace,
                    size_t workspace_bytes, void* stream);

/* dst[b][t] = src[b][L - 1 - t] for rows of row_bytes (% 16 == 0) bytes, src / dst distinct and
 * 16-B aligned: torch.flip(x, dims=(1,)) of a [B, L, C] tensor as the Caduceus BiMambaWrapper
 * applies it (src/models/caduceus/modeling_caduceus.py:68-121). */
int dna_flip_rows(const void* src, int B, int L, size_t row_bytes, void* dst, void* stream);
/* out[i] += sum_{k<s} parts[k*n + i]: split-K partials of a weight gradient folded straight
 * into the flat fp32 gradient buffer (16-byte loads when the buffers are 16-byte aligned and
 * n % 4 == 0, element-wise otherwise). */
int dna_sum_slices_accum(const float* parts, int s, size_t n, float* out, void* stream);
/* out = sum_k parts[k] (same slice order; no zero fill of `out` needed): the weight gradients of
 * the strided GEMM's split-K slices (mamba.InProj / OutProj / ChannelLinear, StridedLinear). */
int dna_sum_slices(const float* parts, int s, size_t n, float* out, void* stream);

/* ------------------------------------------------------------------ GeGLU (+ dropout)
 * a = dropout( gelu_erf(g[:, :inter]) * g[:, inter:] )   (bert_layers.py:292-296)
 *   g [rows, 2*inter] dtype -> a [rows, inter] dtype, and (fac non-NULL) the backward factors
 *   fac [rows, 2*inter] = [k*s*g2*gelu'(g1) | k*s*gelu(g1)] (k the element's keep bit, s =
 *   1/(1-p)); fac may alias g. Backward: dg = [da * fac1 | da * fac2] (the keep bits need no
 *   second draw). */
int dna_geglu_fwd(const void* g, int dtype, int rows, int inter, float p_drop, uint64_t seed,
                  uint64_t offset, void* a, void* fac, void* stream);
int dna_geglu_bwd(const void* da, const void* fac, int dtype, int rows, int inter, void* dg,
                  void* stream);

/* ------------------------------------------------------------------ projections (MFMA GEMM)
 * The encoder's nn.Linear layers (bert_layers.py:158 Wqkv, :214 attention dense, :292
 * gated_layers, :297 wo, :560 MLM transform) and their backward, bf16 in / fp32 accumulate.
 * Row-major everywhere; w is the [N, K] nn.Linear weight (bf16 copy of the fp32 master).
 *   fwd    y[M,N]  = x[M,K] . w^T + bias      (bias fp32 [N] or NULL; K % 64 == 0, N % 8 == 0)
 *   dgrad  dx[M,K] = dy[M,N] . w             (N % 64 == 0, K % 8 == 0)
 *   wgrad  partials[s][N][K] = dy[rows_s]^T . x[rows_s]  for s < splits over equal row slices
 *          (M % (64*splits) == 0); reduce with dna_sum_slices_accum into the fp32 .grad. */
int dna_linear_fwd(const void* x, const void* w, const float* bias, int M, int N, int K, void* y,
                   void* stream);
int dna_linear_dgrad(const void* dy, const void* w, int M, int N, int K, void* dx, void* stream);
/* HyenaDNA Mlp fc1 + activation (flash_attn Mlp: fc2(act(fc1(x))), act = F.gelu(approximate=
 * "tanh"); standalone_hyenadna.py:431 Mlp): h[M,N] = x . w^T + bias (bf16) and
 * act[M,N] = bf16(gelu_tanh(h)) from one persistent-GEMM launch (N % 256 == 0, N <= 8192,
 * K % 128 == 0), replacing fc1's GEMM and torch's separate GELU pass; fc2's data gradient reads h
 * (dna_gelu_linear_dgrad_p), its forward and weight gradient read act. */
int dna_linear_gelu_fwd(const void* x, const void* w, const float* bias, int M, int N, int K,
                        void* h, void* act, void* stream);
int dna_linear_wgrad(const void* dy, const void* x, int M, int N, int K, int splits,
                     float* partials, void* stream);

/* Exact-fp32 projections (csrc/gemm_f32.hip, v_mfma_f32_16x16x4_f32): the fp32 parity mode of
 * the same nn.Linear layers (bert_layers.py:158,214,292,297,560,664) and their backward -- the
 * f32 path of the reference's torch fp32 forward, without a vendor GEMM. Any shape (edges
 * zero-filled), fp32 in / fp32 out.
 *   fwd    y[M,N]  = x[M,K] . w[N,K]^T (+ bias[N], may be null)
 *   dgrad  dx[M,K] = dy[M,N] . w[N,K]
 *   wgrad  partials[s][N][K] = slice s of dy[T,N]^T . x[T,K] (token split from
 *          dna_linear_wgrad_f32_splits); reduce with dna_sum_slices_accum. */
int dna_linear_fwd_f32(const float* x, const float* w, const float* bias, int M, int N, int K,
                       float* y, void* stream);
int dna_linear_dgrad_f32(const float* dy, const float* w, int M, int N, int K, float* dx,
                         void* stream);
int dna_linear_wgrad_f32_splits(int T, int N, int K);
int dna_linear_wgrad_f32(const float* dy, const float* x, int T, int N, int K, int splits,
                         float* partials, void* stream);

/* Strided batched GEMM for the Mamba mixer's skinny projections, computed channel-major so no
 * operand is transposed in memory (replaces the x_proj / dt_proj nn.Linear forward and backward
 * of mamba_ssm Mamba.forward as Caduceus builds it, modeling_caduceus.py:88-91):
 *   C[z][m][n] = sum_k A(m, k) B(k, n),  z = b * splits + s (k slice s of the contraction),
 *   A(m, k) = A[b*saz + m*sam + k*sak] (sak == 1 or sam == 1),
 *   B(k, n) = B[b*sbz + k*sbk + n*sbn] (sbk == 1 or sbn == 1),
 *   C + z*scz, row stride ldc; bf16 in, fp32 accumulate, bf16 or fp32 (out_f32 bit 0) out;
 *   out_f32 bit 1: C += A B (read-modify-write, one rounding after the sum; splits == 1) --
 *   the x_proj data gradient summed into the scan's du without a separate add;
 *   bias_m[M] / bias_n[N] optional (may be null).
 * Weight gradients: splits from dna_gemm_strided_splits, fp32 slices summed over z by
 * dna_sum_slices_accum. csrc/gemm_strided.hip (bf16, MFMA 16x16x32), csrc/gemm_f32.hip (fp32). */
int dna_gemm_strided_splits(int M, int N, int K, int batch);
int dna_gemm_bf16_strided(const void* A, long long sam, long long sak, long long saz,
                          const void* B, long long sbk, long long sbn, long long sbz,
                          void* C, long long ldc, long long scz, int out_f32,
                          const float* bias_m, const float* bias_n, int M, int N, int K,
                          int batch, int splits, void* stream);
/* C[z][c][l] = sum_{j<K} W[c][j] X[z][l'][j] (+ bias[c], fp32), l' = l (reverse == 0) or
 * N-1-l (reverse: the BiMamba reverse direction reads the sequence backwards instead of flipping
 * it in memory): a channel-major projection of a
 * token-major input (bf16; K in {64, 128, 256}, W / X 16-B aligned, C [batch][M][N]) with the
 * weight held in registers and X streamed: the Mamba in_proj forward, `in_proj.weight @
 * rearrange(hidden, "b l d -> d (b l)")` (mamba_ssm Mamba.forward under
 * modeling_caduceus.py:88-91). csrc/proj_cm.hip. */
int dna_proj_cm_bf16(const void* W, const void* X, const float* bias, int M, int N, int K,
                     int batch, int reverse, void* C, void* stream);
/* The same product with the contraction split over two A operands of equal strides:
 * C = [A | A2] . B, A supplying k < K1 and A2 k in [K1, K) (K1 % 32 == 0). Replaces the
 * mm + addmm pair of the Mamba in_proj data gradient (dh = g_x^T W_x + g_z^T W_z,
 * mamba_ssm Mamba.in_proj backward under modeling_caduceus.py:88-91). */
int dna_gemm_bf16_strided_cat(const void* A, const void* A2, int K1, long long sam, long long sak,
                              long long saz, const void* B, long long sbk, long long sbn,
                              long long sbz, void* C, long long ldc, long long scz, int out_f32,
                              const float* bias_m, const float* bias_n, int M, int N, int K,
                              int batch, int splits, void* stream);
int dna_gemm_f32_strided(const float* A, long long sam, long long sak, long long saz,
                         const float* B, long long sbk, long long sbn, long long sbz,
                         float* C, long long ldc, long long scz, const float* bias_n,
                         int M, int N, int K, int batch, int splits, void* stream);
/* dst[cols][rows] = src[rows][cols] (bf16; rows, cols % 8 == 0): the transposed weight copy kept
 * beside the bf16 weights, so the data gradient dx = dy . w runs as
 * dna_linear_fwd(dy, w^T, NULL, M, K, N, dx) on both-operands-K-major MFMA tiles (replaces the
 * dgrad half of torch.nn.Linear's autograd backward, bert_layers.py:158/:214/:292/:297/:560). */
int dna_transpose_bf16(const void* src, int rows, int cols, void* dst, void* stream);
/* Weight gradient on the persistent MFMA kernel, operands token-major as the forward left them:
 * partials[s][N][K] = sum over token chunk s of dy[t][N]^T x[t][K] (chunks of ceil(M/64)/splits
 * 64-token steps; N, K % 256 == 0; rows past M read as zero). splits from
 * dna_linear_wgrad_p_splits (fills the grid evenly); fold with dna_sum_slices_accum. Replaces
 * the weight half of torch.nn.Linear's autograd backward at the same call sites. */
int dna_linear_wgrad_p_splits(int M, int N, int K);
int dna_linear_wgrad_p(const void* dy, const void* x, int M, int N, int K, int splits,
                       float* partials, void* stream);
/* gated_layers + GeGLU + dropout in one launch (bert_layers.py:292-296):
 *   g = x[M,K] . wg^T + bias (bias fp32 [2F] or NULL; rounded to bf16, never stored),
 *   out[M, F] = dropout(gelu_erf(g[:, :F]) * g[:, F:]) and fac[M, 2F] = the backward factors of
 *   dna_geglu_fwd -- the same bits as dna_linear_fwd + dna_geglu_fwd (same Philox mask).
 * K % 64 == 0, F % 128 == 0. */
int dna_geglu_linear_fwd(const void* x, const void* wg, const float* bias, int M, int F, int K,
                         float p_drop, uint64_t seed, uint64_t offset, void* fac, void* out,
                         void* stream);
/* wo dgrad + GeGLU backward in one launch: da = dy[M,N] . wo ([N, F]), then
 * dg[M, 2F] = dna_geglu_bwd(bf16(da), fac). N % 64 == 0, F % 8 == 0. */
int dna_geglu_linear_dgrad(const void* dy, const void* wo, const void* fac, int M, int F, int N,
                           void* dg, void* stream);
/* The same on the persistent kernel (the training step's path), with wo's transposed bf16 copy
 * wt [F, N] (dna_transpose_bf16) as the K-major operand: dg[M, 2F] =
 * dna_geglu_bwd(bf16(dy . wt^T), fac); da never reaches memory. N % 128 == 0, F % 256 == 0.
 * Replaces the backward of wo's nn.Linear and of the GeGLU (bert_layers.py:292-297). */
int dna_geglu_linear_dgrad_p(const void* dy, const void* wt, const void* fac, int M, int F, int N,
                             void* dg, void* stream);

/* dh = gelu_tanh'(h) * bf16(dy . W) -- the data gradient of a Linear fed by a tanh-GELU (the
 * flash_attn Mlp's fc2 in the HyenaDNA Blocks, reference long_conv_lm.py create_mlp_cls with
 * activation gelu(approximate="tanh")) with torch's GeluBackward in the persistent kernel's
 * epilogue. dy [M][N] bf16, wt = W^T [F][N] bf16 (W [N][F]), h / dh [M][F] bf16;
 * N % 128 == 0, F % 256 == 0. */
int dna_gelu_linear_dgrad_p(const void* dy, const void* wt, const void* h, int M, int F, int N,
                            void* dh, void* stream);

/* ------------------------------------------------------------------ HyenaDNA FFT long convolution
 * fftconv_ref (src/models/sequence/hyena.py:60-92) as used by HyenaFilter.forward (:253-280):
 *   y[b,d,t] = sum_{j<L} k[d,j] * u~[b,d,(t-j) mod 2L] + bias[d] * u[b,d,t],   t < L
 * u, y [B, D, L] (dtype: DNA_F32 / DNA_BF16), k [D, L] fp32, bias [D] fp32 or NULL; u~ = u
 * zero-padded to 2L at offset 0 (causal) or pad_before = L/2 (bidirectional, :68-74).
 * L must be a power of two in [64, 131072]. Internally fp32 (four-step FFT of size 2L).
 * kspec: dna_fftconv_kspec_elems(L) floats per channel, written by dna_fftconv_filter: the
 * spectrum of k with the bias folded in as the filter tap that reproduces bias*u (so fwd and bwd
 * take no bias). Its workspace: ceil(D/2) * 2L complex64; dna_fftconv_workspace(1, D, L) is enough. */
size_t dna_fftconv_workspace(int B, int D, int L);
size_t dna_fftconv_kspec_elems(int L);
int dna_fftconv_filter(const float* k, const float* bias, int D, int L, int bidirectional,
                       void* kspec, void* ws, size_t ws_bytes, void* stream);
/* uspec (may be NULL): receives the spectrum of the padded input, ceil(B/2)*D*4L floats, for
 * dna_fftconv_bwd to reuse (saves recomputing it for dk). */
int dna_fftconv_fwd(const void* u, int dtype, const void* kspec, int B, int D, int L,
                    int bidirectional, void* y, void* uspec, void* ws, size_t ws_bytes,
                    void* stream);
/* Gradients of sum(dy * y): du (like u, may be NULL), dk [D, L] fp32 (may be NULL),
 * dbias [D] fp32 (may be NULL). uspec: the forward's saved input spectrum or NULL (recomputed).
 * ws: dna_fftconv_workspace(B, D, L) bytes. */
int dna_fftconv_bwd(const void* dy, const void* u, int dtype, const void* kspec, const void* uspec,
                    int B, int D, int L, int bidirectional, void* du, float* dk, float* dbias,
                    void* ws, size_t ws_bytes, void* stream);

/* ------------------------------------------------------------------ HyenaOperator data movement
 * Around the long convolution in HyenaOperator.forward (src/models/sequence/hyena.py:421-509,
 * num_heads = num_blocks = inner_factor = 1): u = in_proj(x) [B, L, C = (order+1)*d] token-major
 * -> depthwise causal Conv1d (weight [C][K] fp32, bias [C] fp32; padding K-1, first L outputs,
 * :423-425) -> split x_0 .. x_{order-1}, v -> first gate v * x_{order-1} (:459-465).
 * d % 64 == 0, order 2..4, K 2..4; u/xs/vx in dtype (f32 or bf16), fp32 math.
 * xs [B, order-1, d, L] = x_0 .. x_{order-2}; vx [B, d, L] (channel-major, the long conv's layout). */
int dna_hyena_shortconv_fwd(const void* u, int dtype, const float* w, const float* bias, int B,
                            int L, int d, int order, int K, void* xs, void* vx, void* stream);
/* Backward: dxs [B, order-1, d, L], dvx [B, d, L] -> du [B, L, C] (written); dw/dbias as fp32
 * partials part [B * ceil(L/64)][C][K+1] (last column = bias), summed by dna_colsum_f32. */
size_t dna_hyena_shortconv_part_elems(int B, int L, int d, int order, int K);
int dna_hyena_shortconv_bwd(const void* u, int dtype, const float* w, const float* bias, int B,
                            int L, int d, int order, int K, const void* dxs, const void* dvx,
                            void* du, float* part, void* stream);
/* y [B, L, d] = (yc * x_0) rearranged "b d l -> b l d" (:503-507); x_0 rows at x0 + b*x0_bstride. */
int dna_hyena_gate_out_fwd(const void* yc, const void* x0, int dtype, int B, int L, int d,
                           size_t x0_bstride, void* y, void* stream);
/* dyc = dy * x_0, dx0 = dy * yc (channel-major; dx0 with the same batch stride as x_0). */
int dna_hyena_gate_out_bwd(const void* dy, const void* yc, const void* x0, int dtype, int B, int L,
                           int d, size_t x_bstride, void* dyc, void* dx0, void* stream);

/* HyenaFilter's ExponentialModulation fused with the filter transpose (reference hyena.py:140-163,
 * :438-441): k[o][v][t] = h[t][c] * (exp(-tpos[t] * |delta[c]|) + shift), c = v * O + o, for
 * h [L, C] (dtype fp32 / bf16), k [O][C / O][L] fp32. Backward: dh[t][c] = dk[o][v][t] * (same
 * factor) in h's dtype (delta taken as a constant: the reference registers it with lr 0). */
int dna_hyena_modulate_t_fwd(const void* h, int dtype, const float* tpos, const float* delta,
                             float shift, int L, int C, int O, float* k, void* stream);
int dna_hyena_modulate_t_bwd(const float* dk, const float* tpos, const float* delta, float shift,
                             int L, int C, int O, void* dh, int dtype, void* stream);

/* HyenaFilter's implicit filter whole (reference hyena.py:162-247 filter() + the modulation and
 * transpose above): k = modulate(Linear_out(Sin(... Sin(Linear_1(z)) ...))) under the bf16
 * autocast dtype flow (each Linear on bf16-rounded input / weight / bias, bf16 output; Sin in
 * fp32; one shared freq). z [L][E] fp32 (E <= 8), w1 [64][E], b1 [64], wi / bi: NI <= 4 host
 * arrays of device pointers to [64][64] / [64] fp32, w4 [C][64] (C in {64, 128, 256, 512}),
 * freq [64], tpos [L], delta [C]; L % 64 == 0; k [O][C / O][L] fp32. Backward: per-block
 * partial gradients part [grid][dna_hyena_filter_part_stride()] (dna_hyena_filter_part_elems()
 * floats in all; layout w4 [C][64], wi [NI][64][64], bi [NI][64], w1 [64][E], b1 [64], freq [64])
 * for dna_sum_slices, and dz [L][E] (bf16-rounded) when dz is non-null. csrc/hyena_filter.hip. */
int dna_hyena_filter_part_elems(int L, int E, int NI, int C);
int dna_hyena_filter_part_stride(int E, int NI, int C);
int dna_hyena_filter_fwd(const float* z, const float* w1, const float* b1, const float* const* wi,
                         const float* const* bi, int NI, const float* w4, const float* freq,
                         const float* tpos, const float* delta, float shift, int L, int E, int C, int O,
                         float* k, void* stream);
int dna_hyena_filter_bwd(const float* z, const float* w1, const float* b1, const float* const* wi,
                         const float* const* bi, int NI, const float* w4, const float* freq,
                         const float* tpos, const float* delta, float shift, int L, int E, int C, int O,
                         const float* dk, float* part, float* dz, void* stream);
/* the backward's gradient: out[i] = sum_g part[g * P + i] over the G = part_elems / P slices in
 * order, rounded to bf16 (and back) for i < nround -- the weight / bias entries -- fp32 after */
int dna_hyena_filter_finish(const float* part, int G, int P, int nround, float* out, void* stream);

/* ------------------------------------------------------------------ causal depthwise conv1d (+ SiLU)
 * Mamba.forward's x = silu(conv1d(x)[..., :L]) (depthwise, kernel K = d_conv, padding K-1;
 * mamba_ssm via modeling_caduceus.py:88-91): x [B, C, L] (batch stride x_bstride elements,
 * contiguous rows), w [C][K] fp32, bias [C] fp32 or NULL, silu 0/1; out [B, C, L] contiguous.
 * K in 2..4, dtype f32/bf16, fp32 math. */
int dna_causal_conv1d_fwd(const void* x, size_t x_bstride, int dtype, const float* w,
                          const float* bias, int B, int C, int L, int K, int silu, void* out,
                          void* stream);
/* Backward: dx (batch stride dx_bstride) written; dw/dbias partials part
 * [dna_causal_conv1d_part_rows(B, L)][C][K+1] (last column = bias), summed by dna_colsum_f32. */
size_t dna_causal_conv1d_part_rows(int B, int L);
int dna_causal_conv1d_bwd(const void* x, size_t x_bstride, int dtype, const float* w,
                          const float* bias, const void* dout, int B, int C, int L, int K,
                          int silu, void* dx, size_t dx_bstride, float* part, void* stream);

/* ------------------------------------------------------------------ Mamba selective scan (Caduceus)
 * selective_scan_fn as called by mamba_ssm Mamba.forward inside Caduceus' BiMambaWrapper
 * (src/models/caduceus/modeling_caduceus.py:68-121; mamba_ssm is external and not vendored):
 *   delta = softplus(delta + delta_bias) (if delta_softplus; bias may be NULL)
 *   x_t = exp(delta_t A) x_{t-1} + delta_t B_t u_t ;  out_t = (C_t . x_t + D u_t) * silu(z_t)
 * u, delta, z, out [batch, dim, len] (dtype), A [dim, d_state] fp32, B, C [batch, d_state, len]
 * (dtype), D, delta_bias [dim] fp32 (NULL allowed; z NULL = no gating). d_state in {4, 8, 16}.
 * states: dna_selective_scan_states() floats (fp32): chunk-start states kept for the backward,
 * chunk delta sums and the backward's reverse-carry scratch; NULL skips them (and the
 * chunk-parallel kernels, which need the buffer as workspace).
 * last_state [batch, dim, d_state] fp32 or NULL. */
size_t dna_selective_scan_states(int batch, int dim, int len, int d_state);
int dna_selective_scan_fwd(const void* u, const void* delta, const float* A, const void* B,
                           const void* C, const float* D, const void* z, const float* delta_bias,
                           int delta_softplus, int dtype, int batch, int dim, int len, int d_state,
                           void* out, float* states, float* last_state, void* stream);
/* Backward from the forward's states (the buffer's reverse-carry region is rewritten; the
 * forward's part is only read). du, ddelta, dz (dtype) are written; dA [dim, d_state],
 * dB, dC [batch, d_state, len], dD, ddelta_bias [dim] (fp32) are ACCUMULATED (+=, zero them). */
int dna_selective_scan_bwd(const void* u, const void* delta, const float* A, const void* B,
                           const void* C, const float* D, const void* z, const float* delta_bias,
                           int delta_softplus, int dtype, int batch, int dim, int len, int d_state,
                           float* states, const void* dout, void* du, void* ddelta,
                           float* dA, float* dB, float* dC, float* dD, void* dz,
                           float* ddelta_bias, void* stream);

/* ------------------------------------------------------------------ masked-LM cross entropy
 * Per-row CE over the masked rows only (the model computes logits only for labels>0 rows,
 * bert_layers.py:795,:820-824; task loss bert_cross_entropy, src/tasks/metrics.py:268-273).
 *   logits [rows, vocab] dtype; target [rows] int64 -> row_loss, row_lse [rows] fp32. */
int dna_xent_fwd(const void* logits, int dtype, const int64_t* target, int rows, int vocab,
                 float* row_loss, float* row_lse, void* stream);
/* dlogits = (softmax - onehot) * dloss[0] * scale, in logits' dtype. dloss: device scalar. */
int dna_xent_bwd(const void* logits, int dtype, const int64_t* target, const float* row_lse,
                 const float* dloss, float scale, int rows, int vocab, void* dlogits,
                 void* stream);

/* ------------------------------------------------------------------ optimizer (flat buffers)
 * Lightning gradient_clip_val=1.0 (torch.nn.utils.clip_grad_norm_) + torch AdamW
 * (train.py:462-542, registry.optimizer["adamw"]) over ONE flat fp32 parameter buffer.
 * dna_sumsq writes sum(x^2) to out[0] (device). dna_adamw_step reads that sum (if grad_sumsq is
 * not NULL) and applies clip coef min(1, max_norm/(sqrt(sumsq)+1e-6)) * grad_scale to each grad,
 * then the decoupled-weight-decay Adam update; optionally refreshes a bf16 copy of the params. */
size_t dna_sumsq_workspace(size_t n);
int dna_sumsq(const float* x, size_t n, float* out, void* workspace, size_t workspace_bytes,
              void* stream);
int dna_adamw_step(float* param, const float* grad, float* exp_avg, float* exp_avg_sq,
                   void* param_bf16, size_t n, float lr, float beta1, float beta2, float eps,
                   float weight_decay, int step, const float* grad_sumsq, float max_grad_norm,
                   float grad_scale, void* stream);

/* ------------------------------------------------------------------ data path (host, C++)
 * BPE tokenizer: bit-exact with the reference's HF `tokenizers` BPE for
 * DNABERT-2-117M/tokenizer.json as called at src/dataloaders/datasets/hg38_dataset.py:369-379.
 * Accepts an HF tokenizer.json or dna_amd/data/dnabert2_bpe.json. Handles are immutable after
 * creation: thread-safe and fork-safe (DataLoader workers). */
typedef struct dna_bpe dna_bpe;
dna_bpe* dna_bpe_create(const char* json_path);
void dna_bpe_destroy(dna_bpe* h);
int dna_bpe_vocab_size(const dna_bpe* h);
/* Raw encode (no special tokens). Returns the token count (may exceed cap: then only cap ids
 * were written) or a negative DNA_ERR_* code. */
int dna_bpe_encode(const dna_bpe* h, const char* text, int len, int32_t* out_ids, int cap);
/* Dataset-style batch encode: ids = ([CLS] + bpe[:P-2] + [SEP] + [PAD]*)[1:-1] (add_eos 0) or
 * [1:] (add_eos 1). out_ids [n, P-2+add_eos]; out_lens [n] = bpe tokens kept (may be NULL).
 * nthreads <= 0: one thread per hardware core. */
int dna_bpe_encode_batch(const dna_bpe* h, const char* const* seqs, const int* lens, int n,
                         int pad_max_length, int add_eos, int32_t* out_ids, int32_t* out_lens,
                         int nthreads);

/* bert_mask (hg38_dataset.py:238-286): mask = (seq != pad) & U1 < mask_prob; labels = seq or -100;
 * U2 < 1-rand-unchanged -> mask_id; next rand_prob -> uniform non-special id; rest unchanged.
 * _from_draws takes the uniforms / random ids explicitly (exact parity with the reference draws);
 * dna_bert_mask draws them from Philox4x32-10 keyed by (seed, sample_id). */
int dna_bert_mask_from_draws(const int64_t* seq, int n, const float* u1, const float* u2,
                             const int64_t* rand_tok, int mask_id, int pad_id, float mask_prob,
                             float rand_prob, float unchanged_prob, int64_t* out_seq,
                             uint8_t* out_mask, int64_t* out_labels);
int dna_bert_mask(const int64_t* seq, int n, int vocab, const int64_t* special_ids, int n_special,
                  int mask_id, int pad_id, float mask_prob, float rand_prob, float unchanged_prob,
                  uint64_t seed, uint64_t sample_id, int64_t* out_seq, uint8_t* out_mask,
                  int64_t* out_labels);

/* FASTA (+ .fai; created in memory when absent) via mmap -- replaces pyfaidx.Fasta used by
 * FastaInterval (hg38_dataset.py:40-124). Case is preserved like pyfaidx's default. */
typedef struct dna_fasta dna_fasta;
dna_fasta* dna_fasta_open(const char* path);
void dna_fasta_close(dna_fasta* h);
int dna_fasta_num_records(const dna_fasta* h);
const char* dna_fasta_record_name(const dna_fasta* h, int i);
int64_t dna_fasta_record_length(const dna_fasta* h, const char* name);
/* FastaInterval.__call__ (hg38_dataset.py:72-124) for BED interval [start, end):
 * writes the window to out (not NUL-terminated), its length to out_len. rc != 0 reverse-
 * complements (the caller draws the rc_aug coin). */
int dna_fasta_interval(const dna_fasta* h, const char* name, int64_t start, int64_t end,
                       int64_t max_length, int pad_interval, int rc, char* out, int64_t cap,
                       int64_t* out_len);

#ifdef __cplusplus
}
#endif
#endif /* DNA_AMD_H */
