/*
 * libvpf — C-ABI of the MI355X (gfx950) tracking hot path.
 *
 * The reference (tugitbartlomiej/ViTParticleFilterTracker) is a README with no code: its ViT feature
 * extractor and particle filter are named at /root/reference/README.md:7-8 and driven per frame by
 * main.py (README.md:37, 42). It has no FFI; the interface each entry point replaces is therefore the
 * SPEC.md / SURVEY.md §8a row it implements (H1..H14), and the Python binding that a maintainer of the
 * reference would add is `vitparticlefiltertracker_amd/_lib.py` (INTEGRATION.md shows it).
 *
 * Conventions:
 *   - Every pointer is DEVICE memory unless the parameter name ends in `_host`.
 *   - The caller allocates every buffer, including workspaces; the library never allocates or frees.
 *   - Every call only enqueues work on `stream` (a hipStream_t) and never synchronises: re-entrant,
 *     stream-ordered, asynchronous, graph-capturable.
 *   - Return value: 0 on success, otherwise a hipError_t code, or VPF_ERR_ARG (-1) for an argument that
 *     violates the documented shape contract (checked on the host before any launch).
 *   - bf16 tensors are passed as uint16_t (bit pattern of bfloat16).
 *   - Particles are structure-of-arrays float[3][ld] (rows x, y, scale), `ld` >= n.
 */
#ifndef VPF_H
#define VPF_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define VPF_ERR_ARG (-1)

/* GEMM epilogues (vpf_gemm_bf16 / vpf_gemm_f32) */
#define VPF_EPI_BIAS 0          /* C = A W^T + bias                                              */
#define VPF_EPI_BIAS_GELU 1     /* C = gelu_erf(A W^T + bias)                                      */
#define VPF_EPI_BIAS_RESIDUAL 2 /* C = R + (A W^T + bias); R may alias C                          */
#define VPF_EPI_PATCH 3         /* row m -> token (m/g2)*(g2+1)+1+m%g2; C = A W^T + bias + pos[1+m%g2] */
#define VPF_EPI_LN 4            /* LayerNorm folded: C = rstd_m (A W'^T) - rstd_m mean_m colsum + bias'     */
#define VPF_EPI_LN_GELU 5       /* gelu_erf of the above                                                  */

/* library identity: returns a static string "libvpf <version> gfx950" */
const char* vpf_version(void);

/* H1 ParticleFilter.predict: SPEC S2, in place on particles[3][ld] (n local particles whose global
 * indices start at global_begin). */
int vpf_predict(float* particles, int64_t n, int64_t ld, int64_t global_begin, uint64_t seed,
                uint32_t frame, float sig_x, float sig_y, float sig_s, float width, float height,
                float smin, float smax, void* stream);

/* H2+H3 (A operand of the patch embed): bilinear crop + normalise + im2col, SPEC S3.
 * frame: uint8[H][W][3]; rgba_ws: caller-owned workspace of (H+2)*(W+2) uint32 (the zero-bordered RGBA
 * frame the taps read; rewritten by every call); out: [n * (S/patch)^2][Kp] bf16 (vpf_crop_patches_bf16) or
 * fp32 (_f32). norm_ab_host: 6 floats {a0,a1,a2,b0,b1,b2} (SPEC S3). Requires Kp % 8 == 0, Kp >= 3*patch^2. */
int vpf_crop_patches_bf16(const uint8_t* frame, int H, int W, uint32_t* rgba_ws, const float* particles,
                          int64_t ld, int64_t n, float w0, float h0, int S, int patch, int Kp,
                          const float* norm_ab_host, uint16_t* out, void* stream);
int vpf_crop_patches_f32(const uint8_t* frame, int H, int W, uint32_t* rgba_ws, const float* particles,
                         int64_t ld, int64_t n, float w0, float h0, int S, int patch, int Kp,
                         const float* norm_ab_host, float* out, void* stream);

/* H3 (CLS row): tokens[p][0][:] = cls + pos[0] for p < n_part; tokens: [n_part][N][D].
 * stats_out (bf16 only, may be NULL): the CLS rows' entries of the GEMM stats planes (see vpf_gemm_bf16):
 * fp32[parts][n_part*N][2], plane 0 row p*N = {sum, sumsq} of the stored bf16 row, planes 1.. = 0. */
int vpf_cls_rows_bf16(uint16_t* tokens, int64_t n_part, int N, int D, const float* cls,
                      const float* pos, float* stats_out, int parts, void* stream);
int vpf_cls_rows_f32(float* tokens, int64_t n_part, int N, int D, const float* cls, const float* pos,
                     void* stream);

/* H3/H5/H7/H8: C[M][N] = epilogue(A[M][K] * W[N][K]^T). bf16 in/out, fp32 accumulate (MFMA).
 * Row m of A at A + m*lda; row m of C (and of the residual, which has C's layout) at C + m*ldc.
 * bias: fp32[N]; residual: bf16 (EPI_BIAS_RESIDUAL, may alias C); pos: fp32[g2+1][N] (EPI_PATCH, with
 * g2 = patch_rows, M % g2 == 0); EPI_LN / EPI_LN_GELU (LayerNorm folded into the GEMM, A = the raw
 * residual stream): W = W * diag(gamma), colsum fp32[N] = sum_k W[n][k] (of the bf16 W), bias = b + W_orig beta,
 * and row_stats either (stats_parts == 0) fp32[M][2] = {mean, rstd} of A's rows (vpf_row_stats_*), or
 * (stats_parts = P in 1..16) fp32[P][M][2] planes of {sum, sumsq} over
 * disjoint column blocks of A's rows (the stats_out of the GEMM that produced A), combined with eps = ln_eps:
 * rstd = 1/sqrt(sumsq/K - mean^2 + eps).
 * stats_out (EPI_BIAS_RESIDUAL / EPI_PATCH only, may be NULL): fp32[ceil(N/64)][R][2] planes, plane t =
 * {sum, sumsq} of the stored bf16 values of each output row over columns [64t, 64t+64); R = M, or
 * (M/g2)*(g2+1) token rows for EPI_PATCH (plane rows of the CLS tokens are left to vpf_cls_rows_bf16).
 * C8 / Cs (EPI_BIAS_RESIDUAL / EPI_PATCH only, may be NULL): an MX8 copy of the stored bf16 output (rows as in
 * C: token rows for EPI_PATCH) — the A operand of a following vpf_gemm_mx8; ld8 bytes per element row,
 * lds_c >= output rows; requires N % 128 == 0 (see "MX8 operands" below).
 * Unused pointers may be NULL. Requires K % 64 == 0, N % 8 == 0, lda % 8 == 0, ldc % 8 == 0. */
int vpf_gemm_bf16(const uint16_t* A, int64_t lda, const uint16_t* W, const float* bias,
                  const uint16_t* residual, const float* pos, int patch_rows, const float* row_stats,
                  const float* colsum, uint16_t* C, int64_t ldc, int64_t M, int64_t N, int64_t K,
                  int epilogue, int stats_parts, float ln_eps, float* stats_out, uint8_t* C8, int64_t ld8,
                  uint32_t* Cs, int64_t lds_c, void* stream);
/* Split-K form of vpf_gemm_bf16 for GEMMs with few rows (the last block's CLS-row GEMMs): `splits` blocks per
 * 256 x 256 output tile each run K/splits of the K loop into fp32 partial planes (partial_ws: fp32[splits][M][N],
 * ws_elems >= splits*M*N, 16-B aligned), then one pass sums the planes in split order and applies the epilogue.
 * The summation order is fixed by (K, splits), never by M, so a row's result does not depend on how many rows the
 * call has. Epilogues: VPF_EPI_BIAS, _BIAS_GELU, _BIAS_RESIDUAL (residual: C's layout, may alias C; stats_out
 * optional, as vpf_gemm_bf16's with R = M, N % 64 == 0), _LN, _LN_GELU (row_stats = {mean, rstd} per row, colsum).
 * Requires K % (64*splits) == 0, 1 <= splits <= 64, N % 8 == 0, lda % 8 == 0, ldc % 8 == 0, 16-B aligned A, W, C. */
int vpf_gemm_bf16_splitk(const uint16_t* A, int64_t lda, const uint16_t* W, const float* bias,
                         const uint16_t* residual, const float* row_stats, const float* colsum, uint16_t* C,
                         int64_t ldc, int64_t M, int64_t N, int64_t K, int epilogue, int splits, float* stats_out,
                         float* partial_ws, int64_t ws_elems, void* stream);
/* Kernel choice for vpf_gemm_bf16 (process-wide; call it only between launches; tests and A/B timing). The product
 * library has two bf16 kernels and both give the same bits for every epilogue: kernel 1 = the deep-ring k_gemm_bf16
 * (3 A + 2 B K-tiles in LDS), 5 = the ping-pong k_gemm_pp (<= 15 statistics planes; otherwise kernel 1's form).
 * kernel 0 = the per-shape defaults (5 for VPF_EPI_LN, 1 otherwise; A-panel group 2 for N <= 1024, 8 for
 * VPF_EPI_LN_GELU, 4 otherwise). kernel 1 / 5 apply to every shape, with group >= 0 as the A-panel group size of the
 * tile order for every shape (also used by vpf_gemm_mx8; 0 = row-major) or -1 for the per-shape groups. Returns
 * VPF_ERR_ARG for any other kernel (the A/B variants of earlier rounds are in the lab build, tools/gemm_lab) or a
 * group outside [-1, 64]. Nothing in the library reads the environment. */
int vpf_gemm_tune(int kernel, int group);

/* MX8 operands (OCP MX-FP8: e4m3fn elements, one e8m0 scale per 32 consecutive K values):
 *   elements X8[r][k] (uint8, row stride ld8 bytes); scales (e8m0 bytes) in one plane of lds uint32 words per
 *   128-deep K-tile (lds % 64 == 0, lds >= rows), rows in bricks of 64: the scale of row r for K values
 *   [32*(k/32), +32) is byte (r/16)%4 of word (k/128)*lds + (r/64)*64 + ((k/32)%4)*16 + r%16.
 *   value(r, k) = e4m3(X8[r][k]) * 2^(scale - 127).
 * Quantisation (vpf_quantize_mx8 and every fp8-producing epilogue): per block, E = the smallest exponent with
 * amax * 2^-E <= 448 (no element saturates), clamped to [-127, 125]; byte = E + 127; elements = RNE(x * 2^-E).
 *
 * fp8 weight path (configs[4]): C[M][N] = epilogue(value(A8)[M][K] . value(W8)[N][K]^T), fp32 accumulation on
 * v_mfma_scale_f32_16x16x128_f8f6f4. A8 / As: lda bytes per row (lda % 16 == 0), scale planes of lds_a
 * words; W8 [N][K] bytes, Ws scale planes of N words (N % 64 == 0). Epilogues as vpf_gemm_bf16 except EPI_PATCH; LN
 * epilogues take colsum = the row sums of value(W8) and stats_parts <= 13. C (bf16, may be NULL when C8 is
 * given) and/or C8 / Cs (MX8 copy of the output, N % 128 == 0). 16-B aligned A8, W8, As, Ws; K % 128 == 0,
 * N % 8 == 0. */
int vpf_gemm_mx8(const uint8_t* A8, int64_t lda, const uint32_t* As, int64_t lds_a, const uint8_t* W8,
                 const uint32_t* Ws, const float* bias, const uint16_t* residual, const float* row_stats,
                 const float* colsum, uint16_t* C, int64_t ldc, uint8_t* C8, int64_t ld8, uint32_t* Cs,
                 int64_t lds_c, int64_t M, int64_t N, int64_t K, int epilogue, int stats_parts, float ln_eps,
                 float* stats_out, void* stream);
/* bf16 rows -> MX8: row r of X (at X + r*ldx) -> element row r*out_stride of X8 and its scale words.
 * K % 128 == 0, X 16-B aligned, ld8 % 8 == 0, lds >= (rows-1)*out_stride + 1. */
int vpf_quantize_mx8(const uint16_t* X, int64_t ldx, int64_t rows, int64_t K, int64_t out_stride, uint8_t* X8,
                     int64_t ld8, uint32_t* S, int64_t lds, void* stream);
/* fp32 parity mode: same contract with fp32 tensors (exact-f32 MFMA, v_mfma_f32_32x32x2_f32).
 * Requires K % 32 == 0, lda % 4 == 0, ldc % 4 == 0. */
int vpf_gemm_f32(const float* A, int64_t lda, const float* W, const float* bias, const float* residual,
                 const float* pos, int patch_rows, const float* row_stats, const float* colsum, float* C,
                 int64_t ldc, int64_t M, int64_t N, int64_t K, int epilogue, void* stream);

/* H4 (folded form): out[r] = {mean, rstd = 1/sqrt(var + eps)} of row r (at x + r*x_stride), fp32.
 * bf16: D % 8 == 0; fp32: D % 4 == 0; D <= 1024. */
int vpf_row_stats_bf16(const uint16_t* x, int64_t rows, int D, int64_t x_stride, float eps, float* out,
                       void* stream);
int vpf_row_stats_f32(const float* x, int64_t rows, int D, int64_t x_stride, float eps, float* out,
                      void* stream);

/* H4 (folded form, from the producers' statistics planes): out[r] = {mean, rstd} of row r from parts planes
 * fp32[parts][plane_stride][2] of {sum, sumsq} over disjoint column blocks (a vpf_gemm_bf16 stats_out), D the row
 * length: mean = sum/D, rstd = 1/sqrt(max(sumsq/D - mean^2, 0) + eps), computed exactly as vpf_gemm_bf16's in-kernel
 * combine (so an EPI_LN* GEMM given these {mean, rstd} with stats_parts = 0 writes the same bits as one given the
 * planes). For consumers whose plane count exceeds what the ping-pong GEMM keeps in LDS (ViT-L: 16). */
int vpf_stats_combine(const float* planes, int parts, int64_t plane_stride, int64_t rows, int D, float eps, float* out,
                      void* stream);

/* H4: y = LayerNorm(x) per row (fp32 statistics). Row r of x at x + r*x_stride; D % 4 == 0, D <= 1024. */
int vpf_layernorm_bf16(const uint16_t* x, int64_t rows, int D, int64_t x_stride, const float* gamma,
                       const float* beta, float eps, uint16_t* y, int64_t y_stride, void* stream);
int vpf_layernorm_f32(const float* x, int64_t rows, int D, int64_t x_stride, const float* gamma,
                      const float* beta, float eps, float* y, int64_t y_stride, void* stream);

/* H6: per (particle, head) softmax(q k^T * scale) v. qkv: [B][N][3][H][hd], out: [B][N][H][hd].
 * Only the first q_rows queries of every particle are computed (q_rows = N: all; 1: the CLS row, used by
 * the last encoder layer whose other rows feed nothing). hd == 64, N <= 640 (f32: N <= 4096, keys streamed through LDS in 128-key chunks). */
int vpf_attention_bf16(const uint16_t* qkv, uint16_t* out, int64_t B, int N, int H, int hd,
                       float scale, int q_rows, void* stream);
/* fp8 path: vpf_attention_bf16 (all N <= 256 query rows) writing its output as MX8 (out8 / s8: the A operand of
 * the MX8 proj GEMM, "MX8 operands" at vpf_gemm_mx8; D = H*hd, D % 128 == 0, lds >= B*N) instead of bf16. */
int vpf_attention_bf16_mx8(const uint16_t* qkv, int64_t B, int N, int H, int hd, float scale, uint8_t* out8,
                           int64_t ld8, uint32_t* s8, int64_t lds, void* stream);
int vpf_attention_f32(const float* qkv, float* out, int64_t B, int N, int H, int hd, float scale,
                      int q_rows, void* stream);
/* H6 for the last block's CLS query with K and V never materialised (LN-folded bf16 mode). With
 * LNraw_j = (h_j - mean_j) rstd_j (statistics from the planes, as vpf_gemm_bf16's stats_parts), G_h the D-vector
 * W'_k,h^T q_h and c0_h = q_h . bk_h:  p_h = softmax_j((LNraw_j . G_h + c0_h) scale),  out_h = sum_j p_hj LNraw_j.
 * The caller finishes o_h = W'_v,h out_h + b'_v,h with one GEMM over the [n*H][D] rows of out and
 * vpf_head_gather_bf16 (vit.py).
 * tokens: bf16 [n_part][N][D] contiguous (D = 64 H, H in {6, 12, 16}, N <= 640); planes: fp32 [H][plane_rows][2]
 * {sum, sumsq} per 64-column block, row p*N + j; G: bf16 rows of ldg >= H*D ([h][D] per particle);
 * q: bf16 CLS queries (row stride ldq); bk: fp32[D]; out: bf16 rows of ldo >= H*D ([h][D]). */
/* out[p][h*hd + d] = Y[p*H + h][h*hd + d] for p < n (the diagonal blocks of a per-(particle, head) projection
 * Y: bf16 [n*H][H*hd] contiguous); out rows of ldo >= H*hd elements. hd % 8 == 0, 16-B aligned pointers. */
int vpf_head_gather_bf16(const uint16_t* Y, int64_t n, int H, int hd, uint16_t* out, int64_t ldo, void* stream);
int vpf_cls_attn_fold_bf16(const uint16_t* tokens, int64_t n_part, int N, int H, const float* planes,
                           int64_t plane_rows, float eps, const uint16_t* G, int64_t ldg, const uint16_t* q,
                           int64_t ldq, const float* bk, float scale, uint16_t* out, int64_t ldo, void* stream);

/* H9+H10: final LayerNorm of each particle's CLS row (tokens + p*N*D), cosine similarity with the
 * unit template `tmpl`, w = exp(lam (sim - 1)), Q = floor(w 2^bits) (SPEC S5).
 * feat_out (optional, may be NULL): fp32[n][D] LN'd CLS features. sim_out (optional): fp32[n]. */
int vpf_cls_weight_bf16(const uint16_t* tokens, int64_t n, int N, int D, const float* gamma,
                        const float* beta, float eps, const float* tmpl, float lam, int bits,
                        float* feat_out, float* sim_out, int64_t* Q, void* stream);
int vpf_cls_weight_f32(const float* tokens, int64_t n, int N, int D, const float* gamma,
                       const float* beta, float eps, const float* tmpl, float lam, int bits,
                       float* feat_out, float* sim_out, int64_t* Q, void* stream);

/* H10 alone (ParticleFilter.update with explicit features): feat fp32[n][D] (already LN'd CLS features),
 * same weight rule as vpf_cls_weight_*. */
int vpf_cosine_weight_f32(const float* feat, int64_t n, int D, const float* tmpl, float lam, int bits,
                          float* sim_out, int64_t* Q, void* stream);

/* H11: shard partial sums, SPEC S6. out_T: int64[1] = sum Q; out_sums: fp64[3] = sum Q*{x,y,s}.
 * Fixed-order tree reduction (deterministic run to run). */
int vpf_shard_stats(const int64_t* Q, const float* particles, int64_t ld, int64_t n, int64_t* out_T,
                    double* out_sums, void* stream);

/* H12: systematic resample of the slots [slot_begin, slot_end) whose positions fall in this shard
 * (SPEC S7). Q: local weights (n_local); offset: sum of the weights of the shards before this one;
 * total: global sum T; P: global particle count; U: Philox offset word; uniform != 0 treats every
 * Q_i as 1 (T == 0 fallback; the caller passes offset/total in those units).
 * Writes anc_out[j - slot_begin] = global ancestor index (local + global_begin) and
 * states_out[3][out_ld] (x, y, s of the ancestor). cdf_ws: int64[n_local] workspace. */
int vpf_resample(const int64_t* Q, int64_t n_local, int64_t global_begin, int64_t offset,
                 int64_t total, int64_t P, uint32_t U, int uniform, int64_t slot_begin,
                 int64_t slot_end, const float* particles, int64_t ld, int32_t* anc_out,
                 float* states_out, int64_t out_ld, int64_t* cdf_ws, void* stream);

/* H11 + H12 over the GLOBAL particle set, device-resident (the product path of ParticleFilter): every rank
 * holds all P weights and states — its own arrays (world 1: one shard, n_shard = P) or the all-gathered shard
 * chunks (world > 1) — so nothing goes back to the host between the weights and the resample.
 * Global index i is shard r = i / n_shard, k = i % n_shard: Q_i = Q[r*q_stride + k] (int64),
 * (x, y, s)_i = particles[r*p_stride + k + {0, ld, 2*ld}] (fp32).
 * stats_out: int64[4] = {T = sum Q, then the bits of the fp64 sums sum Q*x, Q*y, Q*s} (SPEC S6, fixed-order tree
 * over the global index, so every rank and every world size gets the same bits; when T == 0 the sums are taken
 * with every Q_i = 1 and the estimate is sum / P). cdf_ws: int64[P] workspace (the inclusive CDF).
 * Resample (SPEC S7, uniform when T == 0) of the output slots [slot_begin, slot_end): anc_out = global ancestor
 * index, states_out[3][out_ld] its state. The resample word U = Philox(ctr = (0, frame, 1, 0), key = seed) word 0
 * is drawn on the device (SPEC S1). Requires 0 < P < 2^31, P % n_shard == 0, ld >= n_shard, and for several
 * shards q_stride >= n_shard, p_stride >= 2*ld + n_shard. Two launches (one workgroup, then one thread per slot). */
int vpf_estimate_resample(const int64_t* Q, int64_t q_stride, const float* particles, int64_t ld,
                          int64_t p_stride, int64_t n_shard, int64_t P, uint64_t seed, uint32_t frame,
                          int64_t slot_begin, int64_t slot_end, int32_t* anc_out, float* states_out,
                          int64_t out_ld, int64_t* cdf_ws, int64_t* stats_out, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* VPF_H */
