/*
 * mgp_hip.h -- C-ABI of the MI355X (gfx950) SMGP ELBO hot path.
 *
 * libmgp_hip.so replaces the TensorFlow C++ ops that GPflow 2.7 dispatches for
 * the sparse-variational mixture-of-GP-experts ELBO of LouieMiddle/ModulatedGPs
 * (MixtureGPs/models.py:69-79).  The reference has no native code or FFI of its
 * own: its operator boundary is the GPflow posterior plugin
 * IndependentPosteriorSingleOutputModified._conditional_fused
 * (MixtureGPs/models.py:129-144), the likelihood protocol
 * (MixtureGPs/likelihoods.py:31-32,39-41 via broadcasting_lik.py:39-46) and the
 * model hook SMGP._build_likelihood (models.py:69-79).  Each entry point below
 * names the reference call site it replaces.
 *
 * Conventions
 *  - float32 in HBM, row-major, leading dimensions in ELEMENTS.  Every leading
 *    dimension of a matrix whose rows are read as float4 must be a multiple of
 *    4 and every base pointer 16-byte aligned (MGP_ERR_ALIGN otherwise).
 *  - Hyper-parameters (kernel variance, lengthscales, likelihood variances) are
 *    DEVICE pointers, so a call never synchronises with the host and can be
 *    captured in a hipGraph.
 *  - The caller allocates every buffer, including workspaces sized by the
 *    *_workspace_bytes queries.  The library never allocates, frees or keeps
 *    pointers after returning.
 *  - Every call is asynchronous and ordered on `stream` (a hipStream_t; NULL =
 *    the legacy default stream) and acts on the current device.
 *  - Return value: MGP_OK (0); < 0: the (1-based) index of the first invalid
 *    argument, negated; > 0: an MGP_ERR_* code or MGP_ERR_HIP_BASE + hipError_t.
 */
#ifndef MGP_HIP_H
#define MGP_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef void* mgp_stream_t; /* hipStream_t */

enum {
  MGP_OK = 0,
  MGP_ERR_WORKSPACE = 1,   /* workspace pointer NULL or too small */
  MGP_ERR_ALIGN = 2,       /* leading dimension / pointer alignment */
  MGP_ERR_UNSUPPORTED = 3, /* size outside the supported range (e.g. D > 64, K > 32) */
  MGP_ERR_HIP_BASE = 1000
};

/* Library identity: "mgp_hip <version> gfx950". */
const char* mgp_version(void);
const char* mgp_status_string(int status);

/* ---------------------------------------------------------------- K1 / K2
 * RBF (SquaredExponential) cross-covariance
 *   Kuf[m, n] = var * exp(-0.5 * sum_d ((Z[m,d] - X[n,d]) / ls[d])^2)
 * Replaces Kmn = self.kernel.K(self.X_data.Z, Xnew) (models.py:139; GPflow
 * SquaredExponential.K -> square_distance + K_r2).  n_ls = 1 (isotropic) or D
 * (ARD).  X: [N, D] (ld ldx), Z: [M, D] (ld ldz), Kuf: [M, N] (ld ldk % 4 == 0). */
int mgp_rbf_kuf(const float* X, int64_t ldx, const float* Z, int64_t ldz, int64_t N, int64_t M,
                int32_t D, const float* variance, const float* lengthscales, int32_t n_ls,
                float* Kuf, int64_t ldk, mgp_stream_t stream);

/* Kuu[i, j] = K(Z, Z)[i, j] + jitter * (i == j).
 * Replaces covariances.Kuu(self.X_data, self.kernel, jitter=default_jitter())
 * (models.py:135).  Kuu: [M, M] (ld ldk % 4 == 0). */
int mgp_rbf_kuu(const float* Z, int64_t ldz, int64_t M, int32_t D, const float* variance,
                const float* lengthscales, int32_t n_ls, float jitter, float* Kuu, int64_t ldk,
                mgp_stream_t stream);

/* ---------------------------------------------------------------- K3
 * Batched blocked Cholesky with the triangular inverse fused in, computed in
 * float64 (the M x M work is M^3/3 flops; float32 would lose cond(L) * eps32 on
 * the badly conditioned Kuu of real inducing-point sets):
 *   L = chol(A) (lower, zeros above), LinvT = (L^-1)^T (upper, zeros below),
 * both rounded to float32.  Replaces Lm = tf.linalg.cholesky(Kmm) inside GPflow
 * base_conditional (models.py:141) and supplies L^-1 for its
 * triangular_solve.  `batch` matrices at element strides strideA / strideL
 * (the two SVGP layers of one ELBO share every launch).  info[b] = 0, or the
 * 1-based column of the first non-positive pivot (LAPACK potrf convention);
 * the factor then carries NaN.  L may be NULL.  lda, ldl % 4 == 0. */
size_t mgp_chol_workspace_bytes(int64_t M, int32_t batch);
int mgp_potrf_trtri(const float* A, int64_t lda, int64_t strideA, int64_t M, int32_t batch,
                    float* L, float* LinvT, int64_t ldl, int64_t strideL, int32_t* info,
                    void* workspace, size_t workspace_bytes, mgp_stream_t stream);

/* Same, with Kuu = var_b exp(-0.5 |(z_i - z_j)/l_b|^2) + jitter I built in
 * float64 from Z_b inside the factorisation (fuses K2 into K3; replaces
 * covariances.Kuu at models.py:135 for the ELBO path).  Z, variance,
 * lengthscales: HOST arrays of `batch` (<= 8) DEVICE pointers; n_ls: host
 * array (1 or D per entry).  Every Z_b is [M, D] with leading dimension ldz. */
int mgp_kuu_potrf_trtri(const float* const* Z, int64_t ldz, int64_t M, int32_t D,
                        const float* const* variance, const float* const* lengthscales,
                        const int32_t* n_ls, float jitter, int32_t batch, float* L,
                        float* LinvT, int64_t ldl, int64_t strideL, int32_t* info,
                        void* workspace, size_t workspace_bytes, mgp_stream_t stream);
/* Same; prep_done (a hipEvent_t, nullable) is recorded on the stream once Kuu
 * is built and its first diagonal tile factored, so a caller can start work
 * that is independent of the factorisation (K1, the q_sqrt images) on another
 * stream then rather than beside the build (which it would starve). */
int mgp_kuu_potrf_trtri_ev(const float* const* Z, int64_t ldz, int64_t M, int32_t D,
                           const float* const* variance, const float* const* lengthscales,
                           const int32_t* n_ls, float jitter, int32_t batch, float* L,
                           float* LinvT, int64_t ldl, int64_t strideL, int32_t* info,
                           void* workspace, size_t workspace_bytes, void* prep_done,
                           mgp_stream_t stream);
/* Same; linvt_absmax (nullable host array of `batch` device floats, each
 * nullable) receives max |(L^-1)^T| of that matrix, folded in while K3 writes
 * the inverse (zeroed by the launch itself) -- the scale bound of the L^-T
 * split-f16 image, so mgp_split_upper_f16_bounded needs no reduction pass
 * (pass mgp_x6_bound_ptr(Tfr, M, 0, 1) to write it straight into the image). */
int mgp_kuu_potrf_trtri_ex(const float* const* Z, int64_t ldz, int64_t M, int32_t D,
                           const float* const* variance, const float* const* lengthscales,
                           const int32_t* n_ls, float jitter, int32_t batch, float* L,
                           float* LinvT, int64_t ldl, int64_t strideL, int32_t* info,
                           void* workspace, size_t workspace_bytes, void* prep_done,
                           float* const* linvt_absmax, mgp_stream_t stream);
/* mgp_kuu_potrf_trtri_ex that also writes the Kuf image of every batch entry,
 * K(Z_b, X) (models.py:139, self.kernel.K(Z, Xnew), for pred_layer and assign_layer),
 * exactly as mgp_rbf_kuf_f16 (kfr_format 1) / mgp_rbf_kuf_x6 (kfr_format 0) write it
 * (bit-identical): the image blocks run on extra workgroups of the factorisation's
 * step launches, on the CUs the latency-bound chain leaves idle, instead of as
 * separate launches beside it.  X [N][ldx]; Kfr: host array of `batch` device
 * pointers, each at least mgp_x6_cols_bytes(M, N) bytes (kfr_bytes), 16-B aligned.
 * With M <= 64 (no step launches) the images are written by mgp_rbf_kuf_* launches
 * on the stream after the Kuu build.  -19 .. -24: X, ldx, N, Kfr, kfr_bytes,
 * kfr_format. */
int mgp_kuu_potrf_trtri_kuf(const float* const* Z, int64_t ldz, int64_t M, int32_t D,
                            const float* const* variance, const float* const* lengthscales,
                            const int32_t* n_ls, float jitter, int32_t batch, float* L,
                            float* LinvT, int64_t ldl, int64_t strideL, int32_t* info,
                            void* workspace, size_t workspace_bytes, void* prep_done,
                            float* const* linvt_absmax, const float* X, int64_t ldx, int64_t N,
                            void* const* Kfr, size_t kfr_bytes, int32_t kfr_format, mgp_stream_t stream);

/* ---------------------------------------------------------------- K4
 * Whitened projection A = L^-1 Kuf (as the triangular GEMM LinvT^T . Kuf) plus
 * per-row-tile column statistics for the conditional:
 *   stats[t][0][n]   = sum_{m in row tile t} A[m,n]^2
 *   stats[t][1+k][n] = sum_{m in row tile t} A[m,n] * q_mu[m,k]
 * Replaces A = tf.linalg.triangular_solve(Lm, Kmn), sum(square(A), -2) and
 * fmean = matmul(A, f, transpose_a=True) in GPflow base_conditional
 * (models.py:141-143).  q_mu: [M, K] (ld ldq).  stats: [T][K+1][lds] with
 * T = mgp_stats_tiles(M); lds % 4 == 0, lds >= N. */
int mgp_stats_tiles(int64_t M);
int mgp_trsm_stats(const float* LinvT, int64_t ldl, const float* Kuf, int64_t ldk, int64_t M,
                   int64_t N, const float* q_mu, int64_t ldq, int32_t K, float* A, int64_t lda,
                   float* stats, int64_t lds, mgp_stream_t stream);

/* ---------------------------------------------------------------- K5
 * K-expert whitened conditional, finalised:
 *   fmean[k][n] = sum_t stats[t][1+k][n]
 *   fvar[k][n]  = var - sum_t stats[t][0][n] + sum_{m'} (sum_{m>=m'} L_k[m,m'] A[m,n])^2
 * with L_k = band_part(q_sqrt[k], -1, 0) (the upper triangle is ignored).
 * Replaces the LTA = matmul(L, A_tiled, transpose_a=True) / reduce_sum(square)
 * tail of GPflow base_conditional (models.py:141-143; Knn = var from
 * models.py:133).  q_sqrt: [K][M][ldqs] at element stride strideq.
 * fmean, fvar: [K][ldf] (expert-major; ldf >= N).  Workspace (per-row-tile
 * partial sums): mgp_expert_workspace_bytes(M, N, K).  (Exact-f32 MFMA products;
 * the default-format entry of this operation is mgp_expert_conditional, below.) */
size_t mgp_expert_workspace_bytes(int64_t M, int64_t N, int32_t K);
int mgp_expert_conditional_f32(const float* A, int64_t lda, const float* q_sqrt, int64_t ldqs,
                               int64_t strideq, const float* stats, int64_t lds,
                               const float* variance, int64_t M, int64_t N, int32_t K, float* fmean,
                               float* fvar, int64_t ldf, void* workspace, size_t workspace_bytes,
                               mgp_stream_t stream);

/* ---------------------------------------------------------------- K5, split-bf16
 * The same K-expert conditional on the bf16 matrix cores at f32 accuracy:
 * every f32 operand is split exactly into three bf16 planes and each product
 * is formed from the six plane products of weight >= 2^-16 (f32-accumulated;
 * see csrc/split3.hip).  Operands are passed as "fragment images":
 *   mgp_split_lower_x6: L_k = band_part(q_sqrt[k], -1, 0) -> Lfr
 *       (mgp_x6_lower_bytes(M, K) bytes; replaces the band_part at
 *       models.py:141-143 and is rebuilt whenever q_sqrt changes);
 *   mgp_split_cols_x6:  A [M][lda] -> Afr (mgp_x6_cols_bytes(M, N) bytes);
 *       on the ELBO path K4 (mgp_trsm_stats_x6) writes Afr directly.
 * mgp_expert_conditional_x6 then produces fmean/fvar exactly as
 * mgp_expert_conditional_f32.  Images must be < 4 GiB.  Workspace:
 * mgp_expert_x6_workspace_bytes(M, N, K). */
size_t mgp_x6_lower_bytes(int64_t M, int32_t K);    /* also the LinvT image: K = 1 */
size_t mgp_x6_cols_bytes(int64_t M, int64_t N);
int mgp_split_lower_x6(const float* q_sqrt, int64_t ldqs, int64_t strideq, int64_t M, int32_t K,
                       void* Lfr, size_t lfr_bytes, mgp_stream_t stream);
int mgp_split_cols_x6(const float* A, int64_t lda, int64_t M, int64_t N, void* Afr, size_t afr_bytes,
                      mgp_stream_t stream);
/* Image of LinvT (upper triangle kept) as K4's T operand. */
int mgp_split_upper_x6(const float* LinvT, int64_t ldl, int64_t M, void* Tfr, size_t tfr_bytes,
                       mgp_stream_t stream);
/* K1 writing the image of Kuf directly (same arguments as mgp_rbf_kuf; the
 * f32 Kuf is not materialised). */
int mgp_rbf_kuf_x6(const float* X, int64_t ldx, const float* Z, int64_t ldz, int64_t N, int64_t M,
                   int32_t D, const float* variance, const float* lengthscales, int32_t n_ls,
                   void* Kfr, size_t kfr_bytes, mgp_stream_t stream);
/* K4 on images: A = LinvT^T Kuf from Tfr (mgp_split_upper_x6) and Kfr
 * (mgp_rbf_kuf_x6 / mgp_split_cols_x6), writing A's image Afr (for
 * mgp_expert_conditional_x6) and the stats exactly as mgp_trsm_stats; also
 * the f32 A [M][lda] when A is not NULL (kept for the backward pass). */
int mgp_trsm_stats_x6(const void* Tfr, size_t tfr_bytes, const void* Kfr, size_t kfr_bytes, int64_t M,
                      int64_t N, const float* q_mu, int64_t ldq, int32_t K, void* Afr, size_t afr_bytes,
                      float* stats, int64_t lds, float* A, int64_t lda, mgp_stream_t stream);
size_t mgp_expert_x6_workspace_bytes(int64_t M, int64_t N, int32_t K);
int mgp_expert_conditional_x6(const void* Afr, size_t afr_bytes, const void* Lfr, size_t lfr_bytes,
                              const float* stats, int64_t lds, const float* variance, int64_t M,
                              int64_t N, int32_t K, float* fmean, float* fvar, int64_t ldf,
                              void* workspace, size_t workspace_bytes, mgp_stream_t stream);
/* K5 from the same images using only the leading `planes` bf16 planes of each
 * operand (BASELINE config 5, "bf16 mixed"; K1-K4 stay x6):
 *   planes = 3: identical to mgp_expert_conditional_x6 (six products, f32-accurate);
 *   planes = 2: three products (hi.hi + hi.mid + mid.hi), ~16-bit operands;
 *   planes = 1: one product (bf16 operands, f32 accumulation).
 * Replaces the same call site (GPflow base_conditional, models.py:141-143). */
int mgp_expert_conditional_planes(const void* Afr, size_t afr_bytes, const void* Lfr, size_t lfr_bytes,
                                  const float* stats, int64_t lds, const float* variance, int64_t M,
                                  int64_t N, int32_t K, int32_t planes, float* fmean, float* fvar,
                                  int64_t ldf, void* workspace, size_t workspace_bytes, mgp_stream_t stream);

/* ---------------------------------------------------------------- K5, split-f16 ("f16x3")
 * The same conditional from split-f16 images: each operand, scaled by a power
 * of two 2^e that puts its largest magnitude in [2^13, 2^14), is split into
 * fp16 hi + lo (22 significant bits) and a product is the three f16 MFMA plane
 * products hi.hi + hi.lo + lo.hi (dropped lo.lo <= 2^-22 of it), f32-accumulated:
 * half the matrix-core work of x6 at an operand error of 2^-22 (x6: 2^-24,
 * the f32 input rounding itself).  Same buffer sizes as the x6 images; the
 * image trailer (after the planes) carries the bound from which e is derived.
 *   mgp_split_lower_f16:   q_sqrt -> Lfr (bound = max |tril(q_sqrt)|, computed on device);
 *   mgp_split_cols_f16:    A -> Afr (bound = max |A|);
 *   mgp_trsm_stats_x6_f16: K4 as mgp_trsm_stats_x6 (x6 inputs) writing A's
 *       split-f16 image, bound sqrt(variance) (|A[m][n]| <= sqrt(k(x_n, x_n)));
 *   mgp_expert_conditional_f16: K5 on the two split-f16 images, outputs and
 *       workspace as mgp_expert_conditional_x6.
 * The whole forward chain in split-f16 (K1 -> K4 -> K5, three f16 products per
 * block in K4 as well):
 *   mgp_rbf_kuf_f16:     K1 writing Kuf's split-f16 image (bound = variance,
 *       Kuf <= variance; replaces kernel.K(Z, Xnew), models.py:139);
 *   mgp_split_upper_f16: LinvT (upper triangle) -> Tfr (bound = its max |.|);
 *   mgp_trsm_stats_f16:  K4 as mgp_trsm_stats_x6_f16 on split-f16 Tfr / Kfr
 *       (the triangular solve of base_conditional, models.py:141-143); also
 *       the f32 A [M][lda] when A is not NULL (training);
 *   mgp_conditional_backward_f16: mgp_conditional_backward_x6 with Afr =
 *       A's split-f16 image (mgp_trsm_stats_f16); S_k A runs on f16 products.
 * Replaces the same call sites (GPflow base_conditional, models.py:141-143). */
int mgp_rbf_kuf_f16(const float* X, int64_t ldx, const float* Z, int64_t ldz, int64_t N, int64_t M,
                    int32_t D, const float* variance, const float* lengthscales, int32_t n_ls,
                    void* Kfr, size_t kfr_bytes, mgp_stream_t stream);
int mgp_split_upper_f16(const float* LinvT, int64_t ldl, int64_t M, void* Tfr, size_t tfr_bytes,
                        mgp_stream_t stream);
/* mgp_split_upper_f16 whose image trailer already holds max |LinvT| (from
 * mgp_kuu_potrf_trtri_ex): the split alone, no reduction launches. */
int mgp_split_upper_f16_bounded(const float* LinvT, int64_t ldl, int64_t M, void* Tfr, size_t tfr_bytes,
                                mgp_stream_t stream);
/* mgp_split_upper_f16_bounded for batch (1 or 2) matrices at LinvT + b * strideL
 * (both layers' L^-T from one mgp_kuu_potrf_trtri_ex call) into the images Tfr[b]
 * (host array of device pointers) in one launch; bit-identical to one call each.
 * Replaces the operand preparation of triangular_solve(Lm, Kmn) in
 * base_conditional (models.py:141) for both layers.  -9: batch outside [1, 2]. */
int mgp_split_upper_f16_bounded_batch(int32_t batch, const float* LinvT, int64_t ldl, int64_t strideL, int64_t M,
                                      void* const* Tfr, size_t tfr_bytes, mgp_stream_t stream);
/* Device address of the split-f16 scale bound in an image's trailer: lower /
 * upper triangular images of K matrices (K >= 1), or a column image (K = 0,
 * N columns).  NULL for a NULL image or M <= 0. */
float* mgp_x6_bound_ptr(void* img, int64_t M, int64_t N, int32_t K);
int mgp_trsm_stats_f16(const void* Tfr, size_t tfr_bytes, const void* Kfr, size_t kfr_bytes, int64_t M,
                       int64_t N, const float* q_mu, int64_t ldq, int32_t K, const float* variance,
                       void* Afr, size_t afr_bytes, float* stats, int64_t lds, float* A, int64_t lda,
                       mgp_stream_t stream);
/* mgp_trsm_stats_f16 for batch (1 or 2) layers of equal M, N, K in one launch: the
 * two SMGP layers' triangular solves (models.py:141-143 for pred_layer and
 * assign_layer, one call instead of two).  Tfr, Kfr, q_mu, variance, Afr, stats
 * (and A, if not NULL; A[b] may be NULL) are host arrays of `batch` device
 * pointers; sizes and leading dimensions are shared.  Bit-identical to one
 * mgp_trsm_stats_f16 call per layer.  -17: batch outside [1, 2]. */
int mgp_trsm_stats_f16_batch(int32_t batch, const void* const* Tfr, size_t tfr_bytes, const void* const* Kfr,
                             size_t kfr_bytes, int64_t M, int64_t N, const float* const* q_mu, int64_t ldq,
                             int32_t K, const float* const* variance, void* const* Afr, size_t afr_bytes,
                             float* const* stats, int64_t lds, float* const* A, int64_t lda,
                             mgp_stream_t stream);
/* mgp_expert_conditional_f16 (Cfr == NULL) or mgp_expert_conditional_f16c (Cfr and
 * colmax given) for batch (1 or 2) layers of equal M, N, K: one K5 launch over both
 * layers' items (models.py:141-143's LTA and fvar for pred_layer and assign_layer),
 * then each layer's finalize.  Afr, Lfr, stats, variance, fmean, fvar, workspace (one
 * per layer, mgp_expert_x6_workspace_bytes each), Cfr, colmax are host arrays of
 * `batch` device pointers.  Bit-identical to one call per layer.  -20: batch outside
 * [1, 2]. */
int mgp_expert_conditional_f16_batch(int32_t batch, const void* const* Afr, size_t afr_bytes,
                                     const void* const* Lfr, size_t lfr_bytes, const float* const* stats,
                                     int64_t lds, const float* const* variance, int64_t M, int64_t N, int32_t K,
                                     float* const* fmean, float* const* fvar, int64_t ldf, void* const* workspace,
                                     size_t workspace_bytes, void* const* Cfr, size_t cfr_bytes,
                                     const float* const* colmax, mgp_stream_t stream);
/* mgp_trsm_stats_f16 that also writes plane 2 of A's image (e4m3 cross terms,
 * the operand of mgp_expert_conditional_f16x8).  With A == NULL plane 1 (f16 lo)
 * is not written: the image then feeds mgp_expert_conditional_f16x8 only. */
int mgp_trsm_stats_f16x8(const void* Tfr, size_t tfr_bytes, const void* Kfr, size_t kfr_bytes, int64_t M,
                         int64_t N, const float* q_mu, int64_t ldq, int32_t K, const float* variance,
                         void* Afr, size_t afr_bytes, float* stats, int64_t lds, float* A, int64_t lda,
                         mgp_stream_t stream);
int mgp_split_lower_f16(const float* q_sqrt, int64_t ldqs, int64_t strideq, int64_t M, int32_t K,
                        void* Lfr, size_t lfr_bytes, mgp_stream_t stream);
/* Both SMGP layers' tril(q_sqrt) work in three launches: the split-f16 image of
 * tril(q_sqrt) into Lfr[b] (bit-identical to mgp_split_lower_f16) and the whitened KL
 * (models.py:79, prior_kl) into kl_out[b] (bit-identical to mgp_gauss_kl_white) for
 * b < batch (1 or 2), replacing the five per-layer launches of those two calls (the KL
 * partial sums also fold the image's scale bound).  q_mu [M][ldq >= K], q_sqrt
 * [K][M][ldqs] (stride strideq; ldqs and strideq multiples of 4, 16-B aligned; shared
 * by the layers), Lfr at least mgp_x6_lower_bytes(M, K) bytes (lfr_bytes, 16-B aligned),
 * workspace at least batch * mgp_qsqrt_workspace_bytes(M, K) bytes (16-B aligned).
 * -1 .. -11: batch, q_mu, ldq, q_sqrt, ldqs, strideq, M, K, Lfr, lfr_bytes, kl_out. */
size_t mgp_qsqrt_workspace_bytes(int64_t M, int32_t K);
int mgp_qsqrt_images_kl_f16_batch(int32_t batch, const float* const* q_mu, int64_t ldq,
                                  const float* const* q_sqrt, int64_t ldqs, int64_t strideq, int64_t M,
                                  int32_t K, void* const* Lfr, size_t lfr_bytes, double* const* kl_out,
                                  void* workspace, size_t workspace_bytes, mgp_stream_t stream);
int mgp_split_cols_f16(const float* A, int64_t lda, int64_t M, int64_t N, void* Afr, size_t afr_bytes,
                       mgp_stream_t stream);
int mgp_trsm_stats_x6_f16(const void* Tfr, size_t tfr_bytes, const void* Kfr, size_t kfr_bytes, int64_t M,
                          int64_t N, const float* q_mu, int64_t ldq, int32_t K, const float* variance,
                          void* Afr, size_t afr_bytes, float* stats, int64_t lds, mgp_stream_t stream);
int mgp_expert_conditional_f16(const void* Afr, size_t afr_bytes, const void* Lfr, size_t lfr_bytes,
                               const float* stats, int64_t lds, const float* variance, int64_t M,
                               int64_t N, int32_t K, float* fmean, float* fvar, int64_t ldf,
                               void* workspace, size_t workspace_bytes, mgp_stream_t stream);
/* K5 "f16x8": split-f16 images that also carry plane 2 = e4m3(hi 2^-6) |
 * e4m3(lo 2^6) of each fragment (mgp_split_lower_f16, mgp_split_cols_f16 and
 * mgp_trsm_stats_f16x8 write it); the hi products on
 * the f16 MFMA, both cross terms of two k-steps on one e4m3 MFMA
 * (v_mfma_scale_f32_32x32x64_f8f6f4, unit scales): 4 f16-product-equivalents
 * per k-step pair instead of 6.  Cross terms are <= 2^-11 of the leading one,
 * so e4m3's 3-bit mantissas cost ~2^-15 relative per product. */
int mgp_expert_conditional_f16x8(const void* Afr, size_t afr_bytes, const void* Lfr, size_t lfr_bytes,
                                 const float* stats, int64_t lds, const float* variance, int64_t M,
                                 int64_t N, int32_t K, float* fmean, float* fvar, int64_t ldf,
                                 void* workspace, size_t workspace_bytes, mgp_stream_t stream);
/* Training forward (split-f16): mgp_expert_conditional_f16 that also writes
 * C_k = L_k^T A of every expert as a split-f16 B-layout image (Cfr, at least
 * mgp_c_images_bytes(M, N, K) bytes), for mgp_conditional_backward_f16c.  colmax:
 * DEVICE max column 2-norm of tril(q_sqrt) (mgp_colnorm_max); the images are
 * scaled by the bound colmax * sqrt(variance) >= |C|. */
size_t mgp_c_images_bytes(int64_t M, int64_t N, int32_t K);
int mgp_colnorm_max(const float* q_sqrt, int64_t ldq, int64_t strideq, int64_t M, int32_t K, float* out,
                    mgp_stream_t stream);
int mgp_expert_conditional_f16c(const void* Afr, size_t afr_bytes, const void* Lfr, size_t lfr_bytes,
                                const float* stats, int64_t lds, const float* variance, int64_t M,
                                int64_t N, int32_t K, float* fmean, float* fvar, int64_t ldf,
                                void* workspace, size_t workspace_bytes, void* Cfr, size_t cfr_bytes,
                                const float* colmax, mgp_stream_t stream);

/* ---------------------------------------------------------------- backward of K1-K5
 * Gram products over the data dimension (float32 MFMA, deterministic split-K):
 *   out[i][j] = alpha * sum_n X[i][n] Y[j][n]   (tri != 0: j <= i only, zeros above)
 * X [MI][ldx], Y [MJ][ldy]; workspace mgp_gram_workspace_bytes(MI, MJ, N, tri). */
size_t mgp_gram_workspace_bytes(int64_t MI, int64_t MJ, int64_t N, int32_t tri);
int mgp_gram(const float* X, int64_t ldx, int64_t MI, const float* Y, int64_t ldy, int64_t MJ, int64_t N,
             float alpha, int32_t tri, float* out, int64_t ldo, void* workspace, size_t workspace_bytes,
             mgp_stream_t stream);

/* The same contraction at f32 accuracy on the bf16 MFMA (operands split into
 * three bf16 planes on the fly, six plane products), batched and weighted:
 *   out[b][i][j] = alpha * sum_n X_b[i][n] w_b[n] Y_b[j][n]
 * X_b = X + b sx ([MI][ldx]), Y_b = Y + b sy, w_b = W + b sw (W may be NULL:
 * no weight), out_b = out + b so; mode 0 full, 1 lower triangle (zeros above),
 * 2 symmetric (upper mirrors lower).  ldx, ldy, strides multiples of 4 floats,
 * pointers 16-B aligned.  Workspace mgp_gram_x6_workspace_bytes. */
size_t mgp_gram_x6_workspace_bytes(int64_t MI, int64_t MJ, int64_t N, int32_t batch, int32_t mode);
int mgp_gram_x6(const float* X, int64_t ldx, int64_t sx, int64_t MI, const float* Y, int64_t ldy, int64_t sy,
                int64_t MJ, const float* W, int64_t sw, int64_t N, int32_t batch, float alpha, int32_t mode,
                float* out, int64_t ldo, int64_t so, void* workspace, size_t workspace_bytes, mgp_stream_t stream);
/* Same contraction on the f16 matrix cores: the chunks are split on the fly
 * into power-of-two-scaled fp16 hi / lo planes (three products per fragment
 * pair, 22-bit operands).  x_bound, y_bound, w_bound: DEVICE pointers to
 * bounds of |X|, |Y| and |W| (w_bound only when W != NULL).  Workspace as
 * mgp_gram_x6.  Used by mgp_conditional_backward_f16. */
int mgp_gram_f16(const float* X, int64_t ldx, int64_t sx, int64_t MI, const float* Y, int64_t ldy,
                 int64_t sy, int64_t MJ, const float* W, int64_t sw, int64_t N, int32_t batch, float alpha,
                 int32_t mode, float* out, int64_t ldo, int64_t so, const float* x_bound,
                 const float* y_bound, const float* w_bound, void* workspace, size_t workspace_bytes,
                 mgp_stream_t stream);
/* Row image of X (M x N f32, ldx % 4 == 0) for mgp_gram_f16_rows: fp16 hi / lo
 * planes of X 2^e (e from the DEVICE bound *bound, as mgp_gram_f16 scales X) in
 * the gram's fragment order, [32-row block][16-column k-step] blocks of 2 KiB,
 * zero beyond M and N; mgp_rows_f16_ksteps(N) k-steps per row block. */
int64_t mgp_rows_f16_ksteps(int64_t N);
size_t mgp_rows_f16_bytes(int64_t M, int64_t N);
int mgp_split_rows_f16(const float* X, int64_t ldx, int64_t M, int64_t N, const float* bound, void* img,
                       size_t img_bytes, mgp_stream_t stream);
/* mgp_gram_f16 (weighted: W required; X and the f32 Y 2-D, shared by the batch)
 * with X given as its row image (mgp_split_rows_f16 of X with bound x_bound): X
 * is split once instead of once per tile and batch entry, and one workgroup
 * serves two batch entries.  Bit-identical to mgp_gram_f16.  The P_k =
 * A diag(Gv_k) A^T grams of mgp_conditional_backward_f16 / _f16x8 run here. */
int mgp_gram_f16_rows(const void* ximg, size_t ximg_bytes, int64_t MI, const float* Y, int64_t ldy, int64_t MJ,
                      const float* W, int64_t sw, int64_t N, int32_t batch, float alpha, int32_t mode, float* out,
                      int64_t ldo, int64_t so, const float* x_bound, const float* y_bound, const float* w_bound,
                      void* workspace, size_t workspace_bytes, mgp_stream_t stream);

/* Backward of one layer's whitened conditional (the GradientTape pass through
 * GPflow base_conditional, models.py:141-143, and SVGP's Knn = var,
 * models.py:133), given G_mu = d/d fmean and G_v = d/d fvar ([K][ldg]):
 *   g_q_mu [M][ldgq]       = A G_mu^T
 *   g_q_sqrt[k] [M][ldgs]  = 2 tril(A diag(G_v,k) (L_k^T A)^T)
 *   g_Kuf [M][ldk]         = L^-T gA,  gA = q_mu G_mu - 2 A sum_k G_v,k + 2 sum_k L_k (L_k^T A) diag(G_v,k)
 *   g_Lm [M][ldgl]         = -tril(g_Kuf A^T)          (gradient w.r.t. chol(Kuu))
 *   g_var (double)         = sum G_v                   (through Knn)
 * Inputs: A's split image and f32 A (both from mgp_trsm_stats_x6), q_sqrt
 * (its lower triangle is used), q_mu, LinvT.  The expert terms use
 * S_k = L_k L_k^T (sum_k L_k (L_k^T A) diag(G_v,k) = sum_k (S_k A) diag(G_v,k))
 * and P_k = A diag(G_v,k) A^T (g_q_sqrt[k] = 2 tril(P_k L_k)).  Every product
 * that scales with N runs on the split-bf16 x6 path (f32 accuracy), g_q_mu on
 * the f32 MFMA.  Workspace: mgp_conditional_backward_workspace_bytes. */
size_t mgp_conditional_backward_workspace_bytes(int64_t M, int64_t N, int32_t K);
int mgp_conditional_backward_x6(const void* Afr, size_t afr_bytes, const float* A, int64_t lda,
                                const float* q_sqrt, int64_t ldqs,
                                int64_t strideq, const float* q_mu, int64_t ldq, const float* LinvT,
                                int64_t ldl, const float* Gmu, const float* Gv, int64_t ldg, int64_t M,
                                int64_t N, int32_t K, float* g_q_mu, int64_t ldgq, float* g_q_sqrt,
                                int64_t ldgs, int64_t strideg, float* g_Kuf, int64_t ldk, float* g_Lm,
                                int64_t ldgl, double* g_var, void* workspace, size_t workspace_bytes,
                                mgp_stream_t stream);
/* Same, with Afr = A's split-f16 image (mgp_trsm_stats_f16): S_k = L_k L_k^T is
 * split the same way (bound = max |S_k| on device) and S_k A runs on three f16
 * products per block. */
int mgp_conditional_backward_f16(const void* Afr, size_t afr_bytes, const float* A, int64_t lda,
                                 const float* q_sqrt, int64_t ldqs,
                                 int64_t strideq, const float* q_mu, int64_t ldq, const float* LinvT,
                                 int64_t ldl, const float* Gmu, const float* Gv, int64_t ldg, int64_t M,
                                 int64_t N, int32_t K, float* g_q_mu, int64_t ldgq, float* g_q_sqrt,
                                 int64_t ldgs, int64_t strideg, float* g_Kuf, int64_t ldk, float* g_Lm,
                                 int64_t ldgl, double* g_var, void* workspace, size_t workspace_bytes,
                                 mgp_stream_t stream);
/* Same, with Afr from mgp_trsm_stats_f16x8 (A non-NULL: all three planes): S_k A on
 * f16 hi products + e4m3 cross terms (the f16x8 training step). */
int mgp_conditional_backward_f16x8(const void* Afr, size_t afr_bytes, const float* A, int64_t lda,
                                 const float* q_sqrt, int64_t ldqs,
                                 int64_t strideq, const float* q_mu, int64_t ldq, const float* LinvT,
                                 int64_t ldl, const float* Gmu, const float* Gv, int64_t ldg, int64_t M,
                                 int64_t N, int32_t K, float* g_q_mu, int64_t ldgq, float* g_q_sqrt,
                                 int64_t ldgs, int64_t strideg, float* g_Kuf, int64_t ldk, float* g_Lm,
                                 int64_t ldgl, double* g_var, void* workspace, size_t workspace_bytes,
                                 mgp_stream_t stream);
/* mgp_conditional_backward_f16 with the forward's C_k images (mgp_expert_conditional_f16c
 * on the same Afr, q_sqrt and colmax; l_bound = DEVICE bound of that call's Lfr
 * image): the q_sqrt-weighted part of gA as 2 sum_k L_k C_k diag(Gv_k) on the
 * triangular L_k -- half the products of the S_k = L_k L_k^T form, and no S_k. */
int mgp_conditional_backward_f16c(const void* Afr, size_t afr_bytes, const float* A, int64_t lda,
                                  const float* q_sqrt, int64_t ldqs, int64_t strideq, const float* q_mu, int64_t ldq,
                                  const float* LinvT, int64_t ldl, const float* Gmu, const float* Gv, int64_t ldg,
                                  int64_t M, int64_t N, int32_t K, float* g_q_mu, int64_t ldgq, float* g_q_sqrt,
                                  int64_t ldgs, int64_t strideg, float* g_Kuf, int64_t ldk, float* g_Lm,
                                  int64_t ldgl, double* g_var, void* workspace, size_t workspace_bytes,
                                  const void* Cfr, size_t cfr_bytes, const float* colmax, const float* l_bound,
                                  mgp_stream_t stream);
/* The q_sqrt-only part of mgp_conditional_backward_f16c -- L_k's image (scale l_bound)
 * and the transposed triangles L_k^T -- into prep (mgp_conditional_backward_prep_bytes),
 * e.g. on a side stream while the forward runs, and the backward on it (two launches
 * fewer on its stream, the same results).  t_bound (may be NULL): max |LinvT| as K3's
 * bounded L^-T images carry it (their trailer), so the backward needs no reduction of
 * its own for Linv's split-f16 image.  Prep: -1 .. -7 q_sqrt, ldqs, strideq, M, K,
 * l_bound, prep; prepped: as _f16c, plus -33 prep NULL, -34 prep_bytes. */
size_t mgp_conditional_backward_prep_bytes(int64_t M, int32_t K);
int mgp_conditional_backward_prep_f16c(const float* q_sqrt, int64_t ldqs, int64_t strideq, int64_t M, int32_t K,
                                       const float* l_bound, void* prep, size_t prep_bytes, mgp_stream_t stream);
int mgp_conditional_backward_f16c_prepped(const void* Afr, size_t afr_bytes, const float* A, int64_t lda,
                                          const float* q_sqrt, int64_t ldqs, int64_t strideq, const float* q_mu,
                                          int64_t ldq, const float* LinvT, int64_t ldl, const float* Gmu,
                                          const float* Gv, int64_t ldg, int64_t M, int64_t N, int32_t K,
                                          float* g_q_mu, int64_t ldgq, float* g_q_sqrt, int64_t ldgs,
                                          int64_t strideg, float* g_Kuf, int64_t ldk, float* g_Lm, int64_t ldgl,
                                          double* g_var, void* workspace, size_t workspace_bytes, const void* Cfr,
                                          size_t cfr_bytes, const float* colmax, const float* l_bound,
                                          const void* prep, size_t prep_bytes, const float* t_bound,
                                          mgp_stream_t stream);

/* Reverse mode of Lm = chol(Kuu) (models.py:141): gKuu = sym(Lm^-T Phi(Lm^T gL) Lm^-1),
 * Phi = lower triangle with halved diagonal, in float64 from the float32 L,
 * LinvT = (Lm^-1)^T (both from mgp_potrf_trtri / mgp_kuu_potrf_trtri) and gL
 * (lower).  Output gKuu [M][ldo] float32, symmetric.
 * Workspace: mgp_chol_backward_workspace_bytes(M). */
size_t mgp_chol_backward_workspace_bytes(int64_t M);
int mgp_chol_backward(const float* L, int64_t ldl, const float* LinvT, int64_t ldli, const float* gL,
                      int64_t ldg, int64_t M, float* gKuu, int64_t ldo, void* workspace,
                      size_t workspace_bytes, mgp_stream_t stream);
/* mgp_chol_backward for both SMGP layers (batch 1 .. 8 layers of one M, shared
 * leading dimensions) in five launches instead of eight per layer; bit-identical to
 * batch calls of mgp_chol_backward.  Workspace: batch * mgp_chol_backward_workspace_bytes(M).
 * -1 .. -10: batch, L, ldl, LinvT, ldli, gL, ldg, M, gKuu, ldo. */
int mgp_chol_backward_batch(int32_t batch, const float* const* L, int64_t ldl, const float* const* LinvT,
                            int64_t ldli, const float* const* gL, int64_t ldg, int64_t M, float* const* gKuu,
                            int64_t ldo, void* workspace, size_t workspace_bytes, mgp_stream_t stream);

/* Reverse mode of K(Z, X) (models.py:135,139) for a cotangent gK [M][ldg]:
 * gZ [M][ldgz] (float), g_var and g_ls[n_ls] (double, device).  symmetric = 1
 * for Kuu (X = Z, symmetric gK: Z enters both arguments).  accumulate = 1 adds
 * to the outputs (to combine the Kuf and Kuu contributions).
 * Workspace: mgp_rbf_backward_workspace_bytes(N, M, D). */
size_t mgp_rbf_backward_workspace_bytes(int64_t N, int64_t M, int32_t D);
int mgp_rbf_backward(const float* X, int64_t ldx, const float* Z, int64_t ldz, int64_t N, int64_t M,
                     int32_t D, const float* variance, const float* lengthscales, int32_t n_ls,
                     const float* gK, int64_t ldg, int32_t symmetric, int32_t accumulate, float* gZ,
                     int64_t ldgz, double* g_var, double* g_ls, void* workspace, size_t workspace_bytes,
                     mgp_stream_t stream);
/* Both kernel cotangents of up to 8 layers (models.py:135,139; the layers share X,
 * M, D, n_ls and the leading dimensions) in three launches instead of five per layer:
 * per layer b the Kuf contribution (gKuf[b] [M][ldgf], over X [N][ldx]) and then the
 * Kuu one (gKuu[b] [M][ldgu], symmetric) added to it -- bit-identical to
 * mgp_rbf_backward(Kuf, accumulate) followed by mgp_rbf_backward(Kuu, symmetric = 1,
 * accumulate = 1).  accumulate: 0 the Kuf contribution overwrites gZ, g_var and g_ls,
 * 1 it adds to them, 2 it overwrites gZ and g_ls and adds to g_var (the training
 * step: g_var carries the conditional's part; no zero fills of gZ / g_ls needed).
 * Workspace: batch * mgp_rbf_backward_batch_workspace_bytes(N, M, D).
 * -1 .. -20: batch, X, ldx, N, Z, ldz, M, D, variance, lengthscales, n_ls, gKuf, ldgf,
 * gKuu, ldgu, gZ, ldgz, g_var, g_ls, accumulate. */
size_t mgp_rbf_backward_batch_workspace_bytes(int64_t N, int64_t M, int32_t D);
int mgp_rbf_backward_batch(int32_t batch, const float* X, int64_t ldx, int64_t N, const float* const* Z,
                           int64_t ldz, int64_t M, int32_t D, const float* const* variance,
                           const float* const* lengthscales, int32_t n_ls, const float* const* gKuf,
                           int64_t ldgf, const float* const* gKuu, int64_t ldgu, int32_t accumulate,
                           float* const* gZ, int64_t ldgz, double* const* g_var, double* const* g_ls,
                           void* workspace, size_t workspace_bytes, mgp_stream_t stream);

/* ---------------------------------------------------------------- K7
 * Whitened Gaussian KL (GPflow gauss_kl(q_mu, q_sqrt, K=None), reached through
 * SVGP.prior_kl at models.py:79):
 *   kl = 0.5 * (sum q_mu^2 - M*K - sum_k sum_m log(L_k[m,m]^2) + sum_k ||tril L_k||_F^2)
 * Written as one double to kl_out (device).  Workspace: mgp_kl_workspace_bytes. */
size_t mgp_kl_workspace_bytes(int64_t M, int32_t K);
int mgp_gauss_kl_white(const float* q_mu, int64_t ldq, const float* q_sqrt, int64_t ldqs,
                       int64_t strideq, int64_t M, int32_t K, double* kl_out, void* workspace,
                       size_t workspace_bytes, mgp_stream_t stream);

/* ---------------------------------------------------------------- K6
 * Monte-Carlo data term of the SMGP ELBO for the local data points:
 *   data_sum = sum_n [ logsumexp_s( sum_k W[s,n,k] ve[n,k] ) - log S ]
 *   logits = mu_a + z * sqrt(var_a + jitter)            (models.py:57-58, utils.py:26-27;
 *            jitter = gpflow.config.default_jitter(), 1e-6 unless set)
 *   W = softmax_k((-log(-log u) + logits) / tau)         (models.py:59-60,73-74; TFP 0.18)
 *   ve = -0.5 log 2pi - 0.5 log s2_k - 0.5((y - mu_f)^2 + var_f)/s2_k  (likelihoods.py:39-41)
 * Replaces SMGP.W_dist / E_log_p_Y / the batch sum of models.py:55-76.
 * mu_*, var_*: [K][ldf]; Y: [N]; lik_var: [K] (device).  Noise: explicit
 * noise_z / noise_u [S][N][K] when both non-NULL (parity mode), else in-kernel
 * Philox4x32-10 keyed by (seed, global n = n_offset + n, s, k).  data_sum: one
 * double (device).  Workspace: mgp_elbo_workspace_bytes(N). */
size_t mgp_elbo_workspace_bytes(int64_t N);
int mgp_elbo_terms(const float* mu_f, const float* var_f, const float* mu_a, const float* var_a,
                   int64_t ldf, const float* Y, const float* lik_var, int64_t N, int32_t K,
                   int32_t S, float tau, float jitter, const float* noise_z, const float* noise_u,
                   uint64_t seed, int64_t n_offset, double* data_sum, void* workspace,
                   size_t workspace_bytes, mgp_stream_t stream);

/* SMGPModified.E_log_p_Y (models.py:106-123): as mgp_elbo_terms, plus the
 * assignment layer's own Gaussian var-exp (likelihood variances
 * assign_lik_var [K], device) weighted by the same W, with its own logsumexp:
 *   data_sum = sum_n [lse_s(sum_k W ve_a) - log S + lse_s(sum_k W ve_f) - log S]. */
int mgp_elbo_terms_modified(const float* mu_f, const float* var_f, const float* mu_a,
                            const float* var_a, int64_t ldf, const float* Y, const float* lik_var,
                            const float* assign_lik_var, int64_t N, int32_t K, int32_t S, float tau, float jitter,
                            const float* noise_z, const float* noise_u, uint64_t seed,
                            int64_t n_offset, double* data_sum, void* workspace,
                            size_t workspace_bytes, mgp_stream_t stream);

/* ---------------------------------------------------------------- K6 backward
 * Gradient of the data term (of mgp_elbo_terms, or of mgp_elbo_terms_modified
 * when assign_lik_var is not NULL) with respect to the conditionals and the
 * likelihood variances, for the same noise (explicit or Philox seed/n_offset):
 *   G [4][K][ldg] (float, device) = scale * d(sum_n DT_n)/d(mu_f, var_f, mu_a, var_a)
 *   g_lik_var[K], g_assign_lik_var[K] (double, device) = scale * d(sum_n DT_n)/d(sigma^2)
 * (scale = 1 / N_total gives the ELBO's batch-mean gradient).  Replaces the
 * GradientTape pass through models.py:55-67,73-76 and likelihoods.py:39-41.
 * Workspace: mgp_elbo_backward_workspace_bytes(N, K). */
size_t mgp_elbo_backward_workspace_bytes(int64_t N, int32_t K);
int mgp_elbo_terms_backward(const float* mu_f, const float* var_f, const float* mu_a,
                            const float* var_a, int64_t ldf, const float* Y, const float* lik_var,
                            const float* assign_lik_var, int64_t N, int32_t K, int32_t S, float tau, float jitter,
                            const float* noise_z, const float* noise_u, uint64_t seed,
                            int64_t n_offset, float scale, float* G, int64_t ldg, double* g_lik_var,
                            double* g_assign_lik_var, void* workspace, size_t workspace_bytes,
                            mgp_stream_t stream);

/* elbo = data_sum / n_batch - (kl_f + kl_a) / num_data   (models.py:76,79)
 * All pointers device; elbo_out float32 and elbo_out64 (nullable) double. */
int mgp_elbo_combine(const double* data_sum, const double* kl_f, const double* kl_a,
                     double n_batch, double num_data, float* elbo_out, double* elbo_out64,
                     mgp_stream_t stream);

/* Predictive epilogue (SGP.predict_y, models.py:38-41 -> likelihoods.py:31-32;
 * SMGP.predict_assign, models.py:85-89):
 *   y_mean[n][k] = fmean[k][n]; y_var[n][k] = fvar[k][n] + lik_var[k]
 *   assign[n][k] = softmax_k(amean[k][n])
 * Any output may be NULL.  Outputs are [N][K] row-major (the reference layout). */
int mgp_predict_epilogue(const float* fmean, const float* fvar, const float* amean, int64_t ldf,
                         const float* lik_var, int64_t N, int32_t K, float* y_mean, float* y_var,
                         float* assign, mgp_stream_t stream);

/* SMGP.predict_samples (models.py:91-103): a fresh assignment sample W (as in
 * mgp_elbo_terms) and one normal draw z shared by the y- and f-samples:
 *   samples_y[s][n] = sum_k W (mu_f + z sqrt(var_f + lik_var_k + jitter))
 *   samples_f[s][n] = sum_k W (mu_f + z sqrt(var_f + jitter))
 * (jitter: default_jitter(), the reparameterize of utils.py:26-27)
 * Explicit noise (all three [S][N][K], parity mode) or Philox (streams 0/1 for
 * W, stream 2 for z).  Outputs [S][N]; either may be NULL. */
int mgp_predict_samples(const float* mu_f, const float* var_f, const float* mu_a, const float* var_a,
                        int64_t ldf, const float* lik_var, int64_t N, int32_t K, int32_t S, float tau, float jitter,
                        const float* noise_zw, const float* noise_uw, const float* noise_zy,
                        uint64_t seed, int64_t n_offset, float* samples_y, float* samples_f,
                        mgp_stream_t stream);

/* Raw noise stream (for tests and for SMGP.predict_samples): writes
 * z[s][n][k] (normals) and/or u[s][n][k] (uniforms in (0,1)) exactly as
 * mgp_elbo_terms draws them in Philox mode.  Either pointer may be NULL. */
int mgp_philox_noise(uint64_t seed, int64_t n_offset, int64_t N, int32_t K, int32_t S, float* z,
                     float* u, mgp_stream_t stream);
/* ---------------------------------------------------------------- MultiClass likelihood
 * GPflow 2.7.0 likelihoods.MultiClass(num_classes = K, invlink = RobustMax(K, epsilon))
 * as the pred likelihood (demos/demo_tf2_modified_multiclass.py:43-45, reached
 * through BroadcastingLikelihood, broadcasting_lik.py:19-37,39-46):
 *   p_i(n) = RobustMax.prob_is_largest(i, mu_n, var_n)  (20-point Gauss-Hermite)
 *   ve_n   = p_y log(1 - eps) + (1 - p_y) log(eps / (K - 1)),  y = (int) Y[n]
 * The var-exp is one value per point, multiplied by W and summed over K as the
 * reference does (models.py:65-67).  Arguments as the Gaussian entries with
 * lik_var replaced by epsilon (0 < eps < 1, K >= 2); assign_lik_var != NULL
 * selects SMGPModified (its assign layer keeps the Gaussian likelihood).  The
 * backward has no likelihood-variance gradient (MultiClass has no trainable
 * parameter; RobustMax.epsilon is trainable=False). */
int mgp_elbo_terms_multiclass(const float* mu_f, const float* var_f, const float* mu_a, const float* var_a,
                              int64_t ldf, const float* Y, float epsilon, const float* assign_lik_var,
                              int64_t N, int32_t K, int32_t S, float tau, float jitter, const float* noise_z,
                              const float* noise_u, uint64_t seed, int64_t n_offset, double* data_sum,
                              void* workspace, size_t workspace_bytes, mgp_stream_t stream);
int mgp_elbo_terms_multiclass_backward(const float* mu_f, const float* var_f, const float* mu_a,
                                       const float* var_a, int64_t ldf, const float* Y, float epsilon,
                                       const float* assign_lik_var, int64_t N, int32_t K, int32_t S, float tau, float jitter,
                                       const float* noise_z, const float* noise_u, uint64_t seed,
                                       int64_t n_offset, float scale, float* G, int64_t ldg,
                                       double* g_assign_lik_var, void* workspace, size_t workspace_bytes,
                                       mgp_stream_t stream);
/* MultiClass._predict_mean_and_var: y_mean = ps, y_var = ps - ps^2 ([N][K] row-major),
 * ps[n][i] = p_i(n) (1 - eps) + (1 - p_i(n)) eps / (K - 1). */
int mgp_multiclass_predict(const float* fmean, const float* fvar, int64_t ldf, int64_t N, int32_t K,
                           float epsilon, float* y_mean, float* y_var, mgp_stream_t stream);
/* SMGP.predict_samples with the MultiClass predictive mean / variance for samples_y. */
int mgp_predict_samples_multiclass(const float* mu_f, const float* var_f, const float* mu_a,
                                   const float* var_a, int64_t ldf, float epsilon, int64_t N, int32_t K,
                                   int32_t S, float tau, float jitter, const float* noise_zw, const float* noise_uw,
                                   const float* noise_zy, uint64_t seed, int64_t n_offset, float* samples_y,
                                   float* samples_f, mgp_stream_t stream);

/* Philox stream-2 normals [S][N][K] (the z of mgp_predict_samples), as mgp_philox_noise. */
int mgp_philox_normal2(uint64_t seed, int64_t n_offset, int64_t N, int32_t K, int32_t S, float* z,
                       mgp_stream_t stream);

/* ---------------------------------------------------------------- method-level API
 * The stages K6 fuses, for the reference's public methods.  Latents are
 * expert-major [K][ldf]; sample s of point n is column s * stride_s + n
 * (stride_s = 0: one S-invariant conditional for S tiled copies of X).  Noise:
 * explicit [S][N][K] arrays (nullable) or K6's own Philox streams (z: stream 0,
 * u: stream 1, keyed by (n + n_offset, s, k / 4)), so the three calls below with
 * one seed reproduce mgp_elbo_terms with that seed.
 *
 * SMGP.W_dist (models.py:55-60): assign_layer.predict_f -> reparameterize
 * (utils.py:26-27): logits[s][n][k] = mu_a + z sqrt(var_a + jitter). */
int mgp_assign_logits(const float* mu_a, const float* var_a, int64_t ldf, int64_t stride_s, int64_t N,
                      int32_t K, int32_t S, float jitter, const float* noise_z, uint64_t seed, int64_t n_offset,
                      float* logits, mgp_stream_t stream);
/* RelaxedOneHotCategorical(temperature = tau, logits).sample() (TFP 0.18,
 * models.py:60,73): W[r] = softmax((g + logits[r]) / tau), g = -log(-log u), rows
 * r = s * N + n of logits / W [S * N][K]. */
int mgp_relaxed_onehot_sample(const float* logits, int64_t N, int32_t K, int32_t S, float tau,
                              const float* noise_u, uint64_t seed, int64_t n_offset, float* W,
                              mgp_stream_t stream);
/* SMGP.E_log_p_Y(Xt, Y, W) (models.py:63-67): out[n] = logsumexp_s(sum_k W ve) - log S,
 * W [S][N][K].  lik_var == NULL: the pred likelihood is MultiClass / RobustMax
 * (multiclass_eps); assign_lik_var != NULL: SMGPModified.E_log_p_Y (models.py:112-123),
 * which also reads the assign latents mu_a / var_a. */
int mgp_e_log_p_y(const float* mu_f, const float* var_f, const float* mu_a, const float* var_a, int64_t ldf,
                  int64_t stride_s, const float* Y, const float* lik_var, const float* assign_lik_var,
                  float multiclass_eps, const float* W, int64_t N, int32_t K, int32_t S, float* out,
                  mgp_stream_t stream);

/* ---------------------------------------------------------------- optimizer
 * KL gradient folded into the ELBO gradient: g_q_mu -= q_mu / num_data,
 * g_q_sqrt[k] -= tril(L_k - diag(1 / L_k[m,m])) / num_data (models.py:79). */
int mgp_kl_grad(const float* q_mu, int64_t ldq, const float* q_sqrt, int64_t ldqs, int64_t strideq,
                int64_t M, int32_t K, double num_data, float* g_q_mu, int64_t ldgq, float* g_q_sqrt,
                int64_t ldgs, int64_t strideg, mgp_stream_t stream);

/* One TF-legacy Adam step (tf.optimizers.Adam, utils/training_utils.py:6,10;
 * eps outside the bias correction) on a [rows][cols] block (leading dimension
 * ld) of parameter theta; g = d ELBO / d theta times grad_sign (-1 minimises
 * -ELBO), float or double (grad_is_double); m1, m2, u: rows * cols dense.
 * u != NULL: theta = softplus(u) is a positive parameter and Adam runs on u
 * (GPflow positive()).  t = 1-based step count. */
int mgp_adam_step(float* theta, float* u, const void* g, int32_t grad_is_double, int64_t ldg, float* m1,
                  float* m2, int64_t rows, int64_t cols, int64_t ld, float lr, float beta1, float beta2,
                  float eps, int64_t t, float grad_sign, mgp_stream_t stream);
/* mgp_adam_step on n (1 .. 16) parameter blocks in one launch (per-block arrays of
 * the arguments above; u[j] may be NULL; a block may be empty, its pointers unused), bit-identical to n
 * mgp_adam_step calls.  -1 .. -11: n, theta, u, g, grad_is_double, ldg, m1, m2, rows,
 * cols, ld (NULL array or a bad entry); -16: t. */
int mgp_adam_step_set(int32_t n, float* const* theta, float* const* u, const void* const* g,
                      const int32_t* grad_is_double, const int64_t* ldg, float* const* m1, float* const* m2,
                      const int64_t* rows, const int64_t* cols, const int64_t* ld, float lr, float beta1,
                      float beta2, float eps, int64_t t, float grad_sign, mgp_stream_t stream);


/* ---------------------------------------------------------------- the §8(b) front
 * One entry per reference operation in the default formats: what a
 * binding from another host language needs.  They are thin hosts over the kernels
 * above (csrc/front.hip); the format-specific entries above are the expert surface
 * the Python host uses for its fused, stream-overlapped ELBO step.  Every workspace
 * is sized by mgp_workspace_bytes(op, M, N, K) (0 = none needed; for
 * MGP_OP_RBF_BACKWARD pass D as K) and must be 16-B aligned. */
enum {
  MGP_OP_RBF_KUU_JITTER = 1,
  MGP_OP_RBF_KUF = 2,
  MGP_OP_POTRF_LOWER = 3,
  MGP_OP_TRSM_LLN = 4,
  MGP_OP_EXPERT_CONDITIONAL = 5,
  MGP_OP_GAUSS_KL_WHITE = 6,
  MGP_OP_ELBO_TERMS = 7,
  MGP_OP_ELBO_TERMS_BACKWARD = 8,
  MGP_OP_CONDITIONAL_BACKWARD = 9,
  MGP_OP_CHOL_BACKWARD = 10,
  MGP_OP_RBF_BACKWARD = 11
};
size_t mgp_workspace_bytes(int32_t op, int64_t M, int64_t N, int32_t K);
/* Kuu = K(Z, Z) + jitter I in float32 (covariances.Kuu, models.py:135); same as
 * mgp_rbf_kuu.  The ELBO path builds Kuu in float64 inside the factorisation
 * (mgp_kuu_potrf_trtri): a float32 Kuu carries cond(Kuu) * 2^-24 into L. */
int mgp_rbf_kuu_jitter(const float* Z, int64_t ldz, int64_t M, int32_t D, const float* variance,
                       const float* lengthscales, int32_t n_ls, float jitter, float* Kuu, int64_t ldk,
                       mgp_stream_t stream);
/* In place: A [M][lda] (lower triangle read) <- L = chol(A), zeros above the
 * diagonal; LinvT (nullable, [M][ldl]) <- (L^-1)^T, the form mgp_trsm_lln takes
 * L in.  Factorised in float64 (K3).  info (device int32) = 0 or the 1-based column
 * of the first non-positive pivot (tf.linalg.cholesky at models.py:141 raises
 * there).  lda, ldl % 4 == 0. */
int mgp_potrf_lower(float* A, int64_t lda, int64_t M, float* LinvT, int64_t ldl, int32_t* info,
                    void* workspace, size_t workspace_bytes, mgp_stream_t stream);
/* In place: B [M][ldb] <- L^-1 B, the triangular_solve(Lm, Kmn, lower=True) of
 * base_conditional (models.py:141-143), with L given as LinvT = (L^-1)^T from
 * mgp_potrf_lower (K4 as a triangular GEMM on exact three-plane bf16 images:
 * f32-accurate for any right-hand side). */
int mgp_trsm_lln(const float* LinvT, int64_t ldl, int64_t M, float* B, int64_t ldb, int64_t N,
                 void* workspace, size_t workspace_bytes, mgp_stream_t stream);
/* The K-expert whitened conditional from A = L^-1 Kuf (models.py:141-143):
 *   fmean[k][n] = sum_m A[m,n] q_mu[m,k]
 *   fvar[k][n]  = var - sum_m A[m,n]^2 + sum_m' (sum_{m>=m'} L_k[m,m'] A[m,n])^2
 * with L_k = band_part(q_sqrt[k], -1, 0), in the default split-f16 format (K5 on
 * f16 MFMAs, 22-bit operands).  q_mu [M][ldq >= K]; q_sqrt [K][M][ldqs] at element
 * stride strideq; fmean, fvar [K][ldf] (expert-major).  K <= 32. */
int mgp_expert_conditional(const float* A, int64_t lda, const float* q_mu, int64_t ldq,
                           const float* q_sqrt, int64_t ldqs, int64_t strideq, const float* variance,
                           int64_t M, int64_t N, int32_t K, float* fmean, float* fvar, int64_t ldf,
                           void* workspace, size_t workspace_bytes, mgp_stream_t stream);

#ifdef __cplusplus
}
#endif
#endif /* MGP_HIP_H */
