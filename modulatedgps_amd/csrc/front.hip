// The stable C-ABI front of SURVEY.md §8(b): one entry per reference operation, in the
// default formats, over the same kernels the Python host drives.
// A binding from another host language needs only these names; the format-specific
// entries (_x6, _f16, _f16c, _batch, ...) stay the expert surface the Python host uses
// for the fused, stream-overlapped ELBO step.
//
//   mgp_rbf_kuu_jitter      covariances.Kuu(Z, kernel, jitter)              models.py:135
//   mgp_potrf_lower         tf.linalg.cholesky(Kmm) in base_conditional      models.py:141
//   mgp_trsm_lln            tf.linalg.triangular_solve(Lm, Kmn, lower=True)  models.py:141-143
//   mgp_expert_conditional  fmean = A^T q_mu, fvar = Knn - sum A^2 + sum (L_k^T A)^2
//                                                                            models.py:141-143
//   mgp_workspace_bytes     the workspace any of them (and the other ops) needs
#include <algorithm>

#include "mgp_common.hpp"

namespace mgp {

constexpr int kStatRows = 64;   // rows of one stats tile (mgp_stats_tiles)

static inline size_t align256(size_t x) { return (x + 255) / 256 * 256; }
static inline int64_t round4(int64_t x) { return (x + 3) / 4 * 4; }

// stats[t][0][n] = sum_{m in tile t} A[m][n]^2, stats[t][1 + k][n] = sum_{m in tile t}
// A[m][n] q_mu[m][k] (the column statistics K4 produces beside the solve; here from an
// f32 A): one thread per column, coalesced row reads, q_mu's tile rows in LDS.
template <int KMAX>
__global__ __launch_bounds__(256) void col_stats_kernel(const float* __restrict__ A, int64_t lda,
                                                        const float* __restrict__ q_mu, int64_t ldq, int64_t M,
                                                        int64_t N, int K, float* __restrict__ stats, int64_t lds) {
  __shared__ float sq[kStatRows * KMAX];
  const int64_t t = blockIdx.y, m0 = t * kStatRows;
  for (int i = threadIdx.x; i < kStatRows * KMAX; i += 256) {
    const int r = i / KMAX, k = i % KMAX;
    sq[i] = (m0 + r < M && k < K) ? q_mu[(m0 + r) * ldq + k] : 0.f;
  }
  __syncthreads();
  const int64_t n = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (n >= N) return;
  const int rows = (int)std::min<int64_t>(kStatRows, M - m0);
  float s0 = 0.f, s[KMAX];
#pragma unroll
  for (int k = 0; k < KMAX; ++k) s[k] = 0.f;
  for (int r = 0; r < rows; ++r) {
    const float x = A[(m0 + r) * lda + n];
    s0 = fmaf(x, x, s0);
#pragma unroll
    for (int k = 0; k < KMAX; ++k) s[k] = fmaf(x, sq[r * KMAX + k], s[k]);
  }
  float* dst = stats + t * (K + 1) * lds + n;
  dst[0] = s0;
#pragma unroll
  for (int k = 0; k < KMAX; ++k)
    if (k < K) dst[(int64_t)(1 + k) * lds] = s[k];
}

template <int KMAX>
static int launch_col_stats(const float* A, int64_t lda, const float* q_mu, int64_t ldq, int64_t M, int64_t N, int K,
                            float* stats, int64_t lds, hipStream_t s) {
  const dim3 grid((unsigned)((N + 255) / 256), (unsigned)((M + kStatRows - 1) / kStatRows));
  hipLaunchKernelGGL(col_stats_kernel<KMAX>, grid, dim3(256), 0, s, A, lda, q_mu, ldq, M, N, K, stats, lds);
  return launch_status();
}

// workspace layouts (256-B aligned slots)
struct TrsmWs { size_t tfr, bfr, afr, qz, total; };
static TrsmWs trsm_ws(int64_t M, int64_t N) {
  TrsmWs w;
  w.tfr = 0;
  w.bfr = w.tfr + align256(mgp_x6_lower_bytes(M, 1));
  w.afr = w.bfr + align256(mgp_x6_cols_bytes(M, N));
  w.qz = w.afr + align256(mgp_x6_cols_bytes(M, N));
  w.total = w.qz + align256((size_t)std::max<int64_t>(M, 1) * sizeof(float));
  return w;
}
struct ExpertWs { size_t afr, lfr, stats, xws, total; };
static ExpertWs expert_ws(int64_t M, int64_t N, int32_t K) {
  ExpertWs w;
  w.afr = 0;
  w.lfr = w.afr + align256(mgp_x6_cols_bytes(M, N));
  w.stats = w.lfr + align256(mgp_x6_lower_bytes(M, K));
  w.xws = w.stats + align256((size_t)mgp_stats_tiles(M) * (size_t)(K + 1) * (size_t)round4(N) * sizeof(float));
  w.total = w.xws + align256(mgp_expert_x6_workspace_bytes(M, N, K));
  return w;
}
struct PotrfWs { size_t chol, L, LinvT, total; };
static PotrfWs potrf_ws(int64_t M) {
  PotrfWs w;
  w.chol = 0;
  w.L = align256(mgp_chol_workspace_bytes(M, 1));
  w.LinvT = w.L + align256((size_t)M * (size_t)round4(M) * sizeof(float));
  w.total = w.LinvT + align256((size_t)M * (size_t)round4(M) * sizeof(float));
  return w;
}

}  // namespace mgp

using namespace mgp;

extern "C" size_t mgp_workspace_bytes(int32_t op, int64_t M, int64_t N, int32_t K) {
  if (M < 0 || N < 0 || K < 0) return 0;
  switch (op) {
    case MGP_OP_RBF_KUU_JITTER:
    case MGP_OP_RBF_KUF:
      return 0;
    case MGP_OP_POTRF_LOWER:
      return M > 0 ? potrf_ws(M).total : 0;
    case MGP_OP_TRSM_LLN:
      return (M > 0 && N > 0) ? trsm_ws(M, N).total : 0;
    case MGP_OP_EXPERT_CONDITIONAL:
      return (M > 0 && N > 0 && K > 0) ? expert_ws(M, N, K).total : 0;
    case MGP_OP_GAUSS_KL_WHITE:
      return mgp_kl_workspace_bytes(M, K);
    case MGP_OP_ELBO_TERMS:
      return mgp_elbo_workspace_bytes(N);
    case MGP_OP_ELBO_TERMS_BACKWARD:
      return mgp_elbo_backward_workspace_bytes(N, K);
    case MGP_OP_CONDITIONAL_BACKWARD:
      return mgp_conditional_backward_workspace_bytes(M, N, K);
    case MGP_OP_CHOL_BACKWARD:
      return mgp_chol_backward_workspace_bytes(M);
    case MGP_OP_RBF_BACKWARD:
      return mgp_rbf_backward_workspace_bytes(N, M, K);   // K carries D here
    default:
      return 0;
  }
}

extern "C" int mgp_rbf_kuu_jitter(const float* Z, int64_t ldz, int64_t M, int32_t D, const float* variance,
                                  const float* lengthscales, int32_t n_ls, float jitter, float* Kuu, int64_t ldk,
                                  mgp_stream_t stream) {
  return mgp_rbf_kuu(Z, ldz, M, D, variance, lengthscales, n_ls, jitter, Kuu, ldk, stream);
}

extern "C" int mgp_potrf_lower(float* A, int64_t lda, int64_t M, float* LinvT, int64_t ldl, int32_t* info,
                               void* workspace, size_t workspace_bytes, mgp_stream_t stream) {
  if (!A) return -1;
  if (lda < M || lda % 4) return -2;
  if (M < 0) return -3;
  if (LinvT && (ldl < M || ldl % 4)) return -5;
  if (!info) return -6;
  if (M == 0) return MGP_OK;
  const PotrfWs w = potrf_ws(M);
  if (!workspace || workspace_bytes < w.total) return MGP_ERR_WORKSPACE;
  if (!aligned16(workspace) || !aligned16(A) || (LinvT && !aligned16(LinvT))) return MGP_ERR_ALIGN;
  hipStream_t s = (hipStream_t)stream;
  char* ws = (char*)workspace;
  const int64_t ldw = round4(M);
  float* L = (float*)(ws + w.L);
  float* LT = (float*)(ws + w.LinvT);
  // K3 reads A's lower triangle in its first launch while other workgroups of that
  // launch already write L's first diagonal tile, so L goes to the workspace and is
  // copied over A afterwards (stream-ordered)
  int st = mgp_potrf_trtri(A, lda, 0, M, 1, L, LT, ldw, 0, info, ws + w.chol, w.L - w.chol, stream);
  if (st) return st;
  st = hip_status(hipMemcpy2DAsync(A, lda * sizeof(float), L, ldw * sizeof(float), M * sizeof(float), M,
                                   hipMemcpyDeviceToDevice, s));
  if (st || !LinvT) return st;
  return hip_status(hipMemcpy2DAsync(LinvT, ldl * sizeof(float), LT, ldw * sizeof(float), M * sizeof(float), M,
                                     hipMemcpyDeviceToDevice, s));
}

extern "C" int mgp_trsm_lln(const float* LinvT, int64_t ldl, int64_t M, float* B, int64_t ldb, int64_t N,
                            void* workspace, size_t workspace_bytes, mgp_stream_t stream) {
  if (!LinvT) return -1;
  if (ldl < M) return -2;
  if (M < 0) return -3;
  if (!B) return -4;
  if (ldb < N) return -5;
  if (N < 0) return -6;
  if (M == 0 || N == 0) return MGP_OK;
  const TrsmWs w = trsm_ws(M, N);
  if (!workspace || workspace_bytes < w.total) return MGP_ERR_WORKSPACE;
  if (!aligned16(workspace)) return MGP_ERR_ALIGN;
  hipStream_t s = (hipStream_t)stream;
  char* ws = (char*)workspace;
  // exact three-plane (x6) images of L^-T and B: no scale bound is needed for an
  // arbitrary right-hand side, and the products are f32-accurate; K4 then writes
  // A = L^-1 B in f32 over B (its input is the image, so in place is safe)
  const size_t tb = mgp_x6_lower_bytes(M, 1), cb = mgp_x6_cols_bytes(M, N);
  float* qz = (float*)(ws + w.qz);
  int st = hip_status(hipMemsetAsync(qz, 0, (size_t)M * sizeof(float), s));
  if (st) return st;
  st = mgp_split_upper_x6(LinvT, ldl, M, ws + w.tfr, tb, stream);
  if (st) return st;
  st = mgp_split_cols_x6(B, ldb, M, N, ws + w.bfr, cb, stream);
  if (st) return st;
  return mgp_trsm_stats_x6(ws + w.tfr, tb, ws + w.bfr, cb, M, N, qz, 1, 1, ws + w.afr, cb, nullptr, N, B, ldb,
                           stream);
}

extern "C" int mgp_expert_conditional(const float* A, int64_t lda, const float* q_mu, int64_t ldq,
                                      const float* q_sqrt, int64_t ldqs, int64_t strideq, const float* variance,
                                      int64_t M, int64_t N, int32_t K, float* fmean, float* fvar, int64_t ldf,
                                      void* workspace, size_t workspace_bytes, mgp_stream_t stream) {
  if (!A) return -1;
  if (lda < N) return -2;
  if (!q_mu) return -3;
  if (ldq < K) return -4;
  if (!q_sqrt) return -5;
  if (ldqs < M) return -6;
  if (K > 1 && strideq < ldqs * M) return -7;
  if (!variance) return -8;
  if (M < 0) return -9;
  if (N < 0) return -10;
  if (K < 1) return -11;
  if (K > 32) return MGP_ERR_UNSUPPORTED;
  if (!fmean) return -12;
  if (!fvar) return -13;
  if (ldf < N) return -14;
  if (M == 0 || N == 0) return MGP_OK;
  const ExpertWs w = expert_ws(M, N, K);
  if (!workspace || workspace_bytes < w.total) return MGP_ERR_WORKSPACE;
  if (!aligned16(workspace)) return MGP_ERR_ALIGN;
  hipStream_t s = (hipStream_t)stream;
  char* ws = (char*)workspace;
  const size_t cb = mgp_x6_cols_bytes(M, N), lb = mgp_x6_lower_bytes(M, K);
  const int64_t lds = round4(N);
  float* stats = (float*)(ws + w.stats);
  // the default format (split-f16, 22-bit operands, three f16 products): A's image
  // at its device maximum, tril(q_sqrt)'s image, the column statistics in f32, K5
  int st = mgp_split_cols_f16(A, lda, M, N, ws + w.afr, cb, stream);
  if (st) return st;
  st = mgp_split_lower_f16(q_sqrt, ldqs, strideq, M, K, ws + w.lfr, lb, stream);
  if (st) return st;
  st = K <= 8    ? launch_col_stats<8>(A, lda, q_mu, ldq, M, N, K, stats, lds, s)
       : K <= 16 ? launch_col_stats<16>(A, lda, q_mu, ldq, M, N, K, stats, lds, s)
                 : launch_col_stats<32>(A, lda, q_mu, ldq, M, N, K, stats, lds, s);
  if (st) return st;
  return mgp_expert_conditional_f16(ws + w.afr, cb, ws + w.lfr, lb, stats, lds, variance, M, N, K, fmean, fvar, ldf,
                                    ws + w.xws, mgp_expert_x6_workspace_bytes(M, N, K), stream);
}
