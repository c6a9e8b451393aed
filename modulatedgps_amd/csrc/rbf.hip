// K1 / K2: RBF (SquaredExponential) covariance blocks Kuf = K(Z, X) and
// Kuu = K(Z, Z) + jitter I.
//
// Reference: MixtureGPs/models.py:135 (covariances.Kuu) and :139
// (self.kernel.K(Z, Xnew)); GPflow 2.7 SquaredExponential.K_r2(r2) =
// var * exp(-0.5 r2), r2 = square_distance(X / l, X2 / l).
//
// Roofline: HBM-write bound.  Algorithmic bytes = 4 * (N*D + M*D + M*N); per
// output element the kernel does D subtracts + D FMAs + 1 exp2, far below the
// f32 VALU ridge.  Layout: Kuf [M][ldk] row-major (N contiguous); each thread
// owns 4 consecutive columns (one float4 store per row), a wave writes 1 KiB
// contiguous per row.  The scaled Z rows of the tile are staged once in LDS
// and read as wave-uniform broadcasts.
//
// Numerics: direct-difference form sum_d (z_d - x_d)^2 * c_d^2 (exact symmetric,
// never negative) instead of GPflow's |a|^2 + |b|^2 - 2ab expansion; the
// exp(-0.5 r2) is evaluated as exp2(-r2') with c_d = sqrt(0.5 log2 e) / l_d.
#include <type_traits>

#include "kuf_image.hpp"
#include "mgp_common.hpp"

namespace mgp {

constexpr int kRbfThreads = 256;
constexpr int kRbfCols = 4;                       // columns per thread
constexpr int kRbfTileN = kRbfThreads * kRbfCols; // 1024 columns per workgroup
constexpr int kRbfTileM = 64;                     // rows per workgroup (X re-read M/64 times)

template <int DMAX>
__global__ __launch_bounds__(kRbfThreads) void rbf_kernel(
    const float* __restrict__ X, int64_t ldx, const float* __restrict__ Z, int64_t ldz, int64_t N,
    int64_t M, int D, const float* __restrict__ variance, const float* __restrict__ ls, int n_ls,
    float jitter, float* __restrict__ out, int64_t ldo) {
  __shared__ float zs[kRbfTileM][DMAX];
  __shared__ float cs[DMAX];
  const int t = threadIdx.x;
  const int64_t n0 = (int64_t)blockIdx.x * kRbfTileN + (int64_t)t * kRbfCols;
  const int64_t m0 = (int64_t)blockIdx.y * kRbfTileM;
  const float kHalfLog2e = 0.8493218002880191f;  // sqrt(0.5 * log2(e))

  if (t < DMAX) cs[t] = (t < D) ? kHalfLog2e / ls[n_ls == 1 ? 0 : t] : 0.f;
  __syncthreads();
  for (int i = t; i < kRbfTileM * DMAX; i += kRbfThreads) {
    const int r = i / DMAX, d = i % DMAX;
    const int64_t m = m0 + r;
    zs[r][d] = (m < M && d < D) ? Z[m * ldz + d] * cs[d] : 0.f;
  }
  float xs[kRbfCols][DMAX];
#pragma unroll
  for (int j = 0; j < kRbfCols; ++j) {
    const int64_t n = n0 + j;
#pragma unroll
    for (int d = 0; d < DMAX; ++d) xs[j][d] = (n < N && d < D) ? X[n * ldx + d] * cs[d] : 0.f;
  }
  const float var = variance[0];
  __syncthreads();

  const int rows = (int)((M - m0) < kRbfTileM ? (M - m0) : kRbfTileM);
  for (int r = 0; r < rows; ++r) {
    const int64_t m = m0 + r;
    float v[kRbfCols];
#pragma unroll
    for (int j = 0; j < kRbfCols; ++j) {
      float acc = 0.f;
#pragma unroll
      for (int d = 0; d < DMAX; ++d) {
        const float diff = zs[r][d] - xs[j][d];
        acc = fmaf(diff, diff, acc);
      }
      v[j] = var * exp2f(-acc);
      if (jitter != 0.f && m == n0 + j) v[j] += jitter;
    }
    float* o = out + m * ldo + n0;
    if (n0 + kRbfCols <= N) {
      *reinterpret_cast<floatx4*>(o) = floatx4{v[0], v[1], v[2], v[3]};
    } else {
#pragma unroll
      for (int j = 0; j < kRbfCols; ++j)
        if (n0 + j < N) o[j] = v[j];
    }
  }
}

// K1 writing Kuf's split-bf16 / split-f16 image (split3.hip layout) instead of f32
// Kuf: one block of kuf_image.hpp per 256-thread workgroup (the body, its layout and
// numerics are documented there; the K3 step launches run the same blocks as their
// Kuf side job, mgp_kuu_potrf_trtri_kuf).
template <int DMAX, bool F16 = false>
__global__ __launch_bounds__(kRbfThreads) void rbf_kuf_x6_kernel(
    const float* __restrict__ X, int64_t ldx, const float* __restrict__ Z, int64_t ldz, int64_t N,
    int64_t M, int D, const float* __restrict__ variance, const float* __restrict__ ls, int n_ls, int nmk,
    bf16x8* __restrict__ Kfr, float* __restrict__ bound, int row_blocks) {
  __shared__ float lds[kuf_block_lds_floats<DMAX>()];
  const KufImageArgs a = {X, ldx, Z, ldz, N, M, D, variance, ls, n_ls, nmk, row_blocks, Kfr, bound};
  kuf_image_block<DMAX, F16>(a, blockIdx.x, threadIdx.x, true, lds);
}

static int rbf_launch(const float* X, int64_t ldx, const float* Z, int64_t ldz, int64_t N, int64_t M,
                      int D, const float* variance, const float* ls, int n_ls, float jitter, float* out,
                      int64_t ldo, hipStream_t stream) {
  if (N <= 0 || M <= 0) return MGP_OK;
  dim3 grid((unsigned)((N + kRbfTileN - 1) / kRbfTileN), (unsigned)((M + kRbfTileM - 1) / kRbfTileM));
  dim3 block(kRbfThreads);
#define MGP_RBF_CASE(DM)                                                                            \
  if (D <= DM) {                                                                                     \
    hipLaunchKernelGGL(rbf_kernel<DM>, grid, block, 0, stream, X, ldx, Z, ldz, N, M, D, variance, ls, \
                       n_ls, jitter, out, ldo);                                                      \
    return launch_status();                                                                          \
  }
  MGP_RBF_CASE(1)
  MGP_RBF_CASE(2)
  MGP_RBF_CASE(4)
  MGP_RBF_CASE(8)
  MGP_RBF_CASE(16)
  MGP_RBF_CASE(32)
#undef MGP_RBF_CASE
  return MGP_ERR_UNSUPPORTED;
}

// ------------------------------------------------------------------ RBF backward
// Reverse mode of K(Z, X) = var exp(-1/2 sum_d c_d^2 (z_d - x_d)^2), c = 1 / l
// (models.py:135,139) for a cotangent gK [M][N]: with w_mn = gK_mn k_mn and the
// centred sums (no cancellation between large terms)
//   S0_m = sum_n w_mn,  T1_md = sum_n w_mn (x_nd - z_md),  T2_md = sum_n w_mn (x_nd - z_md)^2
//   g_var = sum w / var,  g_z_md = c_d^2 T1_md,  g_l_d = c_d^3 sum_m T2_md.
// For Kuu (X = Z, symmetric gK) z enters both arguments: g_z doubles.
// Kernel 1: 4 waves x 2 rows of Z per block, lanes stride over an n-chunk four
// points at a time; each lane accumulates its <= 64 points in float32 (sums of
// centred terms), the lane / chunk reduction is float64.  Kernel 2 folds the
// chunks (one thread per sum), kernel 3 writes the grads.
// VEC (ldx % 4 == 0, ldx >= DMAX, X 16-byte aligned): a point's coordinates come
// in DMAX / 4 dwordx4 loads instead of DMAX dword loads at a 4 ldx-byte lane
// stride -- the strided dword loads cost the address unit 8x the cycles and
// bounded this kernel.
constexpr int kRbfRows = 2;  // rows of Z per wave
#ifndef MGP_RBF_PACKED
#define MGP_RBF_PACKED 1
#endif
constexpr bool kRbfPacked = MGP_RBF_PACKED;
typedef float floatx2v __attribute__((ext_vector_type(2)));
// one workgroup's rows (blockIdx.x) over the points [nb, ne); part: this chunk's [M][NS]
template <int DMAX, bool VEC>
__device__ __forceinline__ void rbf_bwd_rows_body(const float* __restrict__ X, int64_t ldx,
                                                  const float* __restrict__ Z, int64_t ldz, int64_t nb, int64_t ne,
                                                  int64_t M, int D, const float* __restrict__ variance,
                                                  const float* __restrict__ ls, int n_ls,
                                                  const float* __restrict__ gK, int64_t ldg,
                                                  double* __restrict__ part) {
  constexpr int NS = 1 + 2 * DMAX, R = kRbfRows;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t m0 = (int64_t)blockIdx.x * 4 * R + R * w;
  float hc2[DMAX], z[R][DMAX];
#pragma unroll
  for (int d = 0; d < DMAX; ++d) {
    const float c = (d < D) ? 1.f / ls[n_ls == 1 ? 0 : d] : 0.f;
    hc2[d] = -0.5f * c * c;
  }
#pragma unroll
  for (int r = 0; r < R; ++r)
#pragma unroll
    for (int d = 0; d < DMAX; ++d) z[r][d] = (m0 + r < M && d < D) ? Z[(m0 + r) * ldz + d] : 0.f;
  const float var = variance[0];
  float acc[R][NS];
#pragma unroll
  for (int r = 0; r < R; ++r)
#pragma unroll
    for (int j = 0; j < NS; ++j) acc[r][j] = 0.f;
  auto point = [&](int64_t n) {
    float x[DMAX], g[R];
    if constexpr (VEC && DMAX >= 4) {
#pragma unroll
      for (int q4 = 0; q4 < DMAX / 4; ++q4) {
        const floatx4 v = *reinterpret_cast<const floatx4*>(X + n * ldx + 4 * q4);
#pragma unroll
        for (int j = 0; j < 4; ++j) x[4 * q4 + j] = (4 * q4 + j < D) ? v[j] : 0.f;
      }
    } else {
#pragma unroll
      for (int d = 0; d < DMAX; ++d) x[d] = (d < D) ? X[n * ldx + d] : 0.f;
    }
#pragma unroll
    for (int r = 0; r < R; ++r) g[r] = (m0 + r < M) ? gK[(m0 + r) * ldg + n] : 0.f;
    if constexpr (kRbfPacked && DMAX % 2 == 0) {
      // coordinate pairs on packed f32 VALU ops (v_pk_add / v_pk_mul / v_pk_fma_f32):
      // half the instructions of the per-coordinate terms
#pragma unroll
      for (int r = 0; r < R; ++r) {
        floatx2v dx[DMAX / 2], qv = {0.f, 0.f};
#pragma unroll
        for (int p = 0; p < DMAX / 2; ++p) {
          dx[p] = floatx2v{x[2 * p], x[2 * p + 1]} - floatx2v{z[r][2 * p], z[r][2 * p + 1]};
          qv = floatx2v{hc2[2 * p], hc2[2 * p + 1]} * dx[p] * dx[p] + qv;
        }
        const float wv = g[r] * (var * __expf(qv[0] + qv[1]));
        acc[r][0] += wv;
        const floatx2v w2 = {wv, wv};
#pragma unroll
        for (int p = 0; p < DMAX / 2; ++p) {
          const floatx2v t = w2 * dx[p];
          floatx2v a1 = {acc[r][1 + 2 * p], acc[r][2 + 2 * p]};
          floatx2v a2 = {acc[r][1 + DMAX + 2 * p], acc[r][2 + DMAX + 2 * p]};
          a1 += t;
          a2 = t * dx[p] + a2;
          acc[r][1 + 2 * p] = a1[0];
          acc[r][2 + 2 * p] = a1[1];
          acc[r][1 + DMAX + 2 * p] = a2[0];
          acc[r][2 + DMAX + 2 * p] = a2[1];
        }
      }
      return;
    }
#pragma unroll
    for (int r = 0; r < R; ++r) {
      float dx[DMAX], q = 0.f;
#pragma unroll
      for (int d = 0; d < DMAX; ++d) {
        dx[d] = x[d] - z[r][d];
        q = fmaf(hc2[d] * dx[d], dx[d], q);
      }
      const float wv = g[r] * (var * __expf(q));
      acc[r][0] += wv;
#pragma unroll
      for (int d = 0; d < DMAX; ++d) {
        const float t = wv * dx[d];
        acc[r][1 + d] += t;
        acc[r][1 + DMAX + d] = fmaf(t, dx[d], acc[r][1 + DMAX + d]);
      }
    }
  };
  int64_t n = nb + lane;
  for (; n + 192 < ne; n += 256) {
    point(n);
    point(n + 64);
    point(n + 128);
    point(n + 192);
  }
  for (; n < ne; n += 64) point(n);
#pragma unroll
  for (int r = 0; r < R; ++r)
#pragma unroll
    for (int j = 0; j < NS; ++j) {
      double v = (double)acc[r][j];
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
      if (lane == 0 && m0 + r < M) part[(m0 + r) * NS + j] = v;
    }
}

template <int DMAX, bool VEC = false>
__global__ __launch_bounds__(256) void rbf_bwd_rows_kernel(const float* __restrict__ X, int64_t ldx,
                                                           const float* __restrict__ Z, int64_t ldz, int64_t N,
                                                           int64_t M, int D, const float* __restrict__ variance,
                                                           const float* __restrict__ ls, int n_ls,
                                                           const float* __restrict__ gK, int64_t ldg,
                                                           int64_t nchunk, double* __restrict__ part) {
  constexpr int NS = 1 + 2 * DMAX;
  const int64_t nb = (int64_t)blockIdx.y * nchunk;
  const int64_t ne = (nb + nchunk < N) ? nb + nchunk : N;
  rbf_bwd_rows_body<DMAX, VEC>(X, ldx, Z, ldz, nb, ne, M, D, variance, ls, n_ls, gK, ldg,
                               part + (int64_t)blockIdx.y * M * NS);
}

// The layers of mgp_rbf_backward_batch: per layer the Kuf cotangent's chunks
// (blockIdx.y < nch, over X) and the Kuu cotangent's (blockIdx.y == nch, X = Z, all
// M points in one chunk), each into its own part slab; blockIdx.z = layer.
constexpr int kRbfMaxBatch = 8;
struct RbfBwdLayers {
  const float* Z[kRbfMaxBatch]; const float* var[kRbfMaxBatch]; const float* ls[kRbfMaxBatch];
  const float* gKuf[kRbfMaxBatch]; const float* gKuu[kRbfMaxBatch];
  float* gZ[kRbfMaxBatch]; double* g_var[kRbfMaxBatch]; double* g_ls[kRbfMaxBatch];
};
template <int DMAX, bool VEC>
__global__ __launch_bounds__(256) void rbf_bwd_rows_batch_kernel(const float* __restrict__ X, int64_t ldx,
                                                                 int64_t N, int64_t ldz, int64_t M, int D, int n_ls,
                                                                 RbfBwdLayers lay, int64_t ldgf, int64_t ldgu,
                                                                 int64_t nchunk, int nch, int64_t slab,
                                                                 double* __restrict__ ws) {
  constexpr int NS = 1 + 2 * DMAX;
  const int b = blockIdx.z, y = blockIdx.y;
  double* part = ws + (int64_t)b * slab + (int64_t)y * M * NS;
  if (y < nch) {
    const int64_t nb = (int64_t)y * nchunk, ne = (nb + nchunk < N) ? nb + nchunk : N;
    rbf_bwd_rows_body<DMAX, VEC>(X, ldx, lay.Z[b], ldz, nb, ne, M, D, lay.var[b], lay.ls[b], n_ls, lay.gKuf[b],
                                 ldgf, part);
  } else {
    rbf_bwd_rows_body<DMAX, VEC>(lay.Z[b], ldz, lay.Z[b], ldz, 0, M, M, D, lay.var[b], lay.ls[b], n_ls,
                                 lay.gKuu[b], ldgu, part);
  }
}

// part[0][m][j] = sum over the chunks of part[ch][m][j] (in place: each thread
// reads only its own (m, j) of every chunk), one thread per (m, j), fixed order.
// blockIdx.y: the layer (part advances by slab doubles)
__global__ __launch_bounds__(256) void rbf_bwd_fold_kernel(double* __restrict__ part, int nchunks, int64_t total,
                                                           int64_t slab = 0) {
  const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
  part += blockIdx.y * slab;
  if (idx >= total) return;
  double v = part[idx];
  for (int ch = 1; ch < nchunks; ++ch) v += part[(int64_t)ch * total + idx];
  part[idx] = v;
}

template <int DMAX>
__device__ __forceinline__ void rbf_bwd_finish_body(const double* __restrict__ part, int nchunks, int64_t M, int D,
                                                    const float* __restrict__ variance, const float* __restrict__ ls,
                                                    int n_ls, float zfactor, int accumulate, float* __restrict__ gZ,
                                                    int64_t ldgz, double* __restrict__ g_var,
                                                    double* __restrict__ g_ls, double* scratch, int acc_var) {
  constexpr int NS = 1 + 2 * DMAX;
  double gl[DMAX], s0tot = 0.0;
#pragma unroll
  for (int d = 0; d < DMAX; ++d) gl[d] = 0.0;
  double c[DMAX];
#pragma unroll
  for (int d = 0; d < DMAX; ++d) c[d] = (d < D) ? 1.0 / (double)ls[n_ls == 1 ? 0 : d] : 0.0;
  for (int64_t m = threadIdx.x; m < M; m += 256) {
    double S[NS];
#pragma unroll
    for (int j = 0; j < NS; ++j) S[j] = 0.0;
    for (int ch = 0; ch < nchunks; ++ch)
#pragma unroll
      for (int j = 0; j < NS; ++j) S[j] += part[((int64_t)ch * M + m) * NS + j];
    s0tot += S[0];
#pragma unroll
    for (int d = 0; d < DMAX; ++d) {
      if (d >= D) break;
      const double gz = zfactor * c[d] * c[d] * S[1 + d];
      gZ[m * ldgz + d] = (float)(accumulate ? (double)gZ[m * ldgz + d] + gz : gz);
      gl[d] += c[d] * c[d] * c[d] * S[1 + DMAX + d];
    }
  }
  const double var = (double)variance[0];
  const double gv = block_sum<double>(s0tot, scratch) / var;
  if (threadIdx.x == 0) *g_var = acc_var ? *g_var + gv : gv;
  double giso = 0.0;
#pragma unroll
  for (int d = 0; d < DMAX; ++d) {
    if (d >= D) break;
    __syncthreads();
    const double v = block_sum<double>(gl[d], scratch);
    if (threadIdx.x == 0) {
      if (n_ls == 1) giso += v;
      else g_ls[d] = accumulate ? g_ls[d] + v : v;
    }
  }
  if (threadIdx.x == 0 && n_ls == 1) g_ls[0] = accumulate ? g_ls[0] + giso : giso;
}

template <int DMAX>
__global__ __launch_bounds__(256) void rbf_bwd_finish_kernel(const double* __restrict__ part, int nchunks, int64_t M,
                                                             int D, const float* __restrict__ variance,
                                                             const float* __restrict__ ls, int n_ls, float zfactor,
                                                             int accumulate, float* __restrict__ gZ, int64_t ldgz,
                                                             double* __restrict__ g_var, double* __restrict__ g_ls) {
  __shared__ double scratch[16];
  rbf_bwd_finish_body<DMAX>(part, nchunks, M, D, variance, ls, n_ls, zfactor, accumulate, gZ, ldgz, g_var, g_ls,
                            scratch, accumulate);
}

// layer blockIdx.x: the Kuf contribution (folded slab 0; accumulate as given), then
// the Kuu one (slab nch, symmetric) added to it -- the two finishes of the per-call path
template <int DMAX>
__global__ __launch_bounds__(256) void rbf_bwd_finish_batch_kernel(const double* __restrict__ ws, int64_t slab,
                                                                   int nch, int64_t M, int D, int n_ls,
                                                                   RbfBwdLayers lay, int accumulate, int64_t ldgz) {
  constexpr int NS = 1 + 2 * DMAX;
  __shared__ double scratch[16];
  const int b = blockIdx.x;
  const double* part = ws + (int64_t)b * slab;
  rbf_bwd_finish_body<DMAX>(part, 1, M, D, lay.var[b], lay.ls[b], n_ls, 1.f, accumulate & 1, lay.gZ[b], ldgz,
                            lay.g_var[b], lay.g_ls[b], scratch, accumulate != 0);
  __syncthreads();
  rbf_bwd_finish_body<DMAX>(part + (int64_t)nch * M * NS, 1, M, D, lay.var[b], lay.ls[b], n_ls, 2.f, 1, lay.gZ[b],
                            ldgz, lay.g_var[b], lay.g_ls[b], scratch, 1);
}

}  // namespace mgp

using namespace mgp;

extern "C" int mgp_rbf_kuf(const float* X, int64_t ldx, const float* Z, int64_t ldz, int64_t N,
                           int64_t M, int32_t D, const float* variance, const float* lengthscales,
                           int32_t n_ls, float* Kuf, int64_t ldk, mgp_stream_t stream) {
  if (!X) return -1;
  if (ldx < D) return -2;
  if (!Z) return -3;
  if (ldz < D) return -4;
  if (N < 0) return -5;
  if (M < 0) return -6;
  if (D < 1) return -7;
  if (D > 32) return MGP_ERR_UNSUPPORTED;
  if (!variance) return -8;
  if (!lengthscales) return -9;
  if (n_ls != 1 && n_ls != D) return -10;
  if (!Kuf) return -11;
  if (ldk < N) return -12;
  if (ldk % 4 || !aligned16(Kuf)) return MGP_ERR_ALIGN;
  return rbf_launch(X, ldx, Z, ldz, N, M, D, variance, lengthscales, n_ls, 0.f, Kuf, ldk,
                    (hipStream_t)stream);
}

extern "C" int mgp_rbf_kuu(const float* Z, int64_t ldz, int64_t M, int32_t D, const float* variance,
                           const float* lengthscales, int32_t n_ls, float jitter, float* Kuu,
                           int64_t ldk, mgp_stream_t stream) {
  if (!Z) return -1;
  if (ldz < D) return -2;
  if (M < 0) return -3;
  if (D < 1) return -4;
  if (D > 32) return MGP_ERR_UNSUPPORTED;
  if (!variance) return -5;
  if (!lengthscales) return -6;
  if (n_ls != 1 && n_ls != D) return -7;
  if (!Kuu) return -9;
  if (ldk < M) return -10;
  if (ldk % 4 || !aligned16(Kuu)) return MGP_ERR_ALIGN;
  return rbf_launch(Z, ldz, Z, ldz, M, M, D, variance, lengthscales, n_ls, jitter, Kuu, ldk,
                    (hipStream_t)stream);
}

extern "C" size_t mgp_x6_cols_bytes(int64_t M, int64_t N);

static int rbf_kuf_image(const float* X, int64_t ldx, const float* Z, int64_t ldz, int64_t N, int64_t M, int32_t D,
                         const float* variance, const float* lengthscales, int32_t n_ls, void* Kfr,
                         size_t kfr_bytes, mgp_stream_t stream, bool f16) {
  if (!X) return -1;
  if (ldx < D) return -2;
  if (!Z) return -3;
  if (ldz < D) return -4;
  if (N < 0) return -5;
  if (M < 0) return -6;
  if (D < 1) return -7;
  if (D > 32) return MGP_ERR_UNSUPPORTED;
  if (!variance) return -8;
  if (!lengthscales) return -9;
  if (n_ls != 1 && n_ls != D) return -10;
  if (!Kfr) return -11;
  if (N == 0 || M == 0) return MGP_OK;
  if (kfr_bytes < mgp_x6_cols_bytes(M, N)) return -12;
  if (!aligned16(Kfr)) return MGP_ERR_ALIGN;
  const int64_t Mp = (M + 127) / 128 * 128, Np = (N + 255) / 256 * 256;
  const int nmk = (int)(Mp / 16);
  const int row_blocks = (int)(Mp / 128);
  const dim3 grid((unsigned)(Np / 128 * row_blocks)), block(kRbfThreads);
  hipStream_t s = (hipStream_t)stream;
  float* bound = (float*)((char*)Kfr + mgp_x6_cols_bytes(M, N) - 256);  // image trailer (split3.hip)
#define MGP_RBF_X6_CASE(DM)                                                                            \
  if (D <= DM) {                                                                                       \
    if (f16)                                                                                           \
      hipLaunchKernelGGL((rbf_kuf_x6_kernel<DM, true>), grid, block, 0, s, X, ldx, Z, ldz, N, M, D,    \
                         variance, lengthscales, n_ls, nmk, (bf16x8*)Kfr, bound, row_blocks);                      \
    else                                                                                               \
      hipLaunchKernelGGL((rbf_kuf_x6_kernel<DM, false>), grid, block, 0, s, X, ldx, Z, ldz, N, M, D,   \
                         variance, lengthscales, n_ls, nmk, (bf16x8*)Kfr, nullptr, row_blocks);                    \
    return launch_status();                                                                            \
  }
  MGP_RBF_X6_CASE(1)
  MGP_RBF_X6_CASE(2)
  MGP_RBF_X6_CASE(4)
  MGP_RBF_X6_CASE(8)
  MGP_RBF_X6_CASE(16)
  MGP_RBF_X6_CASE(32)
#undef MGP_RBF_X6_CASE
  return MGP_ERR_UNSUPPORTED;
}

extern "C" int mgp_rbf_kuf_x6(const float* X, int64_t ldx, const float* Z, int64_t ldz, int64_t N, int64_t M,
                              int32_t D, const float* variance, const float* lengthscales, int32_t n_ls,
                              void* Kfr, size_t kfr_bytes, mgp_stream_t stream) {
  return rbf_kuf_image(X, ldx, Z, ldz, N, M, D, variance, lengthscales, n_ls, Kfr, kfr_bytes, stream, false);
}

extern "C" int mgp_rbf_kuf_f16(const float* X, int64_t ldx, const float* Z, int64_t ldz, int64_t N, int64_t M,
                               int32_t D, const float* variance, const float* lengthscales, int32_t n_ls,
                               void* Kfr, size_t kfr_bytes, mgp_stream_t stream) {
  return rbf_kuf_image(X, ldx, Z, ldz, N, M, D, variance, lengthscales, n_ls, Kfr, kfr_bytes, stream, true);
}

static int64_t rbf_bwd_chunk(int64_t N) { return 4096; }

extern "C" size_t mgp_rbf_backward_workspace_bytes(int64_t N, int64_t M, int32_t D) {
  int dm = D <= 1 ? 1 : D <= 2 ? 2 : D <= 4 ? 4 : D <= 8 ? 8 : D <= 16 ? 16 : 32;
  const int64_t nch = (N + rbf_bwd_chunk(N) - 1) / rbf_bwd_chunk(N);
  return (size_t)((nch > 0 ? nch : 1) * (M > 0 ? M : 1) * (1 + 2 * dm)) * sizeof(double);
}

extern "C" int mgp_rbf_backward(const float* X, int64_t ldx, const float* Z, int64_t ldz, int64_t N, int64_t M,
                                int32_t D, const float* variance, const float* lengthscales, int32_t n_ls,
                                const float* gK, int64_t ldg, int32_t symmetric, int32_t accumulate, float* gZ,
                                int64_t ldgz, double* g_var, double* g_ls, void* workspace,
                                size_t workspace_bytes, mgp_stream_t stream) {
  if (!X) return -1;
  if (ldx < D) return -2;
  if (!Z) return -3;
  if (ldz < D) return -4;
  if (N < 0) return -5;
  if (M < 0) return -6;
  if (D < 1) return -7;
  if (D > 32) return MGP_ERR_UNSUPPORTED;
  if (!variance) return -8;
  if (!lengthscales) return -9;
  if (n_ls != 1 && n_ls != D) return -10;
  if (!gK) return -11;
  if (ldg < N) return -12;
  if (!gZ) return -15;
  if (ldgz < D) return -16;
  if (!g_var) return -17;
  if (!g_ls) return -18;
  if (M == 0) return MGP_OK;
  if (!workspace || workspace_bytes < mgp_rbf_backward_workspace_bytes(N, M, D)) return MGP_ERR_WORKSPACE;
  hipStream_t s = (hipStream_t)stream;
  const int64_t chunk = rbf_bwd_chunk(N);
  const int nch = (int)((N + chunk - 1) / chunk);
  double* part = (double*)workspace;
  const float zf = symmetric ? 2.f : 1.f;
  const dim3 grid((unsigned)((M + 4 * kRbfRows - 1) / (4 * kRbfRows)), (unsigned)(nch > 0 ? nch : 1));
#define MGP_RBF_BWD_CASE(DM)                                                                                  \
  if (D <= DM) {                                                                                              \
    const bool vec = DM >= 4 && ldx % 4 == 0 && ldx >= DM && aligned16(X);                                     \
    if (nch > 0 && vec)                                                                                       \
      hipLaunchKernelGGL((rbf_bwd_rows_kernel<DM, true>), grid, dim3(256), 0, s, X, ldx, Z, ldz, N, M, D,       \
                         variance, lengthscales, n_ls, gK, ldg, chunk, part);                                 \
    else if (nch > 0)                                                                                         \
      hipLaunchKernelGGL(rbf_bwd_rows_kernel<DM>, grid, dim3(256), 0, s, X, ldx, Z, ldz, N, M, D, variance,    \
                         lengthscales, n_ls, gK, ldg, chunk, part);                                           \
    else                                                                                                      \
      hipMemsetAsync(part, 0, mgp_rbf_backward_workspace_bytes(N, M, D), s);                                  \
    if (nch > 1)                                                                                              \
      hipLaunchKernelGGL(rbf_bwd_fold_kernel, dim3((unsigned)((M * (1 + 2 * DM) + 255) / 256)), dim3(256), 0, s, \
                         part, nch, M * (1 + 2 * DM));                                                        \
    hipLaunchKernelGGL(rbf_bwd_finish_kernel<DM>, dim3(1), dim3(256), 0, s, part, 1, M, D, variance,           \
                       lengthscales, n_ls, zf, accumulate, gZ, ldgz, g_var, g_ls);                            \
    return launch_status();                                                                                   \
  }
  MGP_RBF_BWD_CASE(1)
  MGP_RBF_BWD_CASE(2)
  MGP_RBF_BWD_CASE(4)
  MGP_RBF_BWD_CASE(8)
  MGP_RBF_BWD_CASE(16)
  MGP_RBF_BWD_CASE(32)
#undef MGP_RBF_BWD_CASE
  return MGP_ERR_UNSUPPORTED;
}

static int64_t rbf_bwd_batch_nch(int64_t N) {
  const int64_t c = rbf_bwd_chunk(N), n = (N + c - 1) / c;
  return n > 0 ? n : 1;
}

extern "C" size_t mgp_rbf_backward_batch_workspace_bytes(int64_t N, int64_t M, int32_t D) {
  int dm = D <= 1 ? 1 : D <= 2 ? 2 : D <= 4 ? 4 : D <= 8 ? 8 : D <= 16 ? 16 : 32;
  return (size_t)((rbf_bwd_batch_nch(N) + 1) * (M > 0 ? M : 1) * (1 + 2 * dm)) * sizeof(double);
}

extern "C" int mgp_rbf_backward_batch(int32_t batch, const float* X, int64_t ldx, int64_t N,
                                      const float* const* Z, int64_t ldz, int64_t M, int32_t D,
                                      const float* const* variance, const float* const* lengthscales, int32_t n_ls,
                                      const float* const* gKuf, int64_t ldgf, const float* const* gKuu, int64_t ldgu,
                                      int32_t accumulate, float* const* gZ, int64_t ldgz, double* const* g_var,
                                      double* const* g_ls, void* workspace, size_t workspace_bytes,
                                      mgp_stream_t stream) {
  if (batch < 1 || batch > kRbfMaxBatch) return -1;
  if (!X) return -2;
  if (ldx < D) return -3;
  if (N < 0) return -4;
  if (!Z) return -5;
  if (ldz < D) return -6;
  if (M < 0) return -7;
  if (D < 1) return -8;
  if (D > 32) return MGP_ERR_UNSUPPORTED;
  if (!variance) return -9;
  if (!lengthscales) return -10;
  if (n_ls != 1 && n_ls != D) return -11;
  if (!gKuf) return -12;
  if (ldgf < N) return -13;
  if (!gKuu) return -14;
  if (ldgu < M) return -15;
  if (!gZ) return -16;
  if (ldgz < D) return -17;
  if (!g_var) return -18;
  if (!g_ls) return -19;
  if (accumulate < 0 || accumulate > 2) return -20;
  RbfBwdLayers lay = {};
  for (int b = 0; b < batch; ++b) {
    if (!Z[b]) return -5;
    if (!variance[b]) return -9;
    if (!lengthscales[b]) return -10;
    if (!gKuf[b]) return -12;
    if (!gKuu[b]) return -14;
    if (!gZ[b]) return -16;
    if (!g_var[b]) return -18;
    if (!g_ls[b]) return -19;
    lay.Z[b] = Z[b], lay.var[b] = variance[b], lay.ls[b] = lengthscales[b], lay.gKuf[b] = gKuf[b];
    lay.gKuu[b] = gKuu[b], lay.gZ[b] = gZ[b], lay.g_var[b] = g_var[b], lay.g_ls[b] = g_ls[b];
  }
  if (M == 0) return MGP_OK;
  const size_t per = mgp_rbf_backward_batch_workspace_bytes(N, M, D);
  if (!workspace || workspace_bytes < (size_t)batch * per) return MGP_ERR_WORKSPACE;
  hipStream_t s = (hipStream_t)stream;
  const int64_t chunk = rbf_bwd_chunk(N), slab = (int64_t)(per / sizeof(double));
  const int nch = (int)rbf_bwd_batch_nch(N);
  double* ws = (double*)workspace;
  bool zvec = ldz % 4 == 0;
  for (int b = 0; b < batch; ++b) zvec = zvec && aligned16(Z[b]);
  const dim3 grid((unsigned)((M + 4 * kRbfRows - 1) / (4 * kRbfRows)), (unsigned)(nch + 1), (unsigned)batch);
  // the point loads' form only (dwordx4 or dword): the same values either way
#define MGP_RBF_BWDB_CASE(DM)                                                                                   \
  if (D <= DM) {                                                                                                \
    const bool vec = DM >= 4 && ldx % 4 == 0 && ldx >= DM && aligned16(X) && ldz >= DM && zvec;                  \
    if (vec)                                                                                                    \
      hipLaunchKernelGGL((rbf_bwd_rows_batch_kernel<DM, true>), grid, dim3(256), 0, s, X, ldx, N, ldz, M, D,      \
                         n_ls, lay, ldgf, ldgu, chunk, nch, slab, ws);                                          \
    else                                                                                                        \
      hipLaunchKernelGGL((rbf_bwd_rows_batch_kernel<DM, false>), grid, dim3(256), 0, s, X, ldx, N, ldz, M, D,     \
                         n_ls, lay, ldgf, ldgu, chunk, nch, slab, ws);                                          \
    if (nch > 1)                                                                                                \
      hipLaunchKernelGGL(rbf_bwd_fold_kernel, dim3((unsigned)((M * (1 + 2 * DM) + 255) / 256), (unsigned)batch),   \
                         dim3(256), 0, s, ws, nch, M * (1 + 2 * DM), slab);                                     \
    hipLaunchKernelGGL(rbf_bwd_finish_batch_kernel<DM>, dim3((unsigned)batch), dim3(256), 0, s, ws, slab, nch, M, \
                       D, n_ls, lay, accumulate, ldgz);                                                         \
    return launch_status();                                                                                     \
  }
  MGP_RBF_BWDB_CASE(1)
  MGP_RBF_BWDB_CASE(2)
  MGP_RBF_BWDB_CASE(4)
  MGP_RBF_BWDB_CASE(8)
  MGP_RBF_BWDB_CASE(16)
  MGP_RBF_BWDB_CASE(32)
#undef MGP_RBF_BWDB_CASE
  return MGP_ERR_UNSUPPORTED;
}
