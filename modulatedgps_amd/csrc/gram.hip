// Backward "gram" products: contractions over the data dimension N.
//
//   out[i][j] = alpha * sum_n X[i][n] Y[j][n]        (X: [MI][ldx], Y: [MJ][ldy], f32)
//
// used for the gradients that sum over data points (the GradientTape pass of
// GPflow base_conditional, MixtureGPs/models.py:141-143):
//   dL_k   = 2 tril(A diag(Gv_k) (L_k^T A)^T)   X = A, Y = CG_k         (q_sqrt)
//   dLm    = -tril(gKuf A^T)                     X = gKuf, Y = A          (Cholesky factor)
//   dq_mu  = A G_mu^T                            X = A, Y = G_mu          (q_mu)
//
// gfx950 mapping: 128 x 128 output tile per workgroup (4 waves of 64 x 64 =
// 2 x 2 tiles of v_mfma_f32_32x32x2_f32, exact f32), 16-deep n-chunks
// global -> registers -> LDS ([row][16 + 1] images, conflict-free column
// reads), double-buffered.  The n range is split over blockIdx.z (split-K) for
// parallelism; partial tiles go to a workspace and gram_reduce_kernel sums
// them in a fixed order (deterministic), applies alpha and the triangle.
// Roofline: f32 MFMA (2 MI MJ N flops, half for the triangular outputs).
#include "mgp_common.hpp"

namespace mgp {

constexpr int kGT = 128;   // output tile
constexpr int kGK = 16;    // n per chunk
constexpr int kGP = kGK + 1;

__device__ __forceinline__ floatx4 gload4(const float* __restrict__ p, int64_t ld, int64_t r, int64_t c,
                                          int64_t R, int64_t C) {
  if (r < R && c + 3 < C) return *reinterpret_cast<const floatx4*>(p + r * ld + c);
  floatx4 v = {0.f, 0.f, 0.f, 0.f};
  if (r < R) {
#pragma unroll
    for (int e = 0; e < 4; ++e)
      if (c + e < C) v[e] = p[r * ld + c + e];
  }
  return v;
}

// grid: x = tile pair (TRI: bj <= bi only), z = n split.
template <bool TRI>
__global__ __launch_bounds__(256) void gram_kernel(const float* __restrict__ X, int64_t ldx, int64_t MI,
                                                   const float* __restrict__ Y, int64_t ldy, int64_t MJ,
                                                   int64_t N, int64_t nper, int nbj, float* __restrict__ ws,
                                                   int64_t ldw, int64_t split_stride) {
  __shared__ float sx[2][kGT * kGP], sy[2][kGT * kGP];
  int bi, bj;
  if (TRI) {
    int q = blockIdx.x;
    bi = 0;
    while ((bi + 1) * (bi + 2) / 2 <= q) ++bi;
    bj = q - bi * (bi + 1) / 2;
  } else {
    bi = blockIdx.x / nbj;
    bj = blockIdx.x % nbj;
  }
  const int64_t i0 = (int64_t)bi * kGT, j0 = (int64_t)bj * kGT;
  const int64_t nb = (int64_t)blockIdx.z * nper;
  const int64_t ne = (nb + nper < N) ? nb + nper : N;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wi = (w >> 1) * 64, wj = (w & 1) * 64;
  floatx16 acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[a][b][e] = 0.f;
  // thread t loads rows t / 4 and t / 4 + 64, columns 4 (t % 4) .. + 3 of the chunk
  const int lr = tid >> 2, lc = (tid & 3) * 4;
  floatx4 rx[2], ry[2];
  auto load = [&](int64_t n0) {
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      rx[q] = gload4(X, ldx, i0 + lr + 64 * q, n0 + lc, MI, ne);
      ry[q] = gload4(Y, ldy, j0 + lr + 64 * q, n0 + lc, MJ, ne);
    }
  };
  auto store = [&](int buf) {
#pragma unroll
    for (int q = 0; q < 2; ++q)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        sx[buf][(lr + 64 * q) * kGP + lc + e] = rx[q][e];
        sy[buf][(lr + 64 * q) * kGP + lc + e] = ry[q][e];
      }
  };
  if (nb < ne) {
    load(nb);
    store(0);
    __syncthreads();
    int buf = 0;
    for (int64_t n0 = nb; n0 < ne; n0 += kGK) {
      const bool more = n0 + kGK < ne;
      if (more) load(n0 + kGK);
      const float* px = sx[buf];
      const float* py = sy[buf];
#pragma unroll
      for (int ks = 0; ks < kGK / 2; ++ks) {
        const int kk = 2 * ks + (lane >> 5);
        float a[2], b[2];
#pragma unroll
        for (int t2 = 0; t2 < 2; ++t2) {
          a[t2] = px[(wi + 32 * t2 + (lane & 31)) * kGP + kk];
          b[t2] = py[(wj + 32 * t2 + (lane & 31)) * kGP + kk];
        }
#pragma unroll
        for (int ta = 0; ta < 2; ++ta)
#pragma unroll
          for (int tb = 0; tb < 2; ++tb) acc[ta][tb] = mfma32x32x2(a[ta], b[tb], acc[ta][tb]);
      }
      if (more) store(buf ^ 1);
      __syncthreads();
      buf ^= 1;
    }
  }
  float* out = ws + (int64_t)blockIdx.z * split_stride;
#pragma unroll
  for (int ta = 0; ta < 2; ++ta)
#pragma unroll
    for (int tb = 0; tb < 2; ++tb) {
      const int64_t j = j0 + wj + 32 * tb + (lane & 31);
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int64_t i = i0 + wi + 32 * ta + acc_row(e, lane);
        if (i < MI && j < MJ) out[i * ldw + j] = acc[ta][tb][e];
      }
    }
}

// out[i][j] = alpha * sum_z ws[z][i][j]  (TRI: j <= i only, zero above).
__global__ __launch_bounds__(256) void gram_reduce_kernel(const float* __restrict__ ws, int64_t ldw,
                                                          int64_t split_stride, int nsplit, int64_t MI, int64_t MJ,
                                                          float alpha, int tri, float* __restrict__ out,
                                                          int64_t ldo) {
  const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (idx >= MI * MJ) return;
  const int64_t i = idx / MJ, j = idx % MJ;
  float v = 0.f;
  if (!tri || j <= i) {
    for (int z = 0; z < nsplit; ++z) v += ws[(int64_t)z * split_stride + i * ldw + j];
    v *= alpha;
  }
  out[i * ldo + j] = v;
}

}  // namespace mgp

using namespace mgp;

static int gram_splits(int64_t N, int tiles) {
  // aim for >= 1024 workgroups, each with >= 1024 points
  int s = 1;
  while ((int64_t)tiles * s < 1024 && N / (2 * s) >= 1024) s *= 2;
  return s;
}

extern "C" size_t mgp_gram_workspace_bytes(int64_t MI, int64_t MJ, int64_t N, int32_t tri) {
  if (MI <= 0 || MJ <= 0 || N <= 0) return 16;
  const int nbi = (int)((MI + kGT - 1) / kGT), nbj = (int)((MJ + kGT - 1) / kGT);
  const int tiles = tri ? nbi * (nbi + 1) / 2 : nbi * nbj;
  return (size_t)gram_splits(N, tiles) * (size_t)MI * (size_t)MJ * sizeof(float);
}

extern "C" int mgp_gram(const float* X, int64_t ldx, int64_t MI, const float* Y, int64_t ldy, int64_t MJ,
                        int64_t N, float alpha, int32_t tri, float* out, int64_t ldo, void* workspace,
                        size_t workspace_bytes, mgp_stream_t stream) {
  if (!X) return -1;
  if (ldx < N) return -2;
  if (MI < 0) return -3;
  if (!Y) return -4;
  if (ldy < N) return -5;
  if (MJ < 0) return -6;
  if (N < 0) return -7;
  if (tri && MI != MJ) return -9;
  if (!out) return -10;
  if (ldo < MJ) return -11;
  if (MI == 0 || MJ == 0) return MGP_OK;
  if (!workspace || workspace_bytes < mgp_gram_workspace_bytes(MI, MJ, N, tri)) return MGP_ERR_WORKSPACE;
  hipStream_t s = (hipStream_t)stream;
  const int nbi = (int)((MI + kGT - 1) / kGT), nbj = (int)((MJ + kGT - 1) / kGT);
  const int tiles = tri ? nbi * (nbi + 1) / 2 : nbi * nbj;
  const int nsplit = N > 0 ? gram_splits(N, tiles) : 1;
  int64_t nper = (N + nsplit - 1) / nsplit;
  nper = (nper + kGK - 1) / kGK * kGK;
  float* ws = (float*)workspace;
  const int64_t stride = MI * MJ;
  if (tri)
    hipLaunchKernelGGL(gram_kernel<true>, dim3(tiles, 1, nsplit), dim3(256), 0, s, X, ldx, MI, Y, ldy, MJ, N, nper,
                       nbj, ws, MJ, stride);
  else
    hipLaunchKernelGGL(gram_kernel<false>, dim3(tiles, 1, nsplit), dim3(256), 0, s, X, ldx, MI, Y, ldy, MJ, N,
                       nper, nbj, ws, MJ, stride);
  int st = launch_status();
  if (st) return st;
  hipLaunchKernelGGL(gram_reduce_kernel, dim3((unsigned)((MI * MJ + 255) / 256)), dim3(256), 0, s, ws, MJ, stride,
                     nsplit, MI, MJ, alpha, tri, out, ldo);
  return launch_status();
}
