// Optimizer side of the training step (utils/training_utils.py:4-28):
// the whitened-KL gradient and TF 2.10's Keras-legacy Adam
// on the unconstrained parameters.
//
// KL (models.py:79, GPflow gauss_kl whitened):
//   KL = 1/2 (sum q_mu^2 - M K - sum_k sum_m log L_k[m,m]^2 + sum_k |tril L_k|_F^2)
//   dKL/dq_mu = q_mu,  dKL/dL_k[i][j] = L_k[i][j] - [i == j] / L_k[i][i]   (i >= j)
// The ELBO carries -KL / num_data (models.py:79).
//
// Adam (Keras legacy OptimizerV2, eps outside the bias correction):
//   lr_t = lr sqrt(1 - b2^t) / (1 - b1^t);  m = b1 m + (1 - b1) g;  v = b2 v + (1 - b2) g^2
//   u -= lr_t m / (sqrt(v) + eps)
// applied to u = the unconstrained variable: the value itself, or
// softplus^-1 of a positive parameter (GPflow positive(): theta = softplus(u),
// d/du = sigmoid(u)), in which case theta is refreshed from u.
#include <math.h>

#include "mgp_common.hpp"

namespace mgp {

// g_q_mu[m][k] -= q_mu / nd  (rows x K);  g_L[k][i][j] -= (L - [i==j]/L_ii) / nd for j <= i.
__global__ __launch_bounds__(256) void kl_grad_kernel(const float* __restrict__ q_mu, int64_t ldq,
                                                      const float* __restrict__ q_sqrt, int64_t ldqs,
                                                      int64_t strideq, int64_t M, int K, float inv_nd,
                                                      float* __restrict__ g_q_mu, int64_t ldgq,
                                                      float* __restrict__ g_L, int64_t ldgl, int64_t strideg) {
  const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t nL = (int64_t)K * M * M;
  if (idx < nL) {
    const int k = (int)(idx / (M * M));
    const int64_t r = idx % (M * M), i = r / M, j = r % M;
    if (j <= i) {
      const float l = q_sqrt[k * strideq + i * ldqs + j];
      const float d = (i == j) ? l - 1.f / l : l;
      g_L[k * strideg + i * ldgl + j] -= d * inv_nd;
    }
  } else if (idx < nL + M * K) {
    const int64_t r = idx - nL, m = r / K, k = r % K;
    g_q_mu[m * ldgq + k] -= q_mu[m * ldq + k] * inv_nd;
  }
}

__device__ __forceinline__ float softplus_f(float u) { return u > 20.f ? u : log1pf(__expf(u)); }
__device__ __forceinline__ float sigmoid_f(float u) { return 1.f / (1.f + __expf(-u)); }

// One Adam step on a [rows][cols] (leading dimension ld) parameter block.
// g: gradient of the ELBO w.r.t. theta (constrained), scaled by gsign (-1:
// minimise -ELBO).  SOFTPLUS: u holds the unconstrained values, theta = softplus(u).
template <typename GT, bool SOFTPLUS>
__device__ __forceinline__ void adam_elem(float* __restrict__ theta, float* __restrict__ u,
                                          const GT* __restrict__ g, int64_t ldg, float* __restrict__ m1,
                                          float* __restrict__ m2, int64_t idx, int64_t cols, int64_t ld, float lr_t,
                                          float b1, float b2, float eps, float gsign);

template <typename GT, bool SOFTPLUS>
__global__ __launch_bounds__(256) void adam_kernel(float* __restrict__ theta, float* __restrict__ u,
                                                   const GT* __restrict__ g, int64_t ldg,
                                                   float* __restrict__ m1, float* __restrict__ m2, int64_t rows,
                                                   int64_t cols, int64_t ld, float lr_t, float b1, float b2,
                                                   float eps, float gsign) {
  const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (idx >= rows * cols) return;
  adam_elem<GT, SOFTPLUS>(theta, u, g, ldg, m1, m2, idx, cols, ld, lr_t, b1, b2, eps, gsign);
}

// Up to kAdamMaxSet parameter blocks in one launch: workgroup blockIdx.x belongs to
// block j with blk0[j] <= blockIdx.x < blk0[j + 1] and runs adam_kernel's element
// update on it (the same float operations, so the same bits as one launch per block).
constexpr int kAdamMaxSet = 16;
struct AdamSet {
  float* theta[kAdamMaxSet]; float* u[kAdamMaxSet]; const void* g[kAdamMaxSet];
  float* m1[kAdamMaxSet]; float* m2[kAdamMaxSet];
  int64_t rows[kAdamMaxSet], cols[kAdamMaxSet], ld[kAdamMaxSet], ldg[kAdamMaxSet];
  int64_t blk0[kAdamMaxSet + 1];
  int32_t dbl[kAdamMaxSet];
  int32_t n;
};

template <typename GT, bool SOFTPLUS>
__device__ __forceinline__ void adam_elem(float* __restrict__ theta, float* __restrict__ u,
                                          const GT* __restrict__ g, int64_t ldg, float* __restrict__ m1,
                                          float* __restrict__ m2, int64_t idx, int64_t cols, int64_t ld, float lr_t,
                                          float b1, float b2, float eps, float gsign) {
  const int64_t r = idx / cols, c = idx % cols;
  const int64_t p = r * ld + c;
  float gr = gsign * (float)g[r * ldg + c];
  float x = SOFTPLUS ? u[idx] : theta[p];
  if (SOFTPLUS) gr *= sigmoid_f(x);
  const float m = b1 * m1[idx] + (1.f - b1) * gr;
  const float v = b2 * m2[idx] + (1.f - b2) * gr * gr;
  m1[idx] = m;
  m2[idx] = v;
  x -= lr_t * m / (sqrtf(v) + eps);
  if (SOFTPLUS) {
    u[idx] = x;
    theta[p] = softplus_f(x);
  } else {
    theta[p] = x;
  }
}

__global__ __launch_bounds__(256) void adam_set_kernel(AdamSet a, float lr_t, float b1, float b2, float eps,
                                                       float gsign) {
  int j = 0;
  while (j + 1 < a.n && (int64_t)blockIdx.x >= a.blk0[j + 1]) ++j;
  const int64_t idx = ((int64_t)blockIdx.x - a.blk0[j]) * 256 + threadIdx.x;
  if (idx >= a.rows[j] * a.cols[j]) return;
  if (a.dbl[j]) {
    if (a.u[j]) adam_elem<double, true>(a.theta[j], a.u[j], (const double*)a.g[j], a.ldg[j], a.m1[j], a.m2[j], idx,
                                        a.cols[j], a.ld[j], lr_t, b1, b2, eps, gsign);
    else adam_elem<double, false>(a.theta[j], a.u[j], (const double*)a.g[j], a.ldg[j], a.m1[j], a.m2[j], idx,
                                  a.cols[j], a.ld[j], lr_t, b1, b2, eps, gsign);
  } else {
    if (a.u[j]) adam_elem<float, true>(a.theta[j], a.u[j], (const float*)a.g[j], a.ldg[j], a.m1[j], a.m2[j], idx,
                                       a.cols[j], a.ld[j], lr_t, b1, b2, eps, gsign);
    else adam_elem<float, false>(a.theta[j], a.u[j], (const float*)a.g[j], a.ldg[j], a.m1[j], a.m2[j], idx,
                                 a.cols[j], a.ld[j], lr_t, b1, b2, eps, gsign);
  }
}

}  // namespace mgp

using namespace mgp;

extern "C" int mgp_kl_grad(const float* q_mu, int64_t ldq, const float* q_sqrt, int64_t ldqs, int64_t strideq,
                           int64_t M, int32_t K, double num_data, float* g_q_mu, int64_t ldgq, float* g_q_sqrt,
                           int64_t ldgs, int64_t strideg, mgp_stream_t stream) {
  if (!q_mu) return -1;
  if (!q_sqrt) return -3;
  if (M < 0) return -6;
  if (K < 1) return -7;
  if (!(num_data > 0)) return -8;
  if (!g_q_mu) return -9;
  if (!g_q_sqrt) return -11;
  const int64_t n = (int64_t)K * M * M + M * K;
  if (n == 0) return MGP_OK;
  hipLaunchKernelGGL(kl_grad_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, q_mu,
                     ldq, q_sqrt, ldqs, strideq, M, K, (float)(1.0 / num_data), g_q_mu, ldgq, g_q_sqrt, ldgs,
                     strideg);
  return launch_status();
}

// grad_is_double: g is double (scalar hyper-parameters), else float.
extern "C" int mgp_adam_step(float* theta, float* u, const void* g, int32_t grad_is_double, int64_t ldg,
                             float* m1, float* m2, int64_t rows, int64_t cols, int64_t ld, float lr, float beta1,
                             float beta2, float eps, int64_t t, float grad_sign, mgp_stream_t stream) {
  if (!theta) return -1;
  if (!g) return -3;
  if (!m1) return -6;
  if (!m2) return -7;
  if (rows < 0) return -8;
  if (cols < 0) return -9;
  if (ld < cols) return -10;
  if (t < 1) return -15;
  if (rows * cols == 0) return MGP_OK;
  const double lr_t = (double)lr * sqrt(1.0 - pow((double)beta2, (double)t)) / (1.0 - pow((double)beta1, (double)t));
  const dim3 grid((unsigned)((rows * cols + 255) / 256));
  hipStream_t s = (hipStream_t)stream;
  if (grad_is_double) {
    if (u) hipLaunchKernelGGL((adam_kernel<double, true>), grid, dim3(256), 0, s, theta, u, (const double*)g, ldg, m1,
                              m2, rows, cols, ld, (float)lr_t, beta1, beta2, eps, grad_sign);
    else hipLaunchKernelGGL((adam_kernel<double, false>), grid, dim3(256), 0, s, theta, u, (const double*)g, ldg, m1,
                            m2, rows, cols, ld, (float)lr_t, beta1, beta2, eps, grad_sign);
  } else {
    if (u) hipLaunchKernelGGL((adam_kernel<float, true>), grid, dim3(256), 0, s, theta, u, (const float*)g, ldg, m1,
                              m2, rows, cols, ld, (float)lr_t, beta1, beta2, eps, grad_sign);
    else hipLaunchKernelGGL((adam_kernel<float, false>), grid, dim3(256), 0, s, theta, u, (const float*)g, ldg, m1,
                            m2, rows, cols, ld, (float)lr_t, beta1, beta2, eps, grad_sign);
  }
  return launch_status();
}

extern "C" int mgp_adam_step_set(int32_t n, float* const* theta, float* const* u, const void* const* g,
                                 const int32_t* grad_is_double, const int64_t* ldg, float* const* m1,
                                 float* const* m2, const int64_t* rows, const int64_t* cols, const int64_t* ld,
                                 float lr, float beta1, float beta2, float eps, int64_t t, float grad_sign,
                                 mgp_stream_t stream) {
  if (n < 1 || n > kAdamMaxSet) return -1;
  if (!theta) return -2;
  if (!u) return -3;
  if (!g) return -4;
  if (!grad_is_double) return -5;
  if (!ldg) return -6;
  if (!m1) return -7;
  if (!m2) return -8;
  if (!rows) return -9;
  if (!cols) return -10;
  if (!ld) return -11;
  if (t < 1) return -16;
  AdamSet a = {};
  a.n = n;
  int64_t blk = 0;
  for (int j = 0; j < n; ++j) {
    if (rows[j] < 0) return -9;
    if (cols[j] < 0) return -10;
    if (ld[j] < cols[j]) return -11;
    if (rows[j] * cols[j] > 0) {   // an empty block's pointers are not used (torch: NULL)
      if (!theta[j]) return -2;
      if (!g[j]) return -4;
      if (!m1[j]) return -7;
      if (!m2[j]) return -8;
    }
    a.theta[j] = theta[j], a.u[j] = u[j], a.g[j] = g[j], a.m1[j] = m1[j], a.m2[j] = m2[j];
    a.rows[j] = rows[j], a.cols[j] = cols[j], a.ld[j] = ld[j], a.ldg[j] = ldg[j], a.dbl[j] = grad_is_double[j];
    a.blk0[j] = blk;
    blk += (rows[j] * cols[j] + 255) / 256;
  }
  a.blk0[n] = blk;
  if (blk == 0) return MGP_OK;
  const double lr_t = (double)lr * sqrt(1.0 - pow((double)beta2, (double)t)) / (1.0 - pow((double)beta1, (double)t));
  hipLaunchKernelGGL(adam_set_kernel, dim3((unsigned)blk), dim3(256), 0, (hipStream_t)stream, a, (float)lr_t, beta1,
                     beta2, eps, grad_sign);
  return launch_status();
}
