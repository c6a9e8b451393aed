// One SMGP ELBO through the C-ABI of libmgp_hip.so alone (no torch, no Python):
// the split-f16 chain of INTEGRATION.md §2 on hipMalloc'd buffers, as a maintainer
// binding the library from another host language would call it.  Reads a binary
// problem file written by tests/test_gpu_c_abi.py and prints "elbo <value>".
//
// File layout (little endian): int64 N, M, K, D, S; float64 num_data; then float32
// X[N][D], Y[N], and per layer (pred, assign): Z[M][D], variance, lengthscale,
// q_mu[M][K], q_sqrt[K][M][M]; then lik_var[K], z[S][N][K], u[S][N][K].
#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "mgp_hip.h"

#define CHECK_HIP(x)                                                              \
  do {                                                                            \
    hipError_t e_ = (x);                                                          \
    if (e_ != hipSuccess) {                                                       \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      std::exit(2);                                                               \
    }                                                                             \
  } while (0)
#define CHECK_MGP(x)                                                                          \
  do {                                                                                        \
    int s_ = (x);                                                                             \
    if (s_ != MGP_OK) {                                                                       \
      std::fprintf(stderr, "%s:%d %s -> %d (%s)\n", __FILE__, __LINE__, #x, s_, mgp_status_string(s_)); \
      std::exit(3);                                                                           \
    }                                                                                         \
  } while (0)

namespace {

int64_t round4(int64_t x) { return (x + 3) / 4 * 4; }

template <typename T>
void read_into(std::FILE* f, std::vector<T>& v, size_t n) {
  v.resize(n);
  if (std::fread(v.data(), sizeof(T), n, f) != n) {
    std::fprintf(stderr, "short read\n");
    std::exit(4);
  }
}

// device copy of a host [rows][cols] float matrix with leading dimension ld
float* to_device(const float* h, int64_t rows, int64_t cols, int64_t ld, int64_t batch = 1) {
  float* d = nullptr;
  CHECK_HIP(hipMalloc(&d, sizeof(float) * batch * rows * ld));
  CHECK_HIP(hipMemset(d, 0, sizeof(float) * batch * rows * ld));
  CHECK_HIP(hipMemcpy2D(d, ld * sizeof(float), h, cols * sizeof(float), cols * sizeof(float), batch * rows,
                        hipMemcpyHostToDevice));
  return d;
}

void* dev_bytes(size_t n) {
  void* d = nullptr;
  CHECK_HIP(hipMalloc(&d, n < 16 ? 16 : n));
  return d;
}

}  // namespace

int main(int argc, char** argv) {
  // --batched: both layers' K4 and K5 through mgp_trsm_stats_f16_batch /
  // mgp_expert_conditional_f16_batch (per-layer images), else one call per layer;
  // --front: the SURVEY §8(b) names only (mgp_rbf_kuu_jitter, mgp_potrf_lower,
  // mgp_rbf_kuf, mgp_trsm_lln, mgp_expert_conditional, mgp_gauss_kl_white)
  const bool batched = argc == 3 && std::string(argv[2]) == "--batched";
  const bool front = argc == 3 && std::string(argv[2]) == "--front";
  if (argc != 2 && !batched && !front) {
    std::fprintf(stderr, "usage: %s problem.bin [--batched | --front]\n", argv[0]);
    return 1;
  }
  std::FILE* f = std::fopen(argv[1], "rb");
  if (!f) return 1;
  int64_t hdr[5];
  double num_data = 0;
  if (std::fread(hdr, sizeof(int64_t), 5, f) != 5 || std::fread(&num_data, sizeof(double), 1, f) != 1) return 4;
  const int64_t N = hdr[0], M = hdr[1], D = hdr[3];
  const int32_t K = (int32_t)hdr[2], S = (int32_t)hdr[4];
  std::vector<float> X, Y, lik, z, u;
  read_into(f, X, N * D);
  read_into(f, Y, N);
  std::vector<float> Zh[2], var[2], ls[2], qmu[2], qs[2];
  for (int l = 0; l < 2; ++l) {
    read_into(f, Zh[l], M * D);
    read_into(f, var[l], 1);
    read_into(f, ls[l], 1);
    read_into(f, qmu[l], M * K);
    read_into(f, qs[l], (size_t)K * M * M);
  }
  read_into(f, lik, K);
  read_into(f, z, (size_t)S * N * K);
  read_into(f, u, (size_t)S * N * K);
  std::fclose(f);

  hipStream_t s;
  CHECK_HIP(hipStreamCreate(&s));
  const int64_t ldm = round4(M), ldn = round4(N);
  float* dX = to_device(X.data(), N, D, D);
  float* dY = to_device(Y.data(), 1, N, N);
  float* dlik = to_device(lik.data(), 1, K, K);
  float* dz = to_device(z.data(), 1, (int64_t)S * N * K, (int64_t)S * N * K);
  float* du = to_device(u.data(), 1, (int64_t)S * N * K, (int64_t)S * N * K);
  float *dZ[2], *dvar[2], *dls[2], *dqmu[2], *dqs[2];
  for (int l = 0; l < 2; ++l) {
    dZ[l] = to_device(Zh[l].data(), M, D, D);
    dvar[l] = to_device(var[l].data(), 1, 1, 1);
    dls[l] = to_device(ls[l].data(), 1, 1, 1);
    dqmu[l] = to_device(qmu[l].data(), M, K, K);
    dqs[l] = to_device(qs[l].data(), M, M, ldm, K);  // [K][M][ldm]
  }

  float* LinvT = (float*)dev_bytes(sizeof(float) * 2 * M * ldm);
  int32_t* info = (int32_t*)dev_bytes(2 * sizeof(int32_t));
  float *fmean[2], *fvar[2];
  double* kl = (double*)dev_bytes(2 * sizeof(double));
  if (front) {
    size_t wsb = 0;
    for (int32_t op : {MGP_OP_POTRF_LOWER, MGP_OP_TRSM_LLN, MGP_OP_EXPERT_CONDITIONAL, MGP_OP_GAUSS_KL_WHITE})
      wsb = std::max(wsb, mgp_workspace_bytes(op, M, N, K));
    void* ws = dev_bytes(wsb);
    float* Kuu = (float*)dev_bytes(sizeof(float) * M * ldm);
    float* A = (float*)dev_bytes(sizeof(float) * M * ldn);
    for (int l = 0; l < 2; ++l) {
      fmean[l] = (float*)dev_bytes(sizeof(float) * K * ldn);
      fvar[l] = (float*)dev_bytes(sizeof(float) * K * ldn);
      float* lt = LinvT + l * M * ldm;
      CHECK_MGP(mgp_rbf_kuu_jitter(dZ[l], D, M, (int32_t)D, dvar[l], dls[l], 1, 1e-6f, Kuu, ldm, s));
      CHECK_MGP(mgp_potrf_lower(Kuu, ldm, M, lt, ldm, info + l, ws, wsb, s));
      CHECK_MGP(mgp_rbf_kuf(dX, D, dZ[l], D, N, M, (int32_t)D, dvar[l], dls[l], 1, A, ldn, s));
      CHECK_MGP(mgp_trsm_lln(lt, ldm, M, A, ldn, N, ws, wsb, s));
      CHECK_MGP(mgp_expert_conditional(A, ldn, dqmu[l], K, dqs[l], ldm, M * ldm, dvar[l], M, N, K, fmean[l], fvar[l],
                                       ldn, ws, wsb, s));
      CHECK_MGP(mgp_gauss_kl_white(dqmu[l], K, dqs[l], ldm, M * ldm, M, K, kl + l, ws, wsb, s));
    }
  } else {
  // K2 + K3: Kuu of both layers (float64) and its Cholesky + inverse in one batched sweep
  const size_t cwb = mgp_chol_workspace_bytes(M, 2);
  void* cws = dev_bytes(cwb);
  const float* Zs[2] = {dZ[0], dZ[1]};
  const float* vs[2] = {dvar[0], dvar[1]};
  const float* lss[2] = {dls[0], dls[1]};
  const int32_t nls[2] = {1, 1};
  CHECK_MGP(mgp_kuu_potrf_trtri(Zs, D, M, (int32_t)D, vs, lss, nls, 1e-6f, 2, nullptr, LinvT, ldm, M * ldm, info, cws,
                                cwb, s));

  // K1, K4, K5 (split-f16 images) and K7 per layer
  const size_t colb = mgp_x6_cols_bytes(M, N), lowb = mgp_x6_lower_bytes(M, K), tb = mgp_x6_lower_bytes(M, 1);
  const int T = mgp_stats_tiles(M);
  const size_t xwb = mgp_expert_x6_workspace_bytes(M, N, K);
  const size_t kwb = mgp_kl_workspace_bytes(M, K);
  void* kws = dev_bytes(kwb);
  void *Kfr[2], *Afr[2], *Tfr[2], *Lfr[2], *xws[2];
  float* stats[2];
  for (int l = 0; l < 2; ++l) {
    Kfr[l] = dev_bytes(colb);
    Afr[l] = dev_bytes(colb);
    Tfr[l] = dev_bytes(tb);
    Lfr[l] = dev_bytes(lowb);
    stats[l] = (float*)dev_bytes(sizeof(float) * T * (K + 1) * ldn);
    xws[l] = dev_bytes(xwb);
    fmean[l] = (float*)dev_bytes(sizeof(float) * K * ldn);
    fvar[l] = (float*)dev_bytes(sizeof(float) * K * ldn);
    CHECK_MGP(mgp_rbf_kuf_f16(dX, D, dZ[l], D, N, M, (int32_t)D, dvar[l], dls[l], 1, Kfr[l], colb, s));
    CHECK_MGP(mgp_split_upper_f16(LinvT + l * M * ldm, ldm, M, Tfr[l], tb, s));
    CHECK_MGP(mgp_split_lower_f16(dqs[l], ldm, M * ldm, M, K, Lfr[l], lowb, s));
    if (!batched) {
      CHECK_MGP(mgp_trsm_stats_f16(Tfr[l], tb, Kfr[l], colb, M, N, dqmu[l], K, K, dvar[l], Afr[l], colb, stats[l], ldn,
                                   nullptr, N, s));
      CHECK_MGP(mgp_expert_conditional_f16(Afr[l], colb, Lfr[l], lowb, stats[l], ldn, dvar[l], M, N, K, fmean[l],
                                           fvar[l], ldn, xws[l], xwb, s));
    }
    CHECK_MGP(mgp_gauss_kl_white(dqmu[l], K, dqs[l], ldm, M * ldm, M, K, kl + l, kws, kwb, s));
  }
  if (batched) {
    const void* cT[2] = {Tfr[0], Tfr[1]};
    const void* cK[2] = {Kfr[0], Kfr[1]};
    const void* cA[2] = {Afr[0], Afr[1]};
    const void* cL[2] = {Lfr[0], Lfr[1]};
    const float* q[2] = {dqmu[0], dqmu[1]};
    const float* v[2] = {dvar[0], dvar[1]};
    const float* st[2] = {stats[0], stats[1]};
    CHECK_MGP(mgp_trsm_stats_f16_batch(2, cT, tb, cK, colb, M, N, q, K, K, v, Afr, colb, stats, ldn, nullptr, N, s));
    CHECK_MGP(mgp_expert_conditional_f16_batch(2, cA, colb, cL, lowb, st, ldn, v, M, N, K, fmean, fvar, ldn, xws, xwb,
                                               nullptr, 0, nullptr, s));
  }

  }   // (fused chain)

  // K6 with the explicit noise, then the scalar ELBO
  const size_t ewb = mgp_elbo_workspace_bytes(N);
  void* ews = dev_bytes(ewb);
  double* data_sum = (double*)dev_bytes(sizeof(double));
  float* elbo = (float*)dev_bytes(sizeof(float));
  double* elbo64 = (double*)dev_bytes(sizeof(double));
  CHECK_MGP(mgp_elbo_terms(fmean[0], fvar[0], fmean[1], fvar[1], ldn, dY, dlik, N, K, S, 0.01f, 1e-6f, dz, du, 0, 0,
                           data_sum, ews, ewb, s));
  CHECK_MGP(mgp_elbo_combine(data_sum, kl, kl + 1, (double)N, num_data, elbo, elbo64, s));
  CHECK_HIP(hipStreamSynchronize(s));
  int32_t hinfo[2];
  double h64 = 0;
  CHECK_HIP(hipMemcpy(hinfo, info, sizeof(hinfo), hipMemcpyDeviceToHost));
  CHECK_HIP(hipMemcpy(&h64, elbo64, sizeof(double), hipMemcpyDeviceToHost));
  std::printf("info %d %d\nelbo %.10g\n", hinfo[0], hinfo[1], h64);
  return (hinfo[0] == 0 && hinfo[1] == 0) ? 0 : 5;
}
