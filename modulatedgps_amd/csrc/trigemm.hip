// K4 / K5: the two triangular f32 GEMMs of the whitened SVGP conditional.
//
// Reference: GPflow 2.7 base_conditional(..., white=True, full_cov=False) with
// 3-D q_sqrt, reached from MixtureGPs/models.py:141-143:
//     A    = triangular_solve(Lm, Kmn)               [S, M, N] in the reference
//     fvar = Knn - sum_m A^2 ;  fmean = A^T q_mu
//     LTA  = matmul(band_part(q_sqrt), A_tiled, transpose_a=True)   [S, K, M, N]
//     fvar = fvar + sum_m LTA^2
// The reference materialises A and LTA for S identical copies of X
// (models.py:35-36).  Here S is gone (the conditional is S-invariant) and:
//   K4  A = (LinvT)^T Kuf          -- LOWER triangular GEMM, A written once,
//       epilogue: per-row-tile column sums of A^2 and A q_mu (stats partials)
//   K5  C_k = L_k^T A              -- UPPER triangular GEMM per expert k,
//       epilogue: sum of squares over rows; C_k is never written.  One
//       workgroup owns (expert k, n-tile) and walks every row tile, so the
//       result is final (no cross-workgroup reduction, no atomics).
//
// Both are C[i, n] = sum_k T[k][i] * B[k][n] with T row-major [k][i]
// (K4: T = LinvT, nonzero k <= i; K5: T = L_k, nonzero k >= i), B [k][n].
// Tiling for gfx950: 256 threads = 4 waves in a 2x2 grid, workgroup tile
// BM x BN (256x256 or 128x128), wave tile (BM/2)x(BN/2) of 32x32 accumulators
// on v_mfma_f32_32x32x2_f32 (exact f32).  K-chunks of 16 rows of T and B are
// staged global -> registers -> LDS, double buffered with one barrier per
// chunk; row tiles of 32 that lie entirely in the zero triangle of a chunk are
// skipped (wave-uniform branch), so the triangular half is never multiplied.
// Roofline: f32 MFMA bound (K4: M^2 N flops, K5: K M^2 N flops at c3:
// 68.7 / 549.8 GFLOP vs 157.3 TFLOP/s).
#include "mgp_common.hpp"

namespace mgp {

constexpr int kTgThreads = 256;
constexpr int kTgBK = 16;

constexpr int tg_rt(int BM) { return BM / 64; }
constexpr int tg_t4(int BM) { return kTgBK * BM / 4 / kTgThreads; }

template <int BM, int BN>
struct TgTile {
  static constexpr int WM = BM / 2, WN = BN / 2;   // wave tile
  static constexpr int RT = WM / 32, CT = WN / 32; // 32x32 accumulators per wave
  static constexpr int T4 = kTgBK * BM / 4 / kTgThreads;  // float4 of T per thread per chunk
  static constexpr int B4 = kTgBK * BN / 4 / kTgThreads;
  static constexpr int LDS_FLOATS = 2 * kTgBK * (BM + BN);
};

// Stage one K-chunk (rows k0..k0+15) of T[:, i0:i0+BM] and B[:, n0:n0+BN] into
// registers, zero-filling out-of-range and out-of-triangle elements.
template <int BM, int BN, bool UPPER>
__device__ __forceinline__ void tg_load_chunk(floatx4 (&rt)[tg_t4(BM)],
                                              floatx4 (&rb)[tg_t4(BN)],
                                              const float* __restrict__ T, int64_t ldt,
                                              const float* __restrict__ B, int64_t ldb, int64_t M,
                                              int64_t N, int64_t i0, int64_t n0, int64_t k0) {
  using TT = TgTile<BM, BN>;
  const int t = threadIdx.x;
#pragma unroll
  for (int q = 0; q < TT::T4; ++q) {
    const int idx = t + kTgThreads * q;
    const int r = idx / (BM / 4), c = (idx % (BM / 4)) * 4;
    const int64_t k = k0 + r, i = i0 + c;
    floatx4 v = load4_guarded(T, ldt, k, i, M, M);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const bool keep = UPPER ? (k >= i + e) : (k <= i + e);
      if (!keep) v[e] = 0.f;
    }
    rt[q] = v;
  }
#pragma unroll
  for (int q = 0; q < TT::B4; ++q) {
    const int idx = t + kTgThreads * q;
    const int r = idx / (BN / 4), c = (idx % (BN / 4)) * 4;
    rb[q] = load4_guarded(B, ldb, k0 + r, n0 + c, M, N);
  }
}

template <int BM, int BN>
__device__ __forceinline__ void tg_store_chunk(float* __restrict__ sT, float* __restrict__ sB,
                                               const floatx4 (&rt)[tg_t4(BM)],
                                               const floatx4 (&rb)[tg_t4(BN)]) {
  using TT = TgTile<BM, BN>;
  const int t = threadIdx.x;
#pragma unroll
  for (int q = 0; q < TT::T4; ++q) {
    const int idx = t + kTgThreads * q;
    *reinterpret_cast<floatx4*>(sT + idx * 4) = rt[q];  // row-major [16][BM], linear
  }
#pragma unroll
  for (int q = 0; q < TT::B4; ++q) {
    const int idx = t + kTgThreads * q;
    *reinterpret_cast<floatx4*>(sB + idx * 4) = rb[q];
  }
}

// acc[RT][CT] = sum over k in [kbeg, kend) of T[k][i0 + .] B[k][n0 + .] for this
// wave's quadrant.  `lds` holds two [16][BM] + [16][BN] buffers.
template <int BM, int BN, bool UPPER>
__device__ __forceinline__ void tg_mainloop(floatx16 (&acc)[tg_rt(BM)][tg_rt(BN)],
                                            float* __restrict__ lds, const float* __restrict__ T,
                                            int64_t ldt, const float* __restrict__ B, int64_t ldb,
                                            int64_t M, int64_t N, int64_t i0, int64_t n0,
                                            int64_t kbeg, int64_t kend) {
  using TT = TgTile<BM, BN>;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int wr = w >> 1, wc = w & 1;
  const int h = lane >> 5, l32 = lane & 31;
#pragma unroll
  for (int r = 0; r < TT::RT; ++r)
#pragma unroll
    for (int c = 0; c < TT::CT; ++c)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[r][c][e] = 0.f;
  if (kend <= kbeg) return;
  const int nchunks = (int)((kend - kbeg + kTgBK - 1) / kTgBK);
  floatx4 rt[TT::T4], rb[TT::B4];
  tg_load_chunk<BM, BN, UPPER>(rt, rb, T, ldt, B, ldb, M, N, i0, n0, kbeg);
  tg_store_chunk<BM, BN>(lds, lds + kTgBK * BM, rt, rb);
  __syncthreads();
  // wave-uniform row-tile starts (global row index of the first row)
  int64_t rowbase[TT::RT];
#pragma unroll
  for (int r = 0; r < TT::RT; ++r) rowbase[r] = i0 + wr * TT::WM + 32 * r;
  bool colok[TT::CT];
#pragma unroll
  for (int c = 0; c < TT::CT; ++c) colok[c] = (n0 + wc * TT::WN + 32 * c) < N;

  for (int ch = 0; ch < nchunks; ++ch) {
    const int64_t k0 = kbeg + (int64_t)ch * kTgBK;
    float* sT = lds + (ch & 1) * kTgBK * (BM + BN);
    float* sB = sT + kTgBK * BM;
    if (ch + 1 < nchunks) tg_load_chunk<BM, BN, UPPER>(rt, rb, T, ldt, B, ldb, M, N, i0, n0, k0 + kTgBK);
    bool rowok[TT::RT];
#pragma unroll
    for (int r = 0; r < TT::RT; ++r) {
      const bool tri = UPPER ? (k0 + kTgBK - 1 >= rowbase[r]) : (k0 <= rowbase[r] + 31);
      rowok[r] = tri && rowbase[r] < M;
    }
#pragma unroll
    for (int ks = 0; ks < kTgBK / 2; ++ks) {
      const int kl = 2 * ks + h;
      float a[TT::RT], b[TT::CT];
#pragma unroll
      for (int r = 0; r < TT::RT; ++r) a[r] = sT[kl * BM + wr * TT::WM + 32 * r + l32];
#pragma unroll
      for (int c = 0; c < TT::CT; ++c) b[c] = sB[kl * BN + wc * TT::WN + 32 * c + l32];
#pragma unroll
      for (int r = 0; r < TT::RT; ++r) {
        if (!rowok[r]) continue;
#pragma unroll
        for (int c = 0; c < TT::CT; ++c) {
          if (!colok[c]) continue;
          acc[r][c] = mfma32x32x2(a[r], b[c], acc[r][c]);
        }
      }
    }
    if (ch + 1 < nchunks) {
      float* nT = lds + ((ch + 1) & 1) * kTgBK * (BM + BN);
      tg_store_chunk<BM, BN>(nT, nT + kTgBK * BM, rt, rb);
    }
    __syncthreads();
  }
}

// ------------------------------------------------------------------ K4
// grid.x = nTiles_m * nTiles_n; heavy (large i0) row tiles first.
template <int BM, int BN, int KMAX>
__global__ __launch_bounds__(kTgThreads, 1) void trsm_stats_kernel(
    const float* __restrict__ LinvT, int64_t ldl, const float* __restrict__ Kuf, int64_t ldk,
    int64_t M, int64_t N, const float* __restrict__ q_mu, int64_t ldq, int K,
    float* __restrict__ A, int64_t lda, float* __restrict__ stats, int64_t lds_) {
  using TT = TgTile<BM, BN>;
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int nTm = (int)((M + BM - 1) / BM), nTn = (int)((N + BN - 1) / BN);
  const int tm = nTm - 1 - (int)(blockIdx.x / nTn);
  const int tn = (int)(blockIdx.x % nTn);
  const int64_t i0 = (int64_t)tm * BM, n0 = (int64_t)tn * BN;
  const int64_t kend = (i0 + BM < M) ? i0 + BM : M;
  floatx16 acc[TT::RT][TT::CT];
  tg_mainloop<BM, BN, false>(acc, lds, LinvT, ldl, Kuf, ldk, M, N, i0, n0, 0, kend);

  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int wr = w >> 1, wc = w & 1, l32 = lane & 31;
  // ---- write A
#pragma unroll
  for (int r = 0; r < TT::RT; ++r)
#pragma unroll
    for (int c = 0; c < TT::CT; ++c) {
      const int64_t col = n0 + wc * TT::WN + 32 * c + l32;
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int64_t row = i0 + wr * TT::WM + 32 * r + acc_row(e, lane);
        if (row < M && col < N) A[row * lda + col] = acc[r][c][e];
      }
    }
  // ---- stats: stage q_mu rows of this tile (zero beyond M / K)
  float* sQ = lds;                       // [BM][KMAX]
  float* sRed = lds + BM * KMAX;         // [2][KMAX + 1][BN]
  for (int idx = threadIdx.x; idx < BM * KMAX; idx += kTgThreads) {
    const int r = idx / KMAX, kk = idx % KMAX;
    sQ[idx] = (i0 + r < M && kk < K) ? q_mu[(i0 + r) * ldq + kk] : 0.f;
  }
  __syncthreads();
  float sq[TT::CT], qm[TT::CT][KMAX];
#pragma unroll
  for (int c = 0; c < TT::CT; ++c) {
    sq[c] = 0.f;
#pragma unroll
    for (int kk = 0; kk < KMAX; ++kk) qm[c][kk] = 0.f;
  }
#pragma unroll
  for (int r = 0; r < TT::RT; ++r)
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const int lr = wr * TT::WM + 32 * r + acc_row(e, lane);
      float q[KMAX];
#pragma unroll
      for (int kk = 0; kk < KMAX; ++kk) q[kk] = sQ[lr * KMAX + kk];
#pragma unroll
      for (int c = 0; c < TT::CT; ++c) {
        const float v = acc[r][c][e];
        sq[c] = fmaf(v, v, sq[c]);
#pragma unroll
        for (int kk = 0; kk < KMAX; ++kk) qm[c][kk] = fmaf(v, q[kk], qm[c][kk]);
      }
    }
  // combine the two lane halves (rows 4h..), then the two row-waves via LDS
#pragma unroll
  for (int c = 0; c < TT::CT; ++c) {
    sq[c] += __shfl_xor(sq[c], 32, 64);
#pragma unroll
    for (int kk = 0; kk < KMAX; ++kk) qm[c][kk] += __shfl_xor(qm[c][kk], 32, 64);
  }
  if (lane < 32) {
#pragma unroll
    for (int c = 0; c < TT::CT; ++c) {
      const int lc = wc * TT::WN + 32 * c + l32;
      sRed[(wr * (KMAX + 1) + 0) * BN + lc] = sq[c];
#pragma unroll
      for (int kk = 0; kk < KMAX; ++kk) sRed[(wr * (KMAX + 1) + 1 + kk) * BN + lc] = qm[c][kk];
    }
  }
  __syncthreads();
  float* st = stats + (int64_t)tm * (K + 1) * lds_;
  for (int idx = threadIdx.x; idx < (K + 1) * BN; idx += kTgThreads) {
    const int row = idx / BN, lc = idx % BN;
    const int64_t n = n0 + lc;
    if (n < N) st[row * lds_ + n] = sRed[row * BN + lc] + sRed[((KMAX + 1) + row) * BN + lc];
  }
}

// ------------------------------------------------------------------ K5
// grid.x = K * nTiles_n, block b -> (expert k = b / nTn, n-tile = b % nTn):
// the K experts of one n-tile share an XCD group (b % 8) when nTn % 8 == 0.
template <int BM, int BN>
__global__ __launch_bounds__(kTgThreads, 1) void expert_cond_kernel(
    const float* __restrict__ Amat, int64_t lda, const float* __restrict__ q_sqrt, int64_t ldqs,
    int64_t strideq, const float* __restrict__ stats, int64_t lds_, int nTs,
    const float* __restrict__ variance, int64_t M, int64_t N, int K, float* __restrict__ fmean,
    float* __restrict__ fvar, int64_t ldf) {
  using TT = TgTile<BM, BN>;
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int nTn = (int)((N + BN - 1) / BN), nTm = (int)((M + BM - 1) / BM);
  const int k = (int)(blockIdx.x / nTn);
  const int tn = (int)(blockIdx.x % nTn);
  const int64_t n0 = (int64_t)tn * BN;
  const float* Lk = q_sqrt + (int64_t)k * strideq;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int wr = w >> 1, wc = w & 1, l32 = lane & 31;
  float colsq[TT::CT];
#pragma unroll
  for (int c = 0; c < TT::CT; ++c) colsq[c] = 0.f;
  for (int tm = 0; tm < nTm; ++tm) {
    const int64_t i0 = (int64_t)tm * BM;
    floatx16 acc[TT::RT][TT::CT];
    tg_mainloop<BM, BN, true>(acc, lds, Lk, ldqs, Amat, lda, M, N, i0, n0, i0, M);
#pragma unroll
    for (int r = 0; r < TT::RT; ++r)
#pragma unroll
      for (int c = 0; c < TT::CT; ++c)
#pragma unroll
        for (int e = 0; e < 16; ++e) colsq[c] = fmaf(acc[r][c][e], acc[r][c][e], colsq[c]);
  }
#pragma unroll
  for (int c = 0; c < TT::CT; ++c) colsq[c] += __shfl_xor(colsq[c], 32, 64);
  float* sRed = lds;  // [2][BN]
  if (lane < 32) {
#pragma unroll
    for (int c = 0; c < TT::CT; ++c) sRed[wr * BN + wc * TT::WN + 32 * c + l32] = colsq[c];
  }
  __syncthreads();
  const float var = variance[0];
  for (int lc = threadIdx.x; lc < BN; lc += kTgThreads) {
    const int64_t n = n0 + lc;
    if (n >= N) continue;
    float a2 = 0.f, fm = 0.f;
    for (int t = 0; t < nTs; ++t) {
      const float* st = stats + (int64_t)t * (K + 1) * lds_;
      a2 += st[n];
      fm += st[(int64_t)(1 + k) * lds_ + n];
    }
    fmean[(int64_t)k * ldf + n] = fm;
    fvar[(int64_t)k * ldf + n] = (var - a2) + (sRed[lc] + sRed[BN + lc]);
  }
}

// ------------------------------------------------------------------ launchers
static inline bool use_big_tiles(int64_t M, int64_t N) { return N >= 256 * 64 && M >= 256; }

}  // namespace mgp

using namespace mgp;

static constexpr int kStatsTile = 256;  // K4 row tile for big problems (T = ceil(M/256))

extern "C" int mgp_stats_tiles(int64_t M) {
  // Row tiles used by mgp_trsm_stats.  The big-tile path uses 256, the small one
  // 128; report the finer count so callers can size for both.
  return (int)((M + 127) / 128);
}

template <int BM, int KMAX>
static int launch_trsm(const float* LinvT, int64_t ldl, const float* Kuf, int64_t ldk, int64_t M,
                       int64_t N, const float* q_mu, int64_t ldq, int K, float* A, int64_t lda,
                       float* stats, int64_t lds, hipStream_t s) {
  const int nTm = (int)((M + BM - 1) / BM), nTn = (int)((N + BM - 1) / BM);
  const size_t shm = (size_t)TgTile<BM, BM>::LDS_FLOATS * sizeof(float);
  const size_t shm2 = (size_t)(BM * KMAX + 2 * (KMAX + 1) * BM) * sizeof(float);
  hipLaunchKernelGGL((trsm_stats_kernel<BM, BM, KMAX>), dim3(nTm * nTn), dim3(kTgThreads),
                     shm > shm2 ? shm : shm2, s, LinvT, ldl, Kuf, ldk, M, N, q_mu, ldq, K, A, lda,
                     stats, lds);
  return launch_status();
}

template <int BM>
static int dispatch_trsm(const float* LinvT, int64_t ldl, const float* Kuf, int64_t ldk, int64_t M,
                         int64_t N, const float* q_mu, int64_t ldq, int K, float* A, int64_t lda,
                         float* stats, int64_t lds, hipStream_t s) {
  if (K <= 4) return launch_trsm<BM, 4>(LinvT, ldl, Kuf, ldk, M, N, q_mu, ldq, K, A, lda, stats, lds, s);
  if (K <= 8) return launch_trsm<BM, 8>(LinvT, ldl, Kuf, ldk, M, N, q_mu, ldq, K, A, lda, stats, lds, s);
  if (K <= 16) return launch_trsm<BM, 16>(LinvT, ldl, Kuf, ldk, M, N, q_mu, ldq, K, A, lda, stats, lds, s);
  return MGP_ERR_UNSUPPORTED;
}

extern "C" int mgp_trsm_stats(const float* LinvT, int64_t ldl, const float* Kuf, int64_t ldk,
                              int64_t M, int64_t N, const float* q_mu, int64_t ldq, int32_t K,
                              float* A, int64_t lda, float* stats, int64_t lds,
                              mgp_stream_t stream) {
  if (!LinvT) return -1;
  if (ldl < M) return -2;
  if (!Kuf) return -3;
  if (ldk < N) return -4;
  if (M < 0) return -5;
  if (N < 0) return -6;
  if (!q_mu) return -7;
  if (ldq < K) return -8;
  if (K < 1) return -9;
  if (K > 16) return MGP_ERR_UNSUPPORTED;
  if (!A) return -10;
  if (lda < N) return -11;
  if (!stats) return -12;
  if (lds < N) return -13;
  if (ldl % 4 || ldk % 4 || lda % 4 || lds % 4) return MGP_ERR_ALIGN;
  if (!aligned16(LinvT) || !aligned16(Kuf) || !aligned16(A) || !aligned16(stats)) return MGP_ERR_ALIGN;
  if (M == 0 || N == 0) return MGP_OK;
  hipStream_t s = (hipStream_t)stream;
  // The stats tiling must match mgp_expert_conditional: it is encoded by the
  // row tile, which both sides derive from the same use_big_tiles(M, N).
  if (use_big_tiles(M, N)) return dispatch_trsm<256>(LinvT, ldl, Kuf, ldk, M, N, q_mu, ldq, K, A, lda, stats, lds, s);
  return dispatch_trsm<128>(LinvT, ldl, Kuf, ldk, M, N, q_mu, ldq, K, A, lda, stats, lds, s);
}

extern "C" int mgp_expert_conditional(const float* A, int64_t lda, const float* q_sqrt, int64_t ldqs,
                                      int64_t strideq, const float* stats, int64_t lds,
                                      const float* variance, int64_t M, int64_t N, int32_t K,
                                      float* fmean, float* fvar, int64_t ldf, mgp_stream_t stream) {
  if (!A) return -1;
  if (lda < N) return -2;
  if (!q_sqrt) return -3;
  if (ldqs < M) return -4;
  if (K > 1 && strideq < ldqs * M) return -5;
  if (!stats) return -6;
  if (lds < N) return -7;
  if (!variance) return -8;
  if (M < 0) return -9;
  if (N < 0) return -10;
  if (K < 1) return -11;
  if (!fmean) return -12;
  if (!fvar) return -13;
  if (ldf < N) return -14;
  if (lda % 4 || ldqs % 4 || lds % 4) return MGP_ERR_ALIGN;
  if (!aligned16(A) || !aligned16(q_sqrt) || (strideq % 4)) return MGP_ERR_ALIGN;
  if (N == 0) return MGP_OK;
  hipStream_t s = (hipStream_t)stream;
  if (use_big_tiles(M, N)) {
    const int nTn = (int)((N + 255) / 256), nTs = (int)((M + 255) / 256);
    const size_t shm = (size_t)TgTile<256, 256>::LDS_FLOATS * sizeof(float);
    hipLaunchKernelGGL((expert_cond_kernel<256, 256>), dim3(K * nTn), dim3(kTgThreads), shm, s, A,
                       lda, q_sqrt, ldqs, strideq, stats, lds, nTs, variance, M, N, K, fmean, fvar, ldf);
  } else {
    const int nTn = (int)((N + 127) / 128), nTs = (int)((M + 127) / 128);
    const size_t shm = (size_t)TgTile<128, 128>::LDS_FLOATS * sizeof(float);
    hipLaunchKernelGGL((expert_cond_kernel<128, 128>), dim3(K * nTn), dim3(kTgThreads), shm, s, A,
                       lda, q_sqrt, ldqs, strideq, stats, lds, nTs, variance, M, N, K, fmean, fvar, ldf);
  }
  return launch_status();
}
