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
//
// gfx950 mapping: 256 threads = 4 waves (one per SIMD), workgroup tile
// BM x BN (256x256 or 128x128); wave (wr, wc) owns the 32-row tiles
// j = wr, wr+2, ... (interleaved, so both row-waves see the same share of the
// triangle) and BN/2 contiguous columns, as RT x CT accumulators of
// v_mfma_f32_32x32x2_f32 (exact f32, 64 cycles/SIMD).  K-chunks of 16 rows of
// T and B go global -> registers -> LDS (double buffered, one barrier per
// chunk); the chunk's A/B fragments are read into registers before its MFMA
// block.  Chunks that cross the diagonal are masked to the triangle and skip
// the 32-row tiles lying wholly in the zero triangle (scalar branches on
// readfirstlane'd counts); all other chunks run a branch-free MFMA block.
// Roofline: f32 MFMA bound (K4: M^2 N flops, K5: K M^2 N flops at c3:
// 68.7 / 549.8 GFLOP vs 157.3 TFLOP/s).
#include "mgp_common.hpp"

namespace mgp {

constexpr int kTgBK = 16;

// Workgroup tile BM x BN; waves WR (rows) x WC (columns); each wave owns
// (BM/WR) x (BN/WC) as RT x CT 32x32 accumulators.
template <int BM, int BN>
struct TgCfg {
  static constexpr int WR = BM >= 128 ? 2 : 1;
  static constexpr int WC = 4;
  static constexpr int THREADS = WR * WC * 64;
};

template <int BM, int BN, bool UPPER, bool GUARD>
struct TriGemm {
  static constexpr int WR = TgCfg<BM, BN>::WR, WC = TgCfg<BM, BN>::WC;
  static constexpr int NT = TgCfg<BM, BN>::THREADS;
  static constexpr int WM = BM / WR, WN = BN / WC;  // wave tile
  static constexpr int RT = WM / 32, CT = WN / 32;  // 32x32 accumulators per wave
  static constexpr int T4 = kTgBK * BM / 4 / NT;    // float4 of T per thread per chunk
  static constexpr int B4 = kTgBK * BN / 4 / NT;
  static constexpr int LDS_FLOATS = 2 * kTgBK * (BM + BN);
  static constexpr int KS = kTgBK / 2;              // MFMA k-steps per chunk
  static_assert(T4 >= 1 && B4 >= 1, "tile too small for the thread count");

  __device__ static __forceinline__ int tile_row(int wr, int r) { return wr * WM + 32 * r; }

  struct Ctx {
    const float* T; int64_t ldt; const float* B; int64_t ldb;
    int64_t M, N, i0, n0, kbeg;
    int nchunks;
    // fast path: buffer resources + per-thread byte offsets (32-bit addressing)
    __amdgpu_buffer_rsrc_t rT, rB;
    uint32_t vT[T4], vB[B4];
  };

  // Registers -> LDS; a chunk crossing the diagonal is masked to the triangle
  // here (after the loads have landed: the mask is data-only, no control flow).
  __device__ static __forceinline__ void store_chunk(float* __restrict__ sT, floatx4 (&rt)[T4],
                                                     const floatx4 (&rb)[B4], int dk) {
    float* sB = sT + kTgBK * BM;
    const int t = threadIdx.x;
    const bool diag = dk > -kTgBK && dk < BM;   // chunk rows k0..k0+15 meet the row tile
#pragma unroll
    for (int q = 0; q < T4; ++q) {
      const int idx = t + NT * q;
      const int rel = dk + idx / (BM / 4) - (idx % (BM / 4)) * 4;  // k - i of element 0
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const bool keep = !diag || (UPPER ? (rel >= e) : (rel <= e));
        rt[q][e] = keep ? rt[q][e] : 0.f;
      }
      *reinterpret_cast<floatx4*>(sT + idx * 4) = rt[q];
    }
#pragma unroll
    for (int q = 0; q < B4; ++q) *reinterpret_cast<floatx4*>(sB + (t + NT * q) * 4) = rb[q];
  }

  // Issue the global loads of chunk k0 (rows k0..k0+15 of T[:, i0:i0+BM] and
  // B[:, n0:n0+BN]) into registers.  Thread t owns float4 q at row idx/(BM/4),
  // col 4*(idx%(BM/4)), idx = t + NT*q.
  __device__ static __forceinline__ void load_chunk(floatx4 (&rt)[T4], floatx4 (&rb)[B4], const Ctx& cx,
                                                    int64_t k0) {
    const int t = threadIdx.x;
    const uint32_t soT = (uint32_t)((k0 * cx.ldt + cx.i0) * 4);
    const uint32_t soB = (uint32_t)((k0 * cx.ldb + cx.n0) * 4);
#pragma unroll
    for (int q = 0; q < T4; ++q) {
      const int idx = t + NT * q;
      const int r = idx / (BM / 4), c = (idx % (BM / 4)) * 4;
      if (GUARD) rt[q] = load4_guarded(cx.T, cx.ldt, k0 + r, cx.i0 + c, cx.M, cx.M);
      else rt[q] = __builtin_bit_cast(floatx4, __builtin_amdgcn_raw_buffer_load_b128(cx.rT, cx.vT[q], soT, 0));
    }
#pragma unroll
    for (int q = 0; q < B4; ++q) {
      const int idx = t + NT * q;
      const int r = idx / (BN / 4), c = (idx % (BN / 4)) * 4;
      if (GUARD) rb[q] = load4_guarded(cx.B, cx.ldb, k0 + r, cx.n0 + c, cx.M, cx.N);
      else rb[q] = __builtin_bit_cast(floatx4, __builtin_amdgcn_raw_buffer_load_b128(cx.rB, cx.vB[q], soB, 0));
    }
  }

  // acc[RT][CT] = sum over k in [kbeg, kend) of T[k][i0 + .] B[k][n0 + .] for
  // this wave.  One straight-line loop body for every chunk (the triangle is
  // enforced by the store-time mask), so accumulators never cross a branch.
  __device__ static __forceinline__ void run(floatx16 (&acc)[RT][CT], float* __restrict__ lds,
                                             const float* __restrict__ T, int64_t ldt,
                                             const float* __restrict__ B, int64_t ldb, int64_t M,
                                             int64_t N, int64_t i0, int64_t n0, int64_t kbeg,
                                             int64_t kend) {
    const int lane = threadIdx.x & 63;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int wr = w / WC, wc = w % WC;
    const int h = lane >> 5, l32 = lane & 31;
#pragma unroll
    for (int r = 0; r < RT; ++r)
#pragma unroll
      for (int c = 0; c < CT; ++c)
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[r][c][e] = 0.f;
    if (kend <= kbeg) return;
    Ctx cx;
    cx.T = T; cx.ldt = ldt; cx.B = B; cx.ldb = ldb; cx.M = M; cx.N = N;
    cx.i0 = i0; cx.n0 = n0; cx.kbeg = kbeg;
    cx.nchunks = (int)((kend - kbeg + kTgBK - 1) / kTgBK);
    if (!GUARD) {
      cx.rT = __builtin_amdgcn_make_buffer_rsrc((void*)T, (short)0, (int)(M * ldt * 4), 0x00020000);
      cx.rB = __builtin_amdgcn_make_buffer_rsrc((void*)B, (short)0, (int)(M * ldb * 4), 0x00020000);
#pragma unroll
      for (int q = 0; q < T4; ++q) {
        const int idx = threadIdx.x + NT * q;
        cx.vT[q] = (uint32_t)(((idx / (BM / 4)) * ldt + (idx % (BM / 4)) * 4) * 4);
      }
#pragma unroll
      for (int q = 0; q < B4; ++q) {
        const int idx = threadIdx.x + NT * q;
        cx.vB[q] = (uint32_t)(((idx / (BN / 4)) * ldb + (idx % (BN / 4)) * 4) * 4);
      }
    }
    int aoff[RT], boff[CT];
#pragma unroll
    for (int r = 0; r < RT; ++r) aoff[r] = tile_row(wr, r) + l32;
#pragma unroll
    for (int c = 0; c < CT; ++c) boff[c] = wc * WN + 32 * c + l32;

    floatx4 rt[T4], rb[B4];
    load_chunk(rt, rb, cx, kbeg);
    store_chunk(lds, rt, rb, (int)(kbeg - i0));
    __syncthreads();
#pragma nounroll
    for (int ch = 0; ch < cx.nchunks; ++ch) {
      const int64_t k0 = kbeg + (int64_t)ch * kTgBK;
      const float* sT = lds + (ch & 1) * kTgBK * (BM + BN);
      const float* sB = sT + kTgBK * BM;
      const bool more = ch + 1 < cx.nchunks;
      if (more) load_chunk(rt, rb, cx, k0 + kTgBK);
      float fa[KS][RT], fb[KS][CT];
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        const int kl = 2 * ks + h;
#pragma unroll
        for (int r = 0; r < RT; ++r) fa[ks][r] = sT[kl * BM + aoff[r]];
#pragma unroll
        for (int c = 0; c < CT; ++c) fb[ks][c] = sB[kl * BN + boff[c]];
      }
#pragma unroll
      for (int ks = 0; ks < KS; ++ks)
#pragma unroll
        for (int r = 0; r < RT; ++r)
#pragma unroll
          for (int c = 0; c < CT; ++c) acc[r][c] = mfma32x32x2(fa[ks][r], fb[ks][c], acc[r][c]);
      if (more) store_chunk(lds + ((ch + 1) & 1) * kTgBK * (BM + BN), rt, rb, (int)(k0 + kTgBK - i0));
      __syncthreads();
    }
  }
};

// ------------------------------------------------------------------ K4
// grid.x = nTiles_m * nTiles_n; heavy (large i0) row tiles first.
template <int BM, int BN, int KMAX, bool GUARD>
__global__ __launch_bounds__((TgCfg<BM, BN>::THREADS), (TgCfg<BM, BN>::THREADS / 256)) void trsm_stats_kernel(
    const float* __restrict__ LinvT, int64_t ldl, const float* __restrict__ Kuf, int64_t ldk,
    int64_t M, int64_t N, const float* __restrict__ q_mu, int64_t ldq, int K,
    float* __restrict__ A, int64_t lda, float* __restrict__ stats, int64_t lds_) {
  using G = TriGemm<BM, BN, false, GUARD>;
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int nTm = (int)((M + BM - 1) / BM), nTn = (int)((N + BN - 1) / BN);
  const int tm = nTm - 1 - (int)(blockIdx.x / nTn);
  const int tn = (int)(blockIdx.x % nTn);
  const int64_t i0 = (int64_t)tm * BM, n0 = (int64_t)tn * BN;
  const int64_t kend = (i0 + BM < M) ? i0 + BM : M;
  floatx16 acc[G::RT][G::CT];
  G::run(acc, lds, LinvT, ldl, Kuf, ldk, M, N, i0, n0, 0, kend);

  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = w / G::WC, wc = w % G::WC, l32 = lane & 31;
  // ---- write A
#pragma unroll
  for (int r = 0; r < G::RT; ++r)
#pragma unroll
    for (int c = 0; c < G::CT; ++c) {
      const int64_t col = n0 + wc * G::WN + 32 * c + l32;
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int64_t row = i0 + G::tile_row(wr, r) + acc_row(e, lane);
        if (!GUARD || (row < M && col < N)) A[row * lda + col] = acc[r][c][e];
      }
    }
  // ---- stats: stage q_mu rows of this tile (zero beyond M / K)
  float* sQ = lds;                       // [BM][KMAX]
  float* sRed = lds + BM * KMAX;         // [WR][KMAX + 1][BN]
  for (int idx = threadIdx.x; idx < BM * KMAX; idx += G::NT) {
    const int r = idx / KMAX, kk = idx % KMAX;
    sQ[idx] = (i0 + r < M && kk < K) ? q_mu[(i0 + r) * ldq + kk] : 0.f;
  }
  __syncthreads();
  float sq[G::CT], qm[G::CT][KMAX];
#pragma unroll
  for (int c = 0; c < G::CT; ++c) {
    sq[c] = 0.f;
#pragma unroll
    for (int kk = 0; kk < KMAX; ++kk) qm[c][kk] = 0.f;
  }
#pragma unroll
  for (int r = 0; r < G::RT; ++r)
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const int lr = G::tile_row(wr, r) + acc_row(e, lane);
      float q[KMAX];
#pragma unroll
      for (int kk = 0; kk < KMAX; ++kk) q[kk] = sQ[lr * KMAX + kk];
#pragma unroll
      for (int c = 0; c < G::CT; ++c) {
        const float v = acc[r][c][e];
        sq[c] = fmaf(v, v, sq[c]);
#pragma unroll
        for (int kk = 0; kk < KMAX; ++kk) qm[c][kk] = fmaf(v, q[kk], qm[c][kk]);
      }
    }
  // combine the two lane halves (rows 4h..), then the two row-waves via LDS
#pragma unroll
  for (int c = 0; c < G::CT; ++c) {
    sq[c] += __shfl_xor(sq[c], 32, 64);
#pragma unroll
    for (int kk = 0; kk < KMAX; ++kk) qm[c][kk] += __shfl_xor(qm[c][kk], 32, 64);
  }
  if (lane < 32) {
#pragma unroll
    for (int c = 0; c < G::CT; ++c) {
      const int lc = wc * G::WN + 32 * c + l32;
      sRed[(wr * (KMAX + 1) + 0) * BN + lc] = sq[c];
#pragma unroll
      for (int kk = 0; kk < KMAX; ++kk) sRed[(wr * (KMAX + 1) + 1 + kk) * BN + lc] = qm[c][kk];
    }
  }
  __syncthreads();
  float* st = stats + (int64_t)tm * (K + 1) * lds_;
  for (int idx = threadIdx.x; idx < (K + 1) * BN; idx += G::NT) {
    const int row = idx / BN, lc = idx % BN;
    const int64_t n = n0 + lc;
    float v = 0.f;
#pragma unroll
    for (int q = 0; q < G::WR; ++q) v += sRed[(q * (KMAX + 1) + row) * BN + lc];
    if (n < N) st[row * lds_ + n] = v;
  }
}

// ------------------------------------------------------------------ K5
// One workgroup per item (expert k, column tile tn, row tile t): the partial
// sum over the tile's 128 rows of (L_k^T A)^2 is written to part[k][t][n]
// (deterministic; cond_finalize adds the T partials).  Items are dispatched
// heaviest row tile first (LPT: the t-th tile walks M - 128 t rows of K), and
// within a row tile the 8 experts of one column tile sit at block ids that
// are equal mod 8, i.e. on one XCD (round-robin dispatch), so they share the
// A slab in that XCD's L2.
template <int BM, int BN, bool GUARD>
__global__ __launch_bounds__((TgCfg<BM, BN>::THREADS), (TgCfg<BM, BN>::THREADS / 256)) void expert_cond_kernel(
    const float* __restrict__ Amat, int64_t lda, const float* __restrict__ q_sqrt, int64_t ldqs,
    int64_t strideq, int64_t M, int64_t N, int K, float* __restrict__ part, int64_t ldp) {
  using G = TriGemm<BM, BN, true, GUARD>;
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int nTn = (int)((N + BN - 1) / BN), nTm = (int)((M + BM - 1) / BM);
  // block -> (t, tn, k): b = 8 * j + x (x = XCD group); within a group j runs
  // over (t heavy-first, column tiles tn = x mod 8, experts k).
  const int b = blockIdx.x;
  int t, tn, k;
  if (nTn % 8 == 0) {
    const int x = b & 7, j = b >> 3;
    const int per_t = (nTn / 8) * K;
    t = j / per_t;
    const int rem = j % per_t;
    tn = (rem / K) * 8 + x;
    k = rem % K;
  } else {
    const int per_t = nTn * K;
    t = b / per_t;
    tn = (b % per_t) / K;
    k = b % K;
  }
  const int tm = t;                         // heavy first: tile 0 walks all M rows
  const int64_t n0 = (int64_t)tn * BN, i0 = (int64_t)tm * BM;
  const float* Lk = q_sqrt + (int64_t)k * strideq;
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = w / G::WC, wc = w % G::WC, l32 = lane & 31;
  floatx16 acc[G::RT][G::CT];
  G::run(acc, lds, Lk, ldqs, Amat, lda, M, N, i0, n0, i0, M);
  float colsq[G::CT];
#pragma unroll
  for (int c = 0; c < G::CT; ++c) {
    colsq[c] = 0.f;
#pragma unroll
    for (int r = 0; r < G::RT; ++r)
#pragma unroll
      for (int e = 0; e < 16; ++e) colsq[c] = fmaf(acc[r][c][e], acc[r][c][e], colsq[c]);
    colsq[c] += __shfl_xor(colsq[c], 32, 64);
  }
  float* sRed = lds;  // [WR][BN]
  if (lane < 32) {
#pragma unroll
    for (int c = 0; c < G::CT; ++c) sRed[wr * BN + wc * G::WN + 32 * c + l32] = colsq[c];
  }
  __syncthreads();
  float* dst = part + ((int64_t)k * nTm + tm) * ldp;
  for (int lc = threadIdx.x; lc < BN; lc += G::NT) {
    const int64_t n = n0 + lc;
    float v = 0.f;
#pragma unroll
    for (int q = 0; q < G::WR; ++q) v += sRed[q * BN + lc];
    if (n < N) dst[n] = v;
  }
}

// fmean[k][n] = sum_t stats[t][1+k][n];
// fvar[k][n]  = var - sum_t stats[t][0][n] + sum_t part[k][t][n].
// One (n, k) of the finalize: the tile sums in tile order, their loads issued eight
// at a time ahead of the adds (the loop had one dependent load round trip per tile).
__device__ __forceinline__ void cond_finalize_elem(const float* __restrict__ stats, int64_t lds_, int nTs,
                                                   const float* __restrict__ part, int64_t ldp, int nT,
                                                   const float* __restrict__ variance, int K,
                                                   float* __restrict__ fmean, float* __restrict__ fvar, int64_t ldf,
                                                   int64_t n, int k) {
  constexpr int B = 8;
  float a2 = 0.f, fm = 0.f, q = 0.f;
  const int64_t ts = (int64_t)(K + 1) * lds_, fo = (int64_t)(1 + k) * lds_;
  int t = 0;
  for (; t + B <= nTs; t += B) {
    float x[B], y[B];
#pragma unroll
    for (int u = 0; u < B; ++u) {
      const float* st = stats + (int64_t)(t + u) * ts;
      x[u] = st[n];
      y[u] = st[fo + n];
    }
#pragma unroll
    for (int u = 0; u < B; ++u) {
      a2 += x[u];
      fm += y[u];
    }
  }
  for (; t < nTs; ++t) {
    const float* st = stats + (int64_t)t * ts;
    a2 += st[n];
    fm += st[fo + n];
  }
  const float* pk = part + (int64_t)k * nT * ldp + n;
  t = 0;
  for (; t + B <= nT; t += B) {
    float x[B];
#pragma unroll
    for (int u = 0; u < B; ++u) x[u] = pk[(int64_t)(t + u) * ldp];
#pragma unroll
    for (int u = 0; u < B; ++u) q += x[u];
  }
  for (; t < nT; ++t) q += pk[(int64_t)t * ldp];
  fmean[(int64_t)k * ldf + n] = fm;
  fvar[(int64_t)k * ldf + n] = (variance[0] - a2) + q;
}

__global__ __launch_bounds__(256) void cond_finalize_kernel(const float* __restrict__ stats, int64_t lds_,
                                                            int nTs, const float* __restrict__ part, int64_t ldp,
                                                            int nT, const float* __restrict__ variance,
                                                            int64_t N, int K, float* __restrict__ fmean,
                                                            float* __restrict__ fvar, int64_t ldf) {
  const int64_t n = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int k = blockIdx.y;
  if (n >= N) return;
  cond_finalize_elem(stats, lds_, nTs, part, ldp, nT, variance, K, fmean, fvar, ldf, n, k);
}

// cond_finalize_kernel for two layers in one launch (blockIdx.z: the layer), the same
// per-element sums in the same order (bit-identical).
__global__ __launch_bounds__(256) void cond_finalize2_kernel(CondFinLayer l0, CondFinLayer l1, int64_t lds_, int nTs,
                                                             int64_t ldp, int nT, int64_t N, int K, int64_t ldf) {
  const CondFinLayer& l = blockIdx.z ? l1 : l0;
  const int64_t n = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int k = blockIdx.y;
  if (n >= N) return;
  cond_finalize_elem(l.stats, lds_, nTs, l.part, ldp, nT, l.variance, K, l.fmean, l.fvar, ldf, n, k);
}

}  // namespace mgp

using namespace mgp;

// Tile choice shared by K4 and K5: row tile BM = kTgBM always (the stats tiling
// depends on it: T = ceil(M / BM)); column tile 256 for large N, else 128.
#ifndef MGP_TG_BM
#define MGP_TG_BM 64
#endif
constexpr int kTgBM = MGP_TG_BM;
static inline int tg_bn(int64_t N) { return N >= 256 * 64 ? 256 : 128; }

extern "C" int mgp_stats_tiles(int64_t M) { return (int)((M + kTgBM - 1) / kTgBM); }

template <int BN, int KMAX>
static int launch_trsm(const float* LinvT, int64_t ldl, const float* Kuf, int64_t ldk, int64_t M,
                       int64_t N, const float* q_mu, int64_t ldq, int K, float* A, int64_t lda,
                       float* stats, int64_t lds, hipStream_t s) {
  constexpr int BM = kTgBM;
  const int nTm = (int)((M + BM - 1) / BM), nTn = (int)((N + BN - 1) / BN);
  const size_t shm = (size_t)TriGemm<BM, BN, false, false>::LDS_FLOATS * sizeof(float);
  const size_t shm2 = (size_t)(BM * KMAX + 2 * (KMAX + 1) * BN) * sizeof(float);
  const size_t sh = shm > shm2 ? shm : shm2;
  const dim3 grid(nTm * nTn), block(TgCfg<BM, BN>::THREADS);
  if ((M % BM == 0) && (N % BN == 0))
    hipLaunchKernelGGL((trsm_stats_kernel<BM, BN, KMAX, false>), grid, block, sh, s, LinvT, ldl, Kuf, ldk,
                       M, N, q_mu, ldq, K, A, lda, stats, lds);
  else
    hipLaunchKernelGGL((trsm_stats_kernel<BM, BN, KMAX, true>), grid, block, sh, s, LinvT, ldl, Kuf, ldk,
                       M, N, q_mu, ldq, K, A, lda, stats, lds);
  return launch_status();
}

template <int BN>
static int dispatch_trsm(const float* LinvT, int64_t ldl, const float* Kuf, int64_t ldk, int64_t M,
                         int64_t N, const float* q_mu, int64_t ldq, int K, float* A, int64_t lda,
                         float* stats, int64_t lds, hipStream_t s) {
  if (K <= 4) return launch_trsm<BN, 4>(LinvT, ldl, Kuf, ldk, M, N, q_mu, ldq, K, A, lda, stats, lds, s);
  if (K <= 8) return launch_trsm<BN, 8>(LinvT, ldl, Kuf, ldk, M, N, q_mu, ldq, K, A, lda, stats, lds, s);
  if (K <= 16) return launch_trsm<BN, 16>(LinvT, ldl, Kuf, ldk, M, N, q_mu, ldq, K, A, lda, stats, lds, s);
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
  if (M * ldk * 4 >= (int64_t)1 << 31 || M * ldl * 4 >= (int64_t)1 << 31) return MGP_ERR_UNSUPPORTED;
  if (M == 0 || N == 0) return MGP_OK;
  hipStream_t s = (hipStream_t)stream;
  if (tg_bn(N) == 256) return dispatch_trsm<256>(LinvT, ldl, Kuf, ldk, M, N, q_mu, ldq, K, A, lda, stats, lds, s);
  return dispatch_trsm<128>(LinvT, ldl, Kuf, ldk, M, N, q_mu, ldq, K, A, lda, stats, lds, s);
}

int mgp::mgp_launch_cond_finalize(const float* stats, int64_t lds, int nTs, const float* part, int64_t ldp,
                                  int nTp, const float* variance, int64_t N, int K, float* fmean, float* fvar,
                                  int64_t ldf, hipStream_t s) {
  hipLaunchKernelGGL(cond_finalize_kernel, dim3((unsigned)((N + 255) / 256), K), dim3(256), 0, s, stats, lds,
                     nTs, part, ldp, nTp, variance, N, K, fmean, fvar, ldf);
  return launch_status();
}

int mgp::mgp_launch_cond_finalize2(const CondFinLayer& l0, const CondFinLayer& l1, int64_t lds, int nTs, int64_t ldp,
                                   int nTp, int64_t N, int K, int64_t ldf, hipStream_t s) {
  hipLaunchKernelGGL(cond_finalize2_kernel, dim3((unsigned)((N + 255) / 256), K, 2), dim3(256), 0, s, l0, l1, lds,
                     nTs, ldp, nTp, N, K, ldf);
  return launch_status();
}

static int64_t expert_ldp(int64_t N) { return (N + 3) / 4 * 4; }

extern "C" size_t mgp_expert_workspace_bytes(int64_t M, int64_t N, int32_t K) {
  if (M <= 0 || N <= 0 || K <= 0) return 16;
  return (size_t)K * (size_t)((M + kTgBM - 1) / kTgBM) * (size_t)expert_ldp(N) * sizeof(float);
}

template <int BN>
static int launch_expert(const float* A, int64_t lda, const float* q_sqrt, int64_t ldqs,
                         int64_t strideq, const float* stats, int64_t lds, const float* variance,
                         int64_t M, int64_t N, int K, float* fmean, float* fvar, int64_t ldf,
                         float* part, hipStream_t s) {
  constexpr int BM = kTgBM;
  const int nTn = (int)((N + BN - 1) / BN), nTm = (int)((M + BM - 1) / BM);
  const int64_t ldp = expert_ldp(N);
  const size_t shm = (size_t)TriGemm<BM, BN, true, false>::LDS_FLOATS * sizeof(float);
  const dim3 grid(K * nTn * nTm), block(TgCfg<BM, BN>::THREADS);
  if (M % BM == 0 && N % BN == 0)
    hipLaunchKernelGGL((expert_cond_kernel<BM, BN, false>), grid, block, shm, s, A, lda, q_sqrt, ldqs,
                       strideq, M, N, K, part, ldp);
  else
    hipLaunchKernelGGL((expert_cond_kernel<BM, BN, true>), grid, block, shm, s, A, lda, q_sqrt, ldqs,
                       strideq, M, N, K, part, ldp);
  int st = launch_status();
  if (st) return st;
  return mgp_launch_cond_finalize(stats, lds, nTm, part, ldp, nTm, variance, N, K, fmean, fvar, ldf, s);
}

extern "C" int mgp_expert_conditional_f32(const float* A, int64_t lda, const float* q_sqrt, int64_t ldqs,
                                      int64_t strideq, const float* stats, int64_t lds,
                                      const float* variance, int64_t M, int64_t N, int32_t K,
                                      float* fmean, float* fvar, int64_t ldf, void* workspace,
                                      size_t workspace_bytes, mgp_stream_t stream) {
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
  if (M * lda * 4 >= (int64_t)1 << 31 || M * ldqs * 4 >= (int64_t)1 << 31) return MGP_ERR_UNSUPPORTED;
  if (N == 0 || M == 0) return MGP_OK;
  if (!workspace || workspace_bytes < mgp_expert_workspace_bytes(M, N, K)) return MGP_ERR_WORKSPACE;
  hipStream_t s = (hipStream_t)stream;
  float* part = (float*)workspace;
  if (tg_bn(N) == 256)
    return launch_expert<256>(A, lda, q_sqrt, ldqs, strideq, stats, lds, variance, M, N, K, fmean, fvar,
                              ldf, part, s);
  return launch_expert<128>(A, lda, q_sqrt, ldqs, strideq, stats, lds, variance, M, N, K, fmean, fvar,
                            ldf, part, s);
}
