// K3: batched blocked Cholesky of Kuu with the triangular inverse fused in,
// computed in float64 (optionally with Kuu itself built in float64 from Z).
//
// Reference: Lm = tf.linalg.cholesky(Kmm) inside GPflow base_conditional,
// reached from MixtureGPs/models.py:141, with Kmm = covariances.Kuu(Z, kernel,
// jitter) from models.py:135; the inverse replaces the S-batched
// tf.linalg.triangular_solve(Lm, Kmn) by one triangular GEMM (trigemm.hip).
//
// Precision design: the reference runs in float64.  Kuu is often badly
// conditioned (cond 1e4..1e7 for inducing points drawn from the data), and a
// float32 factorisation (LAPACK spotrf included) loses cond(L) * eps32 -- up to
// 1e-3 normwise on the conditional at BASELINE config 2.  The M x M work here is
// M^3/3 flops (0.36 GFLOP at M = 1024, a few microseconds of the chip), so it
// runs in float64 (v_mfma_f64_16x16x4_f64 + f64 VALU) and only the N-scaled
// GEMMs (K4/K5) run in float32.  Outputs L and (L^-1)^T are rounded to float32.
//
// Algorithm (block CB = 64, nb = ceil(M/64), matrix padded with identity to
// nb*64): a right-looking blocked Cholesky that carries the forward
// substitution of L X = I along ("augmented" sweep):
//   step j:  P_i = W_ij D_j^T                    (= L_ij, D_j = L_jj^-1)
//            W_il -= P_i P_l^T        j < l <= i (trailing update, f64 MFMA)
//            X_jc  = D_j B_jc         c <= j     (row block j of X = L^-1)
//            B_ic -= P_i X_jc         i > j      (forward-substitution update)
//            the workgroup that owns tile (j+1, j+1) factors it right after its
//            update (look-ahead), producing L_{j+1,j+1} and D_{j+1}.
// One launch per step; every tile of a step is independent (each workgroup
// recomputes the 64^3 panels it needs); every launch carries all `batch`
// matrices (blockIdx.y).  nb + 1 launches per factorisation.
#include <math.h>
#include <stdlib.h>

#include <algorithm>

#include "mgp_common.hpp"

namespace mgp {

typedef double doublex4 __attribute__((ext_vector_type(4)));

constexpr int CB = 64;        // Cholesky block
constexpr int LDT = CB + 2;   // LDS leading dimension (doubles): conflict-free b64 reads
constexpr int kCholThreads = 256;
constexpr int kMaxBatch = 8;

// Thread index within a 256-thread tile group: the tile helpers below work on one
// 64x64 tile with 4 waves; chol_step_pair runs two such groups per workgroup (512
// threads), every other kernel here is one group (threadIdx.x < 256).
__device__ __forceinline__ int ctid() { return (int)(threadIdx.x & (kCholThreads - 1)); }

#ifdef MGP_DBG_STAMPS
__device__ unsigned long long g_stamps[64 * 16];
// persistent path: chain stamps [batch 2][step 128][8]; worker phase totals [batch 2][wg 128][8]
__device__ unsigned long long g_pchain[2 * 128 * 8];
__device__ unsigned long long g_pwork[2 * 128 * 8];
#define PSTAMP(b, j, k) do { if (ctid() == 0 && (b) < 2 && (j) < 128) g_pchain[((b) * 128 + (j)) * 8 + (k)] = __builtin_amdgcn_s_memtime(); } while (0)
#define PWACC(b, w, k, v) do { if (ctid() == 0 && (b) < 2 && (w) < 128) g_pwork[((b) * 128 + (w)) * 8 + (k)] += (v); } while (0)
#define PNOW() __builtin_amdgcn_s_memtime()
#define STAMP(j, k) do { if (ctid() == 0 && blockIdx.y == 0) g_stamps[(j) * 16 + (k)] = __builtin_amdgcn_s_memtime(); } while (0)
// 100 MHz reference clock (one time base for every CU): slots 14 / 15
#define RSTAMP(j, k) do { if (ctid() == 0 && blockIdx.y == 0) g_stamps[(j) * 16 + (k)] = __builtin_amdgcn_s_memrealtime(); } while (0)
#else
#define STAMP(j, k) do {} while (0)
#define RSTAMP(j, k) do {} while (0)
#define PSTAMP(b, j, k) do {} while (0)
#define PWACC(b, w, k, v) do {} while (0)
#define PNOW() 0ull
#endif

struct CholArgs {
  // input: either a float32 matrix A (per batch at A + b*strideA) ...
  const float* A; int64_t lda, strideA;
  // ... or Kuu built from Z (float64 arithmetic): Kuu = var exp(-0.5 |(zi-zj)/l|^2) + jitter I
  const float* Z[kMaxBatch]; const float* var[kMaxBatch]; const float* ls[kMaxBatch];
  int n_ls[kMaxBatch]; int64_t ldz; int D; double jitter;
  float* L; float* LinvT; int64_t ldl, strideL;   // L may be NULL
  int32_t* info;
  float* lt_absmax[kMaxBatch];                    // optional per batch: max |L^-T| (float bits, atomicMax)
  double* ws; int64_t strideWS;                   // per batch: W, B [Mp][Mp], D [nb][64][64]
  int64_t M, Mp; int nb;
  // persistent path (chol_persist): per-batch sync words and the shared task table
  int* sync; int64_t strideSync;                  // per batch: Wver[nb][nb], Bver[nb][nb], Dready[nb], head, err
  int* tasks; int ntask;                          // task table (chol_task_order), built by chol_prep
};

__device__ __forceinline__ double* ws_W(const CholArgs& a, int b) { return a.ws + (int64_t)b * a.strideWS; }
__device__ __forceinline__ double* ws_B(const CholArgs& a, int b) { return ws_W(a, b) + a.Mp * a.Mp; }
__device__ __forceinline__ double* ws_D(const CholArgs& a, int b, int j) {
  return ws_W(a, b) + 2 * a.Mp * a.Mp + (int64_t)j * CB * CB;
}

// Element (gr, gc) of the padded input matrix, in float64.
__device__ __forceinline__ double input_elem(const CholArgs& a, int b, int64_t gr, int64_t gc) {
  if (gr >= a.M || gc >= a.M) return gr == gc ? 1.0 : 0.0;
  if (a.A) return (double)a.A[(int64_t)b * a.strideA + gr * a.lda + gc];
  // select this batch entry without dynamic indexing of the by-value argument
  // arrays (that would copy the whole struct to scratch)
  const float *Z = a.Z[0], *ls = a.ls[0], *var = a.var[0];
  int nls = a.n_ls[0];
#pragma unroll
  for (int i = 1; i < kMaxBatch; ++i)
    if (b == i) { Z = a.Z[i]; ls = a.ls[i]; var = a.var[i]; nls = a.n_ls[i]; }
  double s = 0.0;
  for (int d = 0; d < a.D; ++d) {
    const double l = (double)ls[nls == 1 ? 0 : d];
    const double diff = ((double)Z[gr * a.ldz + d] - (double)Z[gc * a.ldz + d]) / l;
    s = fma(diff, diff, s);
  }
  double v = (double)var[0] * exp(-0.5 * s);
  if (gr == gc) v += a.jitter;
  return v;
}

// Kuu element (gr, gc) of batch entry b from Z with the inverse lengthscales sil
// (float64, precomputed once per workgroup: no division per element).
__device__ __forceinline__ double kuu_elem(const CholArgs& a, const float* __restrict__ Z,
                                           const double* __restrict__ sil, double var, int64_t gr, int64_t gc) {
  if (gr >= a.M || gc >= a.M) return gr == gc ? 1.0 : 0.0;
  double s = 0.0;
  for (int d = 0; d < a.D; ++d) {
    const double diff = ((double)Z[gr * a.ldz + d] - (double)Z[gc * a.ldz + d]) * sil[d];
    s = fma(diff, diff, s);
  }
  double v = var * exp(-0.5 * s);
  if (gr == gc) v += a.jitter;
  return v;
}

// 64x64 f64 tile (row-major, ld) staged through registers: fetch issues all
// eight 16-B loads per thread before any LDS store, so several tiles' loads
// can be in flight together (fetch, fetch, ..., put, put).
struct TileRegs {
  double2 v[8];
};
__device__ __forceinline__ void tile_fetch(TileRegs& t, const double* __restrict__ g, int64_t ld) {
#pragma unroll
  for (int it = 0; it < 8; ++it) {
    const int idx = ctid() + kCholThreads * it, r = idx >> 5, c = (idx & 31) * 2;
    t.v[it] = *reinterpret_cast<const double2*>(g + (int64_t)r * ld + c);
  }
}
__device__ __forceinline__ void tile_put(double* __restrict__ s, const TileRegs& t) {
#pragma unroll
  for (int it = 0; it < 8; ++it) {
    const int idx = ctid() + kCholThreads * it, r = idx >> 5, c = (idx & 31) * 2;
    s[r * LDT + c] = t.v[it].x;
    s[r * LDT + c + 1] = t.v[it].y;
  }
}
__device__ __forceinline__ void tile_load(double* __restrict__ s, const double* __restrict__ g, int64_t ld) {
  TileRegs t;
  tile_fetch(t, g, ld);
  tile_put(s, t);
}

// LDS tile -> float32 global, optionally transposed (dst[c][r] = s[r][c]),
// guarded to rows < nr, cols < nc of the destination block.
__device__ __forceinline__ void tile_store_f32(float* __restrict__ g, int64_t ld, const double* __restrict__ s,
                                               bool transpose, int nr, int nc) {
  for (int idx = ctid(); idx < CB * CB; idx += kCholThreads) {
    const int r = idx >> 6, c = idx & 63;
    if (r < nr && c < nc) g[(int64_t)r * ld + c] = (float)(transpose ? s[c * LDT + r] : s[r * LDT + c]);
  }
}

// tile_store_f32 that also returns this thread's max |stored value|.
__device__ __forceinline__ float tile_store_f32_max(float* __restrict__ g, int64_t ld, const double* __restrict__ s,
                                                    bool transpose, int nr, int nc) {
  float m = 0.f;
  for (int idx = ctid(); idx < CB * CB; idx += kCholThreads) {
    const int r = idx >> 6, c = idx & 63;
    if (r < nr && c < nc) {
      const float v = (float)(transpose ? s[c * LDT + r] : s[r * LDT + c]);
      g[(int64_t)r * ld + c] = v;
      m = fmaxf(m, fabsf(v));
    }
  }
  return m;
}

// Full 64x64 tile -> float32 global with 16-B stores (ld % 4 == 0, 16-B aligned rows:
// chol_run checks both), optionally transposed; partial tiles fall back to the
// element loop.  Returns this thread's max |stored value|.
__device__ __forceinline__ float tile_store_f32_v4(float* __restrict__ g, int64_t ld, const double* __restrict__ s,
                                                   bool transpose, int nr, int nc) {
  if (nr < CB || nc < CB) return tile_store_f32_max(g, ld, s, transpose, nr, nc);
  float m = 0.f;
#pragma unroll
  for (int it = 0; it < 4; ++it) {
    const int idx = ctid() + kCholThreads * it, r = idx >> 4, c = (idx & 15) * 4;
    float v[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      v[k] = (float)(transpose ? s[(c + k) * LDT + r] : s[r * LDT + c + k]);
      m = fmaxf(m, fabsf(v[k]));
    }
    *reinterpret_cast<float4*>(g + (int64_t)r * ld + c) = make_float4(v[0], v[1], v[2], v[3]);
  }
  return m;
}

// Wave maximum of a non-negative float, folded into *out by one atomic per wave
// (non-negative floats order as their bit patterns).
__device__ __forceinline__ void wave_absmax_atomic(float m, float* out) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
  if ((ctid() & 63) == 0) atomicMax(reinterpret_cast<unsigned int*>(out), __float_as_uint(m));
}

__device__ __forceinline__ void tile_store_f64(double* __restrict__ g, int64_t ld, const double* __restrict__ s) {
  for (int idx = ctid(); idx < CB * CB; idx += kCholThreads) {
    const int r = idx >> 6, c = idx & 63;
    g[(int64_t)r * ld + c] = s[r * LDT + c];
  }
}

// Wave quadrant (32x32 of the 64x64 tile) as 2x2 accumulators of the f64
// 16x16x4 MFMA.  Lane l supplies A[i = l & 15][k = l >> 4], B[k = l >> 4][j = l & 15];
// result register r holds D[row = (l >> 4) + 4 r][col = l & 15].
struct Quad {
  doublex4 c[2][2];
};

__device__ __forceinline__ Quad quad_zero() {
  Quad q;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) q.c[i][j] = doublex4{0.0, 0.0, 0.0, 0.0};
  return q;
}

// q += sign * opA(sa) . opB(sb); opA(X)[i][k] = TA ? X[k][i] : X[i][k]; opB(X)[k][j] = TB ? X[j][k] : X[k][j].
template <bool TA, bool TB>
__device__ __forceinline__ void tile_mma(Quad& q, const double* __restrict__ sa, const double* __restrict__ sb,
                                         double sign) {
  const int lane = ctid() & 63, w = ctid() >> 6;
  const int qi = (w >> 1) * 32, qj = (w & 1) * 32;
  const int l16 = lane & 15, kq = lane >> 4;
#pragma unroll 4
  for (int k0 = 0; k0 < CB; k0 += 4) {
    const int k = k0 + kq;
    double a[2], b[2];
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const int i = qi + 16 * t + l16, j = qj + 16 * t + l16;
      a[t] = sign * (TA ? sa[k * LDT + i] : sa[i * LDT + k]);
      b[t] = TB ? sb[j * LDT + k] : sb[k * LDT + j];
    }
#pragma unroll
    for (int ti = 0; ti < 2; ++ti)
#pragma unroll
      for (int tj = 0; tj < 2; ++tj)
        q.c[ti][tj] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[ti], b[tj], q.c[ti][tj], 0, 0, 0);
  }
}

template <typename F>
__device__ __forceinline__ void quad_foreach(F f) {
  const int lane = ctid() & 63, w = ctid() >> 6;
  const int qi = (w >> 1) * 32, qj = (w & 1) * 32;
#pragma unroll
  for (int ti = 0; ti < 2; ++ti)
#pragma unroll
    for (int tj = 0; tj < 2; ++tj)
#pragma unroll
      for (int r = 0; r < 4; ++r) f(ti, tj, r, qi + 16 * ti + (lane >> 4) + 4 * r, qj + 16 * tj + (lane & 15));
}

__device__ __forceinline__ void quad_to_lds(double* __restrict__ s, const Quad& q) {
  quad_foreach([&](int ti, int tj, int r, int row, int col) { s[row * LDT + col] = q.c[ti][tj][r]; });
}
__device__ __forceinline__ void quad_from_global(Quad& q, const double* __restrict__ g, int64_t ld) {
  quad_foreach([&](int ti, int tj, int r, int row, int col) { q.c[ti][tj][r] = g[(int64_t)row * ld + col]; });
}
__device__ __forceinline__ void quad_to_global(double* __restrict__ g, int64_t ld, const Quad& q) {
  quad_foreach([&](int ti, int tj, int r, int row, int col) { g[(int64_t)row * ld + col] = q.c[ti][tj][r]; });
}

// Wave-striped 64x64 products that skip the zero blocks of a triangular
// operand and give every wave the same MFMA count.  RowBlk: wave w owns the
// 16-row stripe w (blocks (w, tj)); ColBlk: wave w owns the 16-column stripe w
// (blocks (ti, w)).  Lane / register layout per 16x16 block as blk_mma.
struct Blk4 {
  doublex4 c[4];
};
__device__ __forceinline__ Blk4 blk4_zero() {
  Blk4 r;
#pragma unroll
  for (int t = 0; t < 4; ++t) r.c[t] = doublex4{0.0, 0.0, 0.0, 0.0};
  return r;
}

// Row stripe: C[16w + i][16tj + j] += sign * sum_k A(i, k) B(k, j), A = sa[16w + i][k],
// B(k, j) = TB ? sb[16tj + j][k] : sb[k][16tj + j].  TRI = 0: every k; TRI = 1:
// k < 16 (tj + 1) (B = D^T, D lower triangular: 40 of 64 MFMAs); TRI = 2:
// k >= 16 tj (B = D, lower triangular).  BLK: the column blocks tj formed (bit tj).
template <bool TB, int TRI, int BLK = 0xF>
__device__ __forceinline__ void row_mma(Blk4& r, const double* __restrict__ sa, const double* __restrict__ sb,
                                        double sign) {
  const int lane = ctid() & 63, w = ctid() >> 6, l16 = lane & 15, kq = lane >> 4;
#pragma unroll
  for (int k0 = 0; k0 < CB; k0 += 4) {
    const int k = k0 + kq;
    const double av = sign * sa[(16 * w + l16) * LDT + k];
#pragma unroll
    for (int tj = 0; tj < 4; ++tj) {
      if (!((BLK >> tj) & 1)) continue;
      if (TRI == 1 && k0 >= 16 * (tj + 1)) continue;
      if (TRI == 2 && k0 < 16 * tj) continue;
      const double bv = TB ? sb[(16 * tj + l16) * LDT + k] : sb[k * LDT + 16 * tj + l16];
      r.c[tj] = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, r.c[tj], 0, 0, 0);
    }
  }
}

// Column stripe: C[16ti + i][16w + j] += sum_k D[16ti + i][k] sb[k][16w + j] with
// D lower triangular (k < 16 (ti + 1)): X_jc = D_j B_jc.
__device__ __forceinline__ void col_mma_lower(Blk4& r, const double* __restrict__ sD, const double* __restrict__ sb) {
  const int lane = ctid() & 63, w = ctid() >> 6, l16 = lane & 15, kq = lane >> 4;
#pragma unroll
  for (int k0 = 0; k0 < CB; k0 += 4) {
    const int k = k0 + kq;
    const double bv = sb[k * LDT + 16 * w + l16];
#pragma unroll
    for (int ti = 0; ti < 4; ++ti) {
      if (k0 >= 16 * (ti + 1)) continue;
      const double av = sD[(16 * ti + l16) * LDT + k];
      r.c[ti] = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, r.c[ti], 0, 0, 0);
    }
  }
}

template <bool ROW, typename F, int BLK = 0xF>
__device__ __forceinline__ void blk4_foreach(F f) {
  const int lane = ctid() & 63, w = ctid() >> 6;
#pragma unroll
  for (int t = 0; t < 4; ++t)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      if (!((BLK >> t) & 1)) continue;
      const int rr = (lane >> 4) + 4 * q, cc = lane & 15;
      if (ROW) f(t, q, 16 * w + rr, 16 * t + cc);
      else f(t, q, 16 * t + rr, 16 * w + cc);
    }
}
template <bool ROW, int BLK = 0xF>
__device__ __forceinline__ void blk4_to_lds(double* __restrict__ s, const Blk4& r) {
  auto put = [&](int t, int q, int row, int col) { s[row * LDT + col] = r.c[t][q]; };
  blk4_foreach<ROW, decltype(put), BLK>(put);
}
__device__ __forceinline__ void row_from_global(Blk4& r, const double* __restrict__ g, int64_t ld) {
  blk4_foreach<true>([&](int t, int q, int row, int col) { r.c[t][q] = g[(int64_t)row * ld + col]; });
}
__device__ __forceinline__ void row_to_global(double* __restrict__ g, int64_t ld, const Blk4& r) {
  blk4_foreach<true>([&](int t, int q, int row, int col) { g[(int64_t)row * ld + col] = r.c[t][q]; });
}

// Uniform double from lane `lane` (compile-time) of a VGPR pair.
__device__ __forceinline__ double read_lane_f64(double v, int lane) {
  const uint64_t u = (uint64_t)__double_as_longlong(v);
  const uint32_t lo = __builtin_amdgcn_readlane((uint32_t)u, lane);
  const uint32_t hi = __builtin_amdgcn_readlane((uint32_t)(u >> 32), lane);
  return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}

// 1/p to full f64 precision: hardware estimate + two Newton steps.
__device__ __forceinline__ double rcp_f64(double p) {
  double r = __builtin_amdgcn_rcp(p);
  r = fma(r, fma(-p, r, 1.0), r);
  return fma(r, fma(-p, r, 1.0), r);
}

// Quad-broadcast of a double from lane (4q + G) to lanes 4q..4q+3 (DPP quad_perm).
template <int G>
__device__ __forceinline__ double quad_bcast_f64(double v) {
  constexpr int ctrl = G * 0x55;  // quad_perm [G, G, G, G]
  const uint64_t u = (uint64_t)__double_as_longlong(v);
  const uint32_t lo = (uint32_t)__builtin_amdgcn_mov_dpp((int)(uint32_t)u, ctrl, 0xF, 0xF, true);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_mov_dpp((int)(uint32_t)(u >> 32), ctrl, 0xF, 0xF, true);
  return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}

// 1/sqrt(p) to full f64 precision: hardware estimate + two Newton steps.
__device__ __forceinline__ double rsqrt_f64(double p) {
  double r = __builtin_amdgcn_rsq(p);
  const double h = 0.5 * p;
  r = r * fma(-h * r, r, 1.5);
  return r * fma(-h * r, r, 1.5);
}

// 16x16 f64 block product on v_mfma_f64_16x16x4_f64 (one wave):
// acc += sign * opA(sa) . opB(sb), opA(X)[i][k] = X[i][k], opB(X)[k][j] = TB ? X[j][k] : X[k][j].
// Lane l supplies A[l & 15][k0 + (l >> 4)], B[k0 + (l >> 4)][l & 15]; register r of
// acc holds row (l >> 4) + 4 r, column l & 15.
template <bool TB>
__device__ __forceinline__ void blk_mma(doublex4& acc, const double* __restrict__ sa,
                                        const double* __restrict__ sb, double sign) {
  const int lane = ctid() & 63, i = lane & 15, kq = lane >> 4;
#pragma unroll
  for (int k0 = 0; k0 < 16; k0 += 4) {
    const double av = sign * sa[i * LDT + k0 + kq];
    const double bv = TB ? sb[i * LDT + k0 + kq] : sb[(k0 + kq) * LDT + i];
    acc = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, acc, 0, 0, 0);
  }
}

__device__ __forceinline__ doublex4 blk_load(const double* __restrict__ s) {
  const int lane = ctid() & 63;
  doublex4 v;
#pragma unroll
  for (int r = 0; r < 4; ++r) v[r] = s[((lane >> 4) + 4 * r) * LDT + (lane & 15)];
  return v;
}

__device__ __forceinline__ void blk_store(double* __restrict__ s, const doublex4& v) {
  const int lane = ctid() & 63;
#pragma unroll
  for (int r = 0; r < 4; ++r) s[((lane >> 4) + 4 * r) * LDT + (lane & 15)] = v[r];
}

// Lower 16x16 blocks (bi >= bj) of the diagonal tile s -= P P^T, in place in LDS;
// the 10 blocks dealt 3/3/2/2 over the waves (48 MFMAs at most per wave).
__device__ __forceinline__ void diag_lower_update(double* __restrict__ s, const double* __restrict__ sP) {
  const int w = ctid() >> 6;
  for (int q = w; q < 10; q += 4) {
    int bi = 0;
    while ((bi + 1) * (bi + 2) / 2 <= q) ++bi;
    const int bj = q - bi * (bi + 1) / 2;
    doublex4 acc = blk_load(s + 16 * bi * LDT + 16 * bj);
    const int lane = ctid() & 63, l16 = lane & 15, kq = lane >> 4;
#pragma unroll
    for (int k0 = 0; k0 < CB; k0 += 4) {
      const double av = -sP[(16 * bi + l16) * LDT + k0 + kq];
      const double bv = sP[(16 * bj + l16) * LDT + k0 + kq];
      acc = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, acc, 0, 0, 0);
    }
    blk_store(s + 16 * bi * LDT + 16 * bj, acc);
  }
}

// s[R0 .. R0+15][C1 .. C1+15] -= sum over 16 NK columns k of sa[R0 + i][k] sb[C1 + j][k]
// (one wave, f64 MFMA; rows of sa / sb at leading dimension LDT).
template <int NK>
__device__ __forceinline__ void sub_outer_blk(double* __restrict__ s, int R0, int C1, const double* __restrict__ sa,
                                              const double* __restrict__ sb) {
  doublex4 acc = blk_load(s + R0 * LDT + C1);
#pragma unroll
  for (int kk = 0; kk < NK; ++kk) blk_mma<true>(acc, sa + R0 * LDT + 16 * kk, sb + C1 * LDT + 16 * kk, -1.0);
  blk_store(s + R0 * LDT + C1, acc);
}

// Panel P (columns 16P..16P+15) of the diagonal tile, wave 0: lane r keeps the
// 16 panel entries of row r; right-looking sweep whose column broadcasts are
// readlanes from the owning lanes (no LDS round trip on the critical path).
// Per column c the 15 - c broadcasts are read before the pivot chain (they are
// final once column c - 1 is applied), so the only serial work per column is
// rsq + two Newton steps (1/piv = rs^2, no second reciprocal chain) and one
// multiply before the next column's FMA; the remaining FMAs of column c overlap
// the next pivot's chain.  Writes L's panel (zeros above the diagonal) and
// col[16P + c] = 1 / L[16P + c][16P + c].
template <int P>
__device__ __forceinline__ void panel_factor(double* __restrict__ sF, double* __restrict__ col, int r, int& bad) {
  constexpr int C0 = 16 * P;
  double a[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) a[j] = sF[r * LDT + C0 + j];
  double rs[16];
  // software pipeline: column c's pivot chain is issued before column c - 1's
  // remaining FMAs (only a[c] had to be updated first)
  double piv = read_lane_f64(a[0], C0);
  if (!(piv > 0.0) && bad == 0) bad = C0 + 1;
  rs[0] = rsqrt_f64(piv);
#pragma unroll
  for (int c = 0; c < 16; ++c) {
    double v[16];
#pragma unroll
    for (int s2 = c + 1; s2 < 16; ++s2) v[s2] = read_lane_f64(a[c], C0 + s2);  // column c, rows C0 + s2
    const double t = a[c] * (rs[c] * rs[c]);                                // a[r][c] / piv_c
    if (c + 1 < 16) {
      a[c + 1] = fma(-t, v[c + 1], a[c + 1]);
      piv = read_lane_f64(a[c + 1], C0 + c + 1);
      if (!(piv > 0.0) && bad == 0) bad = C0 + c + 2;
      rs[c + 1] = rsqrt_f64(piv);
    }
#pragma unroll
    for (int s2 = c + 2; s2 < 16; ++s2) a[s2] = fma(-t, v[s2], a[s2]);
  }
#pragma unroll
  for (int c = 0; c < 16; ++c) sF[r * LDT + C0 + c] = (r >= C0 + c) ? a[c] * rs[c] : 0.0;
  if (r == 0) {
#pragma unroll
    for (int c = 0; c < 16; ++c) col[C0 + c] = rs[c];  // uniform across lanes
  }
}

// Trailing update after panel P (all waves): W[I][J] -= L[I][panel] L[J][panel]^T
// for the 16x16 blocks I >= J > P (lower triangle of blocks incl. the diagonal).
// Block q of the NBLK goes to wave q % nw (waves w >= nw skip).
template <int P>
__device__ __forceinline__ void panel_update(double* __restrict__ sF, int w, int nw = 4) {
  constexpr int NB = 3 - P, NBLK = NB * (NB + 1) / 2;
  for (int q = w; q < NBLK; q += nw) {
    int bi = 0;
    while ((bi + 1) * (bi + 2) / 2 <= q) ++bi;
    const int bj = q - bi * (bi + 1) / 2;
    const int R0 = 16 * (P + 1 + bi), C1 = 16 * (P + 1 + bj);
    doublex4 acc = blk_load(sF + R0 * LDT + C1);
    blk_mma<true>(acc, sF + R0 * LDT + 16 * P, sF + C1 * LDT + 16 * P, -1.0);
    blk_store(sF + R0 * LDT + C1, acc);
  }
}

// X_pp = L_pp^-1 of diagonal block p (one wave; needs col[16p ..] = 1 / L_rr).
// Lane cc (of 16; the other lanes duplicate) owns column cc of X and runs the
// right-looking forward substitution in registers: x_k = acc_k / L_kk, then
// acc_r -= L_rk x_k for r > k, with the L_rk wave-uniform LDS broadcasts.  The
// serial chain is one multiply and one FMA per row (the quad-layout version
// broadcast every pivot through DPP: ~5 K cycles, this one ~1 K).
__device__ __forceinline__ void inv_diag_block(const double* __restrict__ sF, double* __restrict__ sX,
                                               const double* __restrict__ col, int p, int lane) {
  const int cc = lane & 15;
  const double* L = sF + 16 * p * LDT + 16 * p;
  double acc[16], rs[16];
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    acc[r] = (r == cc) ? 1.0 : 0.0;
    rs[r] = col[16 * p + r];
  }
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    acc[k] *= rs[k];                      // x_k (final)
#pragma unroll
    for (int r = k + 1; r < 16; ++r) acc[r] = fma(-L[r * LDT + k], acc[k], acc[r]);
  }
  if (lane < 16) {
#pragma unroll
    for (int r = 0; r < 16; ++r) sX[(16 * p + r) * LDT + 16 * p + cc] = acc[r];
  }
}

// X_ij = -X_ii sum_{k=j}^{i-1} L_ik X_kj (one wave, f64 MFMA; the product's
// accumulator registers are directly the B operand of the second product).
__device__ __forceinline__ void inv_offdiag_block(const double* __restrict__ sF, double* __restrict__ sX, int i,
                                                  int j, int lane) {
  doublex4 y = {0.0, 0.0, 0.0, 0.0};
  for (int k = j; k < i; ++k) blk_mma<false>(y, sF + 16 * i * LDT + 16 * k, sX + 16 * k * LDT + 16 * j, 1.0);
  doublex4 xv = {0.0, 0.0, 0.0, 0.0};
  const double* Xii = sX + 16 * i * LDT + 16 * i;
#pragma unroll
  for (int s4 = 0; s4 < 4; ++s4) {
    const double av = -Xii[(lane & 15) * LDT + 4 * s4 + (lane >> 4)];
    xv = __builtin_amdgcn_mfma_f64_16x16x4f64(av, y[s4], xv, 0, 0, 0);
  }
  blk_store(sX + 16 * i * LDT + 16 * j, xv);
}

// -X_ii Y for Y in accumulator layout (the registers are the B operand as they stand).
__device__ __forceinline__ doublex4 neg_x_times(const double* __restrict__ Xii, const doublex4& y, int lane) {
  doublex4 xv = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
  for (int s4 = 0; s4 < 4; ++s4) {
    const double av = -Xii[(lane & 15) * LDT + 4 * s4 + (lane >> 4)];
    xv = __builtin_amdgcn_mfma_f64_16x16x4f64(av, y[s4], xv, 0, 0, 0);
  }
  return xv;
}

// Factor the symmetric 64x64 tile in sF (lower part used) in place: sF <- L
// (zeros above), sX <- L^-1 (zeros above).  Called by all 256 threads.
//
// Blocked in four 16-column panels: wave 0 factors a panel (register rows,
// readlane broadcasts, division-free chain), then the waves apply its rank-16
// update to the trailing blocks on the f64 MFMA.  The inverse is built by the
// idle waves while wave 0 runs the next panel: X_pp = L_pp^-1 as soon as panel
// p is final, X_ij (i > j) = -X_ii sum_k L_ik X_kj as soon as its operands are:
//   S0  w0 panel 0          | w1..w3 the caller's pending P P^T update of the
//                             blocks right of column block 0 (sPend, look-ahead)
//   U0  update 0 of column block 1 (w0..w2) | w3 zero the upper blocks of X
//   S1  w0 panel 1          | w1 X_00 | w2, w3 update 0 of blocks (2,2), (3,2), (3,3)
//   U1  update 1 of column block 2 (w0, w1)
//   S2  w0 panel 2          | w1 X_11 | w2 update 1 of block (3,3)
//   U2  update 2 (w0)       | w1 X_10
// (a trailing update runs on the critical path only for the column block the
// next panel sweeps; the rest runs beside that sweep)
//   S3  w0 panel 3          | w1 X_22, X_21 | w2 T_20 = L_20 X_00 + L_21 X_10,
//                                             T_30 = L_30 X_00 + L_31 X_10 | w3 T_31 = L_31 X_11
//   I1  w0 X_33             | w1 Y_32 = L_32 X_22 | w2 X_20 = -X_22 T_20 | w3 Y_31 = T_31 + L_32 X_21
//   I2  w0 X_32 = -X_33 Y_32 | w1 X_31 = -X_33 Y_31 | w2 X_30 = -X_33 (T_30 + L_32 X_20)
// (the sums over the already final blocks run beside panel 3; T / Y live in
// four of X's upper blocks, zeroed again by the wave that reads them last).
// Records the first non-positive pivot (LAPACK info, 1-based, + gcol0).
// sPend (optional, may alias sX): the caller's pending update sF -= sPend sPend^T
// of the lower blocks right of column block 0 (column block 0 already applied).
__device__ __forceinline__ void factor_diag_tile(double* __restrict__ sF, double* sX,
                                                 double* __restrict__ col, int32_t* info, int64_t gcol0,
                                                 const double* sPend = nullptr) {
  const int w = ctid() >> 6, lane = ctid() & 63;
  int bad = 0;
  const int js = (int)(gcol0 / CB) - 1;
  if (w == 0) {
    panel_factor<0>(sF, col, lane, bad);
  } else if (sPend) {  // blocks (1,1), (2,1) | (3,1), (2,2) | (3,2), (3,3)
    const int bi0 = (w == 1) ? 1 : 3, bj0 = (w == 3) ? 2 : 1;
    const int bi1 = (w == 3) ? 3 : 2, bj1 = (w == 1) ? 1 : (w == 2 ? 2 : 3);
    sub_outer_blk<4>(sF, 16 * bi0, 16 * bj0, sPend, sPend);
    sub_outer_blk<4>(sF, 16 * bi1, 16 * bj1, sPend, sPend);
  }
  STAMP(js, 8);
  __syncthreads();
  const double* P0 = sF;  // panel p's L columns: sF + 16 p
  if (w < 3) {
    sub_outer_blk<1>(sF, 16 * (w + 1), 16, P0, P0);  // update 0 of (1,1), (2,1), (3,1)
  } else {
    for (int q = 0; q < 6; ++q) {  // upper blocks (i < j) of X are zero
      const int i = q < 3 ? 0 : (q < 5 ? 1 : 2), j = q < 3 ? q + 1 : (q < 5 ? q - 1 : 3);
      blk_store(sX + 16 * i * LDT + 16 * j, doublex4{0.0, 0.0, 0.0, 0.0});
    }
  }
  __syncthreads();
  STAMP(js, 9);
  if (w == 0) {
    panel_factor<1>(sF, col, lane, bad);
  } else if (w == 1) {
    inv_diag_block(sF, sX, col, 0, lane);
  } else if (w == 2) {
    sub_outer_blk<1>(sF, 32, 32, P0, P0);  // update 0 of (2,2), (3,2)
    sub_outer_blk<1>(sF, 48, 32, P0, P0);
  } else {
    sub_outer_blk<1>(sF, 48, 48, P0, P0);  // update 0 of (3,3)
  }
  STAMP(js, 10);
  __syncthreads();
  if (w < 2) sub_outer_blk<1>(sF, 32 + 16 * w, 32, sF + 16, sF + 16);  // update 1 of (2,2), (3,2)
  __syncthreads();
  STAMP(js, 11);
  if (w == 0) panel_factor<2>(sF, col, lane, bad);
  else if (w == 1) inv_diag_block(sF, sX, col, 1, lane);
  else if (w == 2) sub_outer_blk<1>(sF, 48, 48, sF + 16, sF + 16);  // update 1 of (3,3)
  STAMP(js, 12);
  __syncthreads();
  if (w == 0) panel_update<2>(sF, 0, 1);
  else if (w == 1) inv_offdiag_block(sF, sX, 1, 0, lane);
  __syncthreads();
  auto L_ = [&](int bi, int bj) { return sF + 16 * bi * LDT + 16 * bj; };
  auto X_ = [&](int bi, int bj) { return sX + 16 * bi * LDT + 16 * bj; };
  // scratch: T_20 -> X(0,1), T_30 -> X(0,2), T_31 / Y_31 -> X(0,3), Y_32 -> X(1,2)
  auto S_ = [&](int bi, int bj) {
    const int q = (bi == 2) ? 1 : (bj == 0 ? 2 : (bj == 1 ? 3 : 6));
    return sX + 16 * (q >> 2) * LDT + 16 * (q & 3);
  };
  const doublex4 zero4 = {0.0, 0.0, 0.0, 0.0};
  if (w == 0) {
    panel_factor<3>(sF, col, lane, bad);
    if (bad && lane == 0) atomicCAS(info, 0, (int32_t)(gcol0 + bad));
  } else if (w == 1) {
    inv_diag_block(sF, sX, col, 2, lane);
    inv_offdiag_block(sF, sX, 2, 1, lane);
  } else if (w == 2) {
    doublex4 t = {0.0, 0.0, 0.0, 0.0};
    blk_mma<false>(t, L_(2, 0), X_(0, 0), 1.0);
    blk_mma<false>(t, L_(2, 1), X_(1, 0), 1.0);
    blk_store(S_(2, 0), t);
    t = doublex4{0.0, 0.0, 0.0, 0.0};
    blk_mma<false>(t, L_(3, 0), X_(0, 0), 1.0);
    blk_mma<false>(t, L_(3, 1), X_(1, 0), 1.0);
    blk_store(S_(3, 0), t);
  } else {
    doublex4 t = {0.0, 0.0, 0.0, 0.0};
    blk_mma<false>(t, L_(3, 1), X_(1, 1), 1.0);
    blk_store(S_(3, 1), t);
  }
  __syncthreads();
  STAMP(js, 5);
  if (w == 0) {
    inv_diag_block(sF, sX, col, 3, lane);
  } else if (w == 1) {
    doublex4 y = {0.0, 0.0, 0.0, 0.0};
    blk_mma<false>(y, L_(3, 2), X_(2, 2), 1.0);
    blk_store(S_(3, 2), y);
  } else if (w == 2) {
    const doublex4 t = blk_load(S_(2, 0));
    blk_store(S_(2, 0), zero4);
    blk_store(X_(2, 0), neg_x_times(X_(2, 2), t, lane));
  } else {
    doublex4 y = blk_load(S_(3, 1));
    blk_mma<false>(y, L_(3, 2), X_(2, 1), 1.0);
    blk_store(S_(3, 1), y);
  }
  __syncthreads();
  STAMP(js, 13);
  if (w == 0) {
    const doublex4 y = blk_load(S_(3, 2));
    blk_store(S_(3, 2), zero4);
    blk_store(X_(3, 2), neg_x_times(X_(3, 3), y, lane));
  } else if (w == 1) {
    const doublex4 y = blk_load(S_(3, 1));
    blk_store(S_(3, 1), zero4);
    blk_store(X_(3, 1), neg_x_times(X_(3, 3), y, lane));
  } else if (w == 2) {
    doublex4 y = blk_load(S_(3, 0));
    blk_store(S_(3, 0), zero4);
    blk_mma<false>(y, L_(3, 2), X_(2, 0), 1.0);
    blk_store(X_(3, 0), neg_x_times(X_(3, 3), y, lane));
  }
  __syncthreads();
}

// Write the factored diagonal tile j: L block (f32, guarded to M; optional) and D_j (f64).
// Full tiles with 16-B stores (ld of L is a multiple of 4, tile origins 64-aligned).
__device__ __forceinline__ void write_diag(const CholArgs& a, int b, int j, const double* sF, const double* sX) {
  const int64_t g0 = (int64_t)j * CB;
  const int nr = (int)min<int64_t>(CB, a.M - g0);
  if (a.L) {
    float* g = a.L + (int64_t)b * a.strideL + g0 * a.ldl + g0;
    if (nr == CB) {
#pragma unroll
      for (int it = 0; it < 4; ++it) {
        const int idx = ctid() + kCholThreads * it, r = idx >> 4, c = (idx & 15) * 4;
        const double* sr = sF + r * LDT + c;
        *reinterpret_cast<float4*>(g + (int64_t)r * a.ldl + c) =
            make_float4((float)sr[0], (float)sr[1], (float)sr[2], (float)sr[3]);
      }
    } else {
      tile_store_f32(g, a.ldl, sF, false, nr, nr);
    }
  }
  double* d = ws_D(a, b, j);
#pragma unroll
  for (int it = 0; it < 8; ++it) {
    const int idx = ctid() + kCholThreads * it, r = idx >> 5, c = (idx & 31) * 2;
    *reinterpret_cast<double2*>(d + r * CB + c) = make_double2(sX[r * LDT + c], sX[r * LDT + c + 1]);
  }
}

// ------------------------------------------------------------------ persistent-path task order
// The single-launch factorisation (chol_persist) runs the tile work of all steps
// from one task table; every product is formed once and handed on through the
// workspace (no per-tile recomputation).  Task kinds (nb = Mp / 64 tile rows):
//   PAN(i, j)   L_ij = W_ij D_j^T, in place of W_ij (i >= j + 2; L_{j+1,j} is the chain's);
//   U(i, l, j)  trailing update W_il -= L_ij L_lj^T of step j (j < l <= i), except the
//               look-ahead tile (j+1, j+1), which the chain updates and factors;
//   XR(j, c)    row block j of X = L^-1: X_jc = D_j B_jc, in place of B_jc (c < j);
//   FU(i, c, j) forward substitution B_ic -= L_ij X_jc (i > j, c <= j; X_jj = D_j).
// Order per step j: the tasks the chain's next step waits for (PAN(j+2, j),
// U(j+2, j+1, j), U(j+2, j+2, j)), the other panels, the other updates by column;
// the forward-substitution work of step j (F_j = XR(j, .), FU(., ., j)), needed only
// at the end, one step later:  A_0 B_0 C_0, A_1 B_1 C_1, F_0, A_2 B_2 C_2, F_1, ...,
// F_{nb-2}, XR(nb-1, .).  Every dependency of a task lies earlier in the table or is
// a chain output whose own inputs do, so in-order dequeueing cannot deadlock.
enum { kTaskPan = 0, kTaskU = 1, kTaskXR = 2, kTaskFU = 3 };

// block q: q < 4 (nb - 1): step j = q / 4, slot s = q % 4 (A_j, B_j, C_j, F_{j-1});
// then F_{nb-2}, then the last row.
__host__ __device__ inline int task_block_count(int nb) { return 4 * (nb - 1) + 2; }
__host__ __device__ inline int task_block_size(int q, int nb) {
  if (q < 4 * (nb - 1)) {
    const int j = q / 4, slot = q % 4, T = nb - 1 - j;
    if (slot == 0) return T >= 2 ? 3 : 0;
    if (slot == 1) return T >= 3 ? T - 2 : 0;
    if (slot == 2) return T * (T + 1) / 2 - 1 - (T >= 2 ? 2 : 0);
    return j >= 1 ? (j - 1) + (nb - j) * j : 0;      // F_{j-1}
  }
  if (q == 4 * (nb - 1)) return nb >= 2 ? (nb - 2) + (nb - 1 - (nb - 2)) * (nb - 1) : 0;   // F_{nb-2}
  return nb - 1;                                                                          // XR(nb-1, .)
}
__host__ __device__ inline int task_count(int nb) {
  int n = 0;
  for (int q = 0; q < task_block_count(nb); ++q) n += task_block_size(q, nb);
  return n;
}
__host__ __device__ inline int task_encode(int kind, int j, int i, int l) {
  return (kind << 24) | (j << 16) | (i << 8) | l;
}
// entry e of the forward-substitution block F_j
__device__ __forceinline__ int task_f(int j, int e) {
  if (e < j) return task_encode(kTaskXR, j, j, e);
  e -= j;
  return task_encode(kTaskFU, j, j + 1 + e / (j + 1), e % (j + 1));
}
__device__ __forceinline__ int task_entry(int q, int e, int nb) {
  if (q < 4 * (nb - 1)) {
    const int j = q / 4, slot = q % 4, T = nb - 1 - j;
    if (slot == 0) {
      if (e == 0) return task_encode(kTaskPan, j, j + 2, j);
      return task_encode(kTaskU, j, j + 2, e == 1 ? j + 1 : j + 2);
    }
    if (slot == 1) return task_encode(kTaskPan, j, j + 3 + e, j);
    if (slot == 2) {
      // the column-major triangle (l = j+1 .., i = l ..) without (j+1, j+1), (j+2, j+1), (j+2, j+2)
      int f = e + 2;
      if (T >= 2 && f >= T) ++f;                       // (j+2, j+2) sits at f = T
      int l = j + 1;
      while (f >= nb - l) { f -= nb - l; ++l; }
      return task_encode(kTaskU, j, l + f, l);
    }
    return task_f(j - 1, e);
  }
  if (q == 4 * (nb - 1)) return task_f(nb - 2, e);
  return task_encode(kTaskXR, nb - 1, nb - 1, e);
}

// Per-batch sync words of the persistent path: Wver[nb][nb] (tile (i, l) of W: the
// number of updates applied, then l + 1 once it holds L_il), Bver[nb][nb] (tile
// (i, c) of B: updates applied, then +1 once it holds X_ic), Dready[nb], head (next
// task), err (a bounded wait gave up).
__host__ __device__ inline int64_t chol_sync_words(int nb) { return ((int64_t)2 * nb * nb + nb + 2 + 63) / 64 * 64; }

// chol_prep's share of the persistent state: zero this batch's sync words (Dready[0]
// = 1: prep factors tile (0, 0)) and, for batch 0, fill the task table (block q of
// the order by workgroup q).
__device__ __forceinline__ void prep_persist_state(const CholArgs& a, int b) {
  const int nb = a.nb;
  int* s = a.sync + (int64_t)b * a.strideSync;
  const int64_t nw = chol_sync_words(nb), d0 = (int64_t)2 * nb * nb;
  for (int64_t w = (int64_t)blockIdx.x * kCholThreads + ctid(); w < nw; w += (int64_t)gridDim.x * kCholThreads)
    s[w] = (w == d0) ? 1 : 0;
  const int q = blockIdx.x;
  if (b != 0 || q >= task_block_count(nb)) return;
  int start = 0;
  for (int r = 0; r < q; ++r) start += task_block_size(r, nb);
  const int n = task_block_size(q, nb);
  for (int e = ctid(); e < n; e += kCholThreads) a.tasks[start + e] = task_entry(q, e, nb);
}

// ------------------------------------------------------------------ prep launch
__global__ __launch_bounds__(kCholThreads) void chol_prep(CholArgs a) {
  __shared__ double s1[CB * LDT], s2[CB * LDT], col[CB];
  __shared__ double sil[32];
  const int b = blockIdx.y;
  const float* Zb = a.Z[0];
  double varb = 0.0;
  if (!a.A) {  // Kuu from Z: select this batch entry (no dynamic indexing of the argument arrays)
    const float *ls = a.ls[0], *var = a.var[0];
    int nls = a.n_ls[0];
#pragma unroll
    for (int i = 1; i < kMaxBatch; ++i)
      if (b == i) { Zb = a.Z[i]; ls = a.ls[i]; var = a.var[i]; nls = a.n_ls[i]; }
    if (threadIdx.x < a.D) sil[threadIdx.x] = 1.0 / (double)ls[nls == 1 ? 0 : threadIdx.x];
    varb = (double)var[0];
    __syncthreads();
  }
  auto elem = [&](int64_t gr, int64_t gc) {
    return a.A ? input_elem(a, b, gr, gc) : kuu_elem(a, Zb, sil, varb, gr, gc);
  };
  if (a.sync) prep_persist_state(a, b);
  if (blockIdx.x == 0) {  // factor tile (0, 0) straight from the input (dispatched first)
    if (threadIdx.x == 0) {
      a.info[b] = 0;
      float* lt = a.lt_absmax[0];
#pragma unroll
      for (int i = 1; i < kMaxBatch; ++i)
        if (b == i) lt = a.lt_absmax[i];
      if (lt) *lt = 0.f;
    }
    for (int idx = threadIdx.x; idx < CB * CB; idx += kCholThreads) {
      const int r = idx >> 6, c = idx & 63;
      s1[r * LDT + c] = elem(r, c);
    }
    __syncthreads();
    factor_diag_tile(s1, s2, col, a.info + b, 0);
    __syncthreads();
    write_diag(a, b, 0, s1, s2);
    return;
  }
  const int bi = (blockIdx.x - 1) / a.nb, bl = (blockIdx.x - 1) % a.nb;
  const int64_t r0 = (int64_t)bi * CB, c0 = (int64_t)bl * CB;
  if (bl <= bi) {
    double* W = ws_W(a, b) + r0 * a.Mp + c0;
    for (int idx = threadIdx.x; idx < CB * CB; idx += kCholThreads) {
      const int r = idx >> 6, c = idx & 63;
      W[(int64_t)r * a.Mp + c] = elem(r0 + r, c0 + c);
    }
  }
  // zero L above / LinvT below the block diagonal (within M x M)
  if (bl != bi && (bl < bi || a.L)) {
    float* dst = (bl > bi ? a.L : a.LinvT) + (int64_t)b * a.strideL;
    for (int idx = threadIdx.x; idx < CB * CB; idx += kCholThreads) {
      const int r = idx >> 6, c = idx & 63;
      const int64_t gr = r0 + r, gc = c0 + c;
      if (gr < a.M && gc < a.M) dst[gr * a.ldl + gc] = 0.f;
    }
  }
}

// ------------------------------------------------------------------ step launch j
// The look-ahead's factorisation of tile (j+1, j+1): s1 holds P = L_{j+1,j}, s2 the
// tile with column block 0 of -P P^T still to apply.
__device__ __forceinline__ void lookahead_factor(const CholArgs& a, int b, int j, double* s1, double* s2,
                                                 double* col) {
  // column block 0 of W_ii -= P_i P_i^T (one block per wave); the other six
  // lower blocks are applied beside the first panel sweep
  sub_outer_blk<4>(s2, 16 * (threadIdx.x >> 6), 0, s1, s1);
  __syncthreads();
  STAMP(j, 3);
  STAMP(j, 4);
  factor_diag_tile(s2, s1, col, a.info + b, (int64_t)(j + 1) * CB, s1);
  STAMP(j, 6);
  __syncthreads();
  write_diag(a, b, j + 1, s2, s1);
  __syncthreads();
  STAMP(j, 7);
  RSTAMP(j, 15);
}

__global__ __launch_bounds__(kCholThreads) void chol_step(CholArgs a, int j) {
  __shared__ double s1[CB * LDT], s2[CB * LDT], sD[CB * LDT], col[CB];
  const int b = blockIdx.y;
  const int T = a.nb - j - 1;
  const int nU = T * (T + 1) / 2;
  const int idx = blockIdx.x;
  double* W = ws_W(a, b);
  double* Bm = ws_B(a, b);
  float* LinvT = a.LinvT + (int64_t)b * a.strideL;
  const int64_t Mp = a.Mp;
  auto Wt = [&](int bi, int bl) { return W + (int64_t)bi * CB * Mp + (int64_t)bl * CB; };
  auto Bt = [&](int bi, int bl) { return Bm + (int64_t)bi * CB * Mp + (int64_t)bl * CB; };
  float* lt_max = a.lt_absmax[0];  // this batch entry's max |L^-T| (no dynamic indexing of the arguments)
#pragma unroll
  for (int q = 1; q < kMaxBatch; ++q)
    if (b == q) lt_max = a.lt_absmax[q];
  auto store_linvT = [&](int c, const double* sx) {  // X_jc -> LinvT block (c, j)
    const int64_t gr = (int64_t)c * CB, gc = (int64_t)j * CB;
    const float m = tile_store_f32_max(LinvT + gr * a.ldl + gc, a.ldl, sx, true, (int)min<int64_t>(CB, a.M - gr),
                                       (int)min<int64_t>(CB, a.M - gc));
    if (lt_max) wave_absmax_atomic(m, lt_max);
  };

  if (T == 0) {  // last step: row block j of X only
    const int c = idx;
    tile_load(sD, ws_D(a, b, j), CB);
    if (c < j) tile_load(s1, Bt(j, c), Mp);
    __syncthreads();
    if (c < j) {
      Blk4 x = blk4_zero();
      col_mma_lower(x, sD, s1);
      __syncthreads();
      blk4_to_lds<false>(s1, x);
      __syncthreads();
      store_linvT(c, s1);
    } else {
      store_linvT(c, sD);
    }
    return;
  }

  if (idx < nU) {  // ---------------- trailing update tile (i, l), j < l <= i
    int ai = 0;
    while ((ai + 1) * (ai + 2) / 2 <= idx) ++ai;
    const int bl_ = idx - ai * (ai + 1) / 2;
    const int i = j + 1 + ai, l = j + 1 + bl_;
    const bool la = (ai == 0 && bl_ == 0);
    if (la) { RSTAMP(j, 14); STAMP(j, 0); }
    TileRegs r1, rD, r2;
    Blk4 u;
    tile_fetch(r1, Wt(i, j), Mp);
    tile_fetch(rD, ws_D(a, b, j), CB);
    tile_fetch(r2, (l != i) ? Wt(l, j) : Wt(i, l), Mp);  // P_l's operand, or the diagonal tile itself
    if (l != i) row_from_global(u, Wt(i, l), Mp);      // the updated tile, in flight with the operands
    tile_put(s1, r1);
    tile_put(sD, rD);
    tile_put(s2, r2);
    __syncthreads();
    if (la) STAMP(j, 1);
    Blk4 pi = blk4_zero(), pl = blk4_zero();
    row_mma<true, 1>(pi, s1, sD, 1.0);                 // P_i = W_ij D_j^T (D lower: 40 MFMAs/wave)
    if (l != i) row_mma<true, 1>(pl, s2, sD, 1.0);     // P_l
    __syncthreads();
    blk4_to_lds<true>(s1, pi);
    if (l != i) blk4_to_lds<true>(s2, pl);
    __syncthreads();
    if (la) STAMP(j, 2);
    if (l == i && !la && a.L) {  // L_ij (the look-ahead's L_{j+1,j}: by forward-substitution tile (j+1, j))
      const int64_t gr = (int64_t)i * CB, gc = (int64_t)j * CB;
      tile_store_f32(a.L + (int64_t)b * a.strideL + gr * a.ldl + gc, a.ldl, s1, false,
                     (int)min<int64_t>(CB, a.M - gr), (int)min<int64_t>(CB, a.M - gc));
    }
    if (l != i) {
      row_mma<true, 0>(u, s1, s2, -1.0);               // W_il -= P_i P_l^T
      row_to_global(Wt(i, l), Mp, u);
      return;
    }
    if (la) {  // look-ahead: factor the next diagonal tile
      lookahead_factor(a, b, j, s1, s2, col);
    } else {
      // diagonal tile (i, i): lower blocks of W_ii -= P_i P_i^T in place in LDS (s2)
      diag_lower_update(s2, s1);
      __syncthreads();
      tile_store_f64(Wt(i, l), Mp, s2);
    }
    return;
  }

  // ------------------ forward-substitution tile (i, c), i > j, c <= j
  const int x = idx - nU;
  const int i = j + 1 + x / (j + 1), c = x % (j + 1);
  TileRegs r1, rD, r2;
  Blk4 u = blk4_zero();
  tile_fetch(r1, Wt(i, j), Mp);
  tile_fetch(rD, ws_D(a, b, j), CB);
  if (c < j) {
    tile_fetch(r2, Bt(j, c), Mp);
    row_from_global(u, Bt(i, c), Mp);
  }
  tile_put(s1, r1);
  tile_put(sD, rD);
  if (c < j) tile_put(s2, r2);
  __syncthreads();
  Blk4 pi = blk4_zero(), xq = blk4_zero();
  row_mma<true, 1>(pi, s1, sD, 1.0);                   // P_i
  if (c < j) col_mma_lower(xq, sD, s2);                // X_jc = D_j B_jc
  __syncthreads();
  blk4_to_lds<true>(s1, pi);
  if (c < j) blk4_to_lds<false>(s2, xq);
  __syncthreads();
  if (i == j + 1 && c == j && a.L) {                   // L_{j+1,j} (off the look-ahead's chain)
    const int64_t gr = (int64_t)i * CB, gc = (int64_t)j * CB;
    tile_store_f32(a.L + (int64_t)b * a.strideL + gr * a.ldl + gc, a.ldl, s1, false,
                   (int)min<int64_t>(CB, a.M - gr), (int)min<int64_t>(CB, a.M - gc));
  }
  if (c < j) {
    if (i == j + 1) store_linvT(c, s2);
    row_mma<false, 0>(u, s1, s2, -1.0);                // B_ic -= P_i X_jc
  } else {                                             // X_jj = D_j (lower triangular)
    if (i == j + 1) store_linvT(c, sD);
    row_mma<false, 2>(u, s1, sD, -1.0);
  }
  row_to_global(Bt(i, c), Mp, u);
}

// ------------------------------------------------------------------ step launch j, tile pairs
// chol_step with the trailing-update and forward-substitution tiles of step j taken two
// at a time along a tile row i, one 256-thread group per tile in a 512-thread
// workgroup (workgroup 0 is the look-ahead, on its first group).  chol_step's tile
// workgroups each form P_i = W_ij D_j^T for themselves and run their three products
// with one wave per SIMD; here the pair loads W_ij and D_j once, each group forms half
// of P_i's column blocks and then its tile's own first product (P_l or X_jc), and the
// two groups' MFMAs share every SIMD (two waves each), so a step's tiles take half the
// workgroups for about the time of one.  Per tile the products are chol_step's, on the same
// operands in the same order: L and L^-T are bit-identical.
// After P_i the groups take their tiles' own paths: a __syncthreads on one path waits
// for the live waves of both groups wherever they are, so it still orders that group's
// own LDS hand-off (and a group that has ended is not waited for: a barrier counts only
// the waves that have not terminated).
// Row i's tiles in order: the update tiles (i, l), l = j + 1 .. i (rows i > j + 1;
// l = i is the diagonal tile), then the forward-substitution tiles (i, c), c = 0 .. j.
constexpr int kPairThreads = 2 * kCholThreads;
__host__ __device__ inline int step_row_tiles(int i, int j) { return i == j + 1 ? j + 1 : i + 1; }
__host__ __device__ inline int step_pair_count(int nb, int j) {
  int n = 0;
  for (int i = j + 1; i < nb; ++i) n += (step_row_tiles(i, j) + 1) / 2;
  return n;
}

__global__ __launch_bounds__(kPairThreads) void chol_step_pair(CholArgs a, int j) {
  __shared__ double s1[CB * LDT], sD[CB * LDT], s2[2][CB * LDT], col[CB];
  const int b = blockIdx.y;
  const int g = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 8));  // tile group
  double* W = ws_W(a, b);
  double* Bm = ws_B(a, b);
  float* LinvT = a.LinvT + (int64_t)b * a.strideL;
  const int64_t Mp = a.Mp;
  auto Wt = [&](int bi, int bl) { return W + (int64_t)bi * CB * Mp + (int64_t)bl * CB; };
  auto Bt = [&](int bi, int bl) { return Bm + (int64_t)bi * CB * Mp + (int64_t)bl * CB; };
  float* lt_max = a.lt_absmax[0];
#pragma unroll
  for (int q = 1; q < kMaxBatch; ++q)
    if (b == q) lt_max = a.lt_absmax[q];
  auto store_linvT = [&](int c, const double* sx) {  // X_jc -> LinvT block (c, j)
    const int64_t gr = (int64_t)c * CB, gc = (int64_t)j * CB;
    const float m = tile_store_f32_max(LinvT + gr * a.ldl + gc, a.ldl, sx, true, (int)min<int64_t>(CB, a.M - gr),
                                       (int)min<int64_t>(CB, a.M - gc));
    if (lt_max) wave_absmax_atomic(m, lt_max);
  };
  int i = j + 1;
  if (blockIdx.x == 0) {  // look-ahead: tile (j+1, j+1), group 0 (group 1's waves end here:
    if (g != 0) return;   // a barrier waits only for the waves that have not terminated)
    RSTAMP(j, 14);
    STAMP(j, 0);
    TileRegs r1, rD, r2;
    tile_fetch(r1, Wt(i, j), Mp);
    tile_fetch(rD, ws_D(a, b, j), CB);
    tile_fetch(r2, Wt(i, i), Mp);
    tile_put(s1, r1);
    tile_put(sD, rD);
    tile_put(s2[0], r2);
    __syncthreads();
    STAMP(j, 1);
    Blk4 pi = blk4_zero();
    row_mma<true, 1>(pi, s1, sD, 1.0);
    __syncthreads();
    blk4_to_lds<true>(s1, pi);
    __syncthreads();
    STAMP(j, 2);
    lookahead_factor(a, b, j, s1, s2[0], col);
    return;
  }
  // pair -> (row i, tile e of the row)
  int q = blockIdx.x - 1, nt = 0;
  for (; i < a.nb; ++i) {
    nt = step_row_tiles(i, j);
    const int np = (nt + 1) / 2;
    if (q < np) break;
    q -= np;
  }
  const int e = 2 * q + g;
  const bool has = e < nt;  // an odd row's last pair: group 1 has no tile (it forms its half of P_i)
  const int nupd = (i == j + 1) ? 0 : i - j;
  const bool upd = has && e < nupd;
  const int l = j + 1 + e, c = e - nupd;
  const bool fwd = has && !upd && c < j;  // forward-substitution tile reading B_jc
  const bool first = (upd && l != i) || fwd;  // P_l / X_jc before the update
  double* sT = s2[g];
  // this tile's operands: sT's tile (when it reads one) and the updated tile (u)
  TileRegs r1, rD, r2;
  Blk4 u = blk4_zero();  // B_ij is zero before step j
  if (g == 0) {
    tile_fetch(r1, Wt(i, j), Mp);
    tile_fetch(rD, ws_D(a, b, j), CB);
  }
  if (upd) {
    if (l != i) {
      tile_fetch(r2, Wt(l, j), Mp);
      row_from_global(u, Wt(i, l), Mp);
    } else {
      tile_fetch(r2, Wt(i, i), Mp);
    }
  } else if (fwd) {
    tile_fetch(r2, Bt(j, c), Mp);
    row_from_global(u, Bt(i, c), Mp);
  }
  if (g == 0) {
    tile_put(s1, r1);
    tile_put(sD, rD);
  }
  if (upd || fwd) tile_put(sT, r2);
  __syncthreads();
  // P_i's column blocks split over the groups with equal MFMA counts (D_j^T upper:
  // block tj takes 4 (tj + 1) k-steps): group 0 blocks 0 and 3, group 1 blocks 1 and 2;
  // each group then forms its tile's own first product
  Blk4 pi = blk4_zero(), t = blk4_zero();
  if (g == 0) row_mma<true, 1, 0x9>(pi, s1, sD, 1.0);  // P_i = W_ij D_j^T = L_ij
  else row_mma<true, 1, 0x6>(pi, s1, sD, 1.0);
  if (first) {
    if (upd) row_mma<true, 1>(t, sT, sD, 1.0);   // P_l = W_lj D_j^T
    else col_mma_lower(t, sD, sT);               // X_jc = D_j B_jc
  }
  __syncthreads();
  if (g == 0) blk4_to_lds<true, 0x9>(s1, pi);
  else blk4_to_lds<true, 0x6>(s1, pi);
  if (first) upd ? blk4_to_lds<true>(sT, t) : blk4_to_lds<false>(sT, t);
  __syncthreads();
  if (g == 0 && q == 0 && a.L) {  // L_ij, once per row
    const int64_t gr = (int64_t)i * CB, gc = (int64_t)j * CB;
    tile_store_f32(a.L + (int64_t)b * a.strideL + gr * a.ldl + gc, a.ldl, s1, false,
                   (int)min<int64_t>(CB, a.M - gr), (int)min<int64_t>(CB, a.M - gc));
  }
  if (!has) return;
  if (upd && l != i) {
    row_mma<true, 0>(u, s1, sT, -1.0);    // W_il -= P_i P_l^T
    row_to_global(Wt(i, l), Mp, u);
  } else if (upd) {                        // diagonal tile (i, i): lower blocks of W_ii -= P_i P_i^T
    diag_lower_update(sT, s1);
    __syncthreads();
    tile_store_f64(Wt(i, i), Mp, sT);
  } else if (fwd) {
    if (i == j + 1) store_linvT(c, sT);
    row_mma<false, 0>(u, s1, sT, -1.0);    // B_ic -= P_i X_jc
    row_to_global(Bt(i, c), Mp, u);
  } else {                                 // X_jj = D_j (lower triangular)
    if (i == j + 1) store_linvT(c, sD);
    row_mma<false, 2>(u, s1, sD, -1.0);
    row_to_global(Bt(i, c), Mp, u);
  }
}

// ------------------------------------------------------------------ persistent launch
// chol_persist: the nb - 1 steps after chol_prep in ONE launch.  Per batch entry,
// workgroup 0 is the CHAIN: it keeps D_j in LDS and, step after step, forms the
// look-ahead panel P = W_{j+1,j} D_j^T, applies P P^T to W_{j+1,j+1}, factors it
// (factor_diag_tile) and publishes D_{j+1}; it never waits for a launch boundary.
// Workgroups 1.. are WORKERS: they take tasks from the table in order (one
// returning atomic add per task) and wait only for the tiles and D a task reads.
// Hand-offs (MI355X_MICROARCH.md, inter-workgroup visibility, the flag form with
// sc1 payload): every byte another workgroup reads is stored write-through (sc1) by
// 8/16-B buffer stores, every storing wave drains vmcnt(0), the workgroup barrier,
// then ONE lane's relaxed agent-scope store of the version / ready word; consumers
// poll with relaxed agent loads (sc1) and read every handed-off byte with sc1
// buffer loads (no acquire fence needed).  Every wait is bounded: on a give-up the
// workgroup records err and info and leaves.
typedef __attribute__((address_space(1))) int gint;
constexpr int kSc1 = 16;                 // buffer instruction aux bits: sc1
constexpr uint32_t kSpinLimit = 1u << 22;  // polls (~s_sleep 2 each) before a wait gives up

// sc1 buffer accesses: voff = this lane's part of the offset (a VGPR), soff = the
// wave-uniform part (an SGPR: tile origin + compile-time element offsets)
__device__ __forceinline__ double2 ld16c(__amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff) {
  return __builtin_bit_cast(double2, __builtin_amdgcn_raw_buffer_load_b128(r, voff, soff, kSc1));
}
__device__ __forceinline__ double ld8c(__amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff) {
  return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(r, voff, soff, kSc1));
}
__device__ __forceinline__ void st16c(__amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff, double x, double y) {
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4v, make_double2(x, y)), r, voff, soff, kSc1);
}
__device__ __forceinline__ void st8c(__amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff, double x) {
  typedef unsigned int u32x2v __attribute__((ext_vector_type(2)));
  __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2v, x), r, voff, soff, kSc1);
}
// Lane offsets (bytes) of the two access patterns within a tile of leading dimension ld:
//   pair pattern (tile_fetch / tile_store): element (tid / 32 + 8 it, 2 (tid % 32)), soff += 64 it ld
//   row-stripe accumulator pattern (Blk4, blk4_foreach<true>): (16 w + lane / 16 + 4 q, 16 t + lane % 16)
__device__ __forceinline__ uint32_t lane_off_pair(int64_t ld) {
  return (uint32_t)((((int)threadIdx.x >> 5) * ld + (threadIdx.x & 31) * 2) * 8);
}
__device__ __forceinline__ uint32_t lane_off_row(int64_t ld) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  return (uint32_t)(((16 * w + (lane >> 4)) * ld + (lane & 15)) * 8);
}
// 64x64 f64 tile at byte offset `off` (leading dimension ld doubles), sc1 loads
__device__ __forceinline__ void tile_fetch_c(TileRegs& t, __amdgpu_buffer_rsrc_t r, uint32_t off, int64_t ld) {
  const uint32_t v = lane_off_pair(ld);
#pragma unroll
  for (int it = 0; it < 8; ++it) t.v[it] = ld16c(r, v, off + (uint32_t)(it * 64 * ld));
}
__device__ __forceinline__ void row_from_global_c(Blk4& u, __amdgpu_buffer_rsrc_t r, uint32_t off, int64_t ld) {
  const uint32_t v = lane_off_row(ld);
#pragma unroll
  for (int t = 0; t < 4; ++t)
#pragma unroll
    for (int q = 0; q < 4; ++q) u.c[t][q] = ld8c(r, v, off + (uint32_t)((4 * q * ld + 16 * t) * 8));
}
__device__ __forceinline__ void row_to_global_c(__amdgpu_buffer_rsrc_t r, uint32_t off, int64_t ld, const Blk4& u) {
  const uint32_t v = lane_off_row(ld);
#pragma unroll
  for (int t = 0; t < 4; ++t)
#pragma unroll
    for (int q = 0; q < 4; ++q) st8c(r, v, off + (uint32_t)((4 * q * ld + 16 * t) * 8), u.c[t][q]);
}
__device__ __forceinline__ void tile_store_c(__amdgpu_buffer_rsrc_t r, uint32_t off, int64_t ld, const double* s) {
  const uint32_t v = lane_off_pair(ld);
  const int rr = threadIdx.x >> 5, c = (threadIdx.x & 31) * 2;
#pragma unroll
  for (int it = 0; it < 8; ++it)
    st16c(r, v, off + (uint32_t)(it * 64 * ld), s[(rr + 8 * it) * LDT + c], s[(rr + 8 * it) * LDT + c + 1]);
}
__device__ __forceinline__ int flag_load(const int* p) {
  return __hip_atomic_load((gint*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void flag_store(int* p, int v) {
  __hip_atomic_store((gint*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// All threads: wait until every word p[k] >= v[k] (k < n <= 4; one lane polls each),
// then the workgroup barrier.  Returns false (uniformly) when a wait gave up.
__device__ __forceinline__ bool wait_all(const int* const (&p)[4], const int (&v)[4], int n, int* err,
                                         int* s_flag) {
  if (threadIdx.x < 64) {
    const int lane = threadIdx.x;
    const int* mp = p[0];
    int mv = v[0];
#pragma unroll
    for (int k = 1; k < 4; ++k)
      if (lane == k) { mp = p[k]; mv = v[k]; }
    bool ok = true;
    for (uint32_t it = 0;; ++it) {
      const bool mine = lane >= n || flag_load(mp) >= mv;
      if (__all(mine)) break;
      if (it >= kSpinLimit || flag_load(err) != 0) {
        ok = false;
        break;
      }
      __builtin_amdgcn_s_sleep(2);
    }
    if (lane == 0) {
      *s_flag = ok ? 1 : 0;
      if (!ok) __hip_atomic_store((gint*)err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  __syncthreads();
  const bool ok = *s_flag != 0;
  __syncthreads();
  return ok;
}

// All threads: one poll of the words (no wait); true (uniformly) when every p[k] >= v[k].
__device__ __forceinline__ bool poll_all(const int* const (&p)[4], const int (&v)[4], int n, int* s_flag) {
  if (threadIdx.x < 64) {
    const int lane = threadIdx.x;
    const int* mp = p[0];
    int mv = v[0];
#pragma unroll
    for (int k = 1; k < 4; ++k)
      if (lane == k) { mp = p[k]; mv = v[k]; }
    const bool mine = lane >= n || flag_load(mp) >= mv;
    const bool all = __all(mine);
    if (lane == 0) *s_flag = all ? 1 : 0;
  }
  __syncthreads();
  const bool ok = *s_flag != 0;
  __syncthreads();
  return ok;
}

// every storing wave drains its sc1 stores, then one lane publishes `v` at p
__device__ __forceinline__ void publish(int* p, int v) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) flag_store(p, v);
}

__global__ __launch_bounds__(kCholThreads) void chol_persist(CholArgs a) {
  __shared__ double bufA[CB * LDT], bufB[CB * LDT], bufC[CB * LDT], col[CB];
  __shared__ int s_task, s_flag;
  const int b = blockIdx.y, nb = a.nb;
  const int64_t Mp = a.Mp;
  int* sync = a.sync + (int64_t)b * a.strideSync;
  int* Wver = sync;
  int* Bver = sync + nb * nb;
  int* Dready = sync + 2 * nb * nb;
  int* head = Dready + nb;
  int* err = head + 1;
  const __amdgpu_buffer_rsrc_t R = __builtin_amdgcn_make_buffer_rsrc(
      (void*)ws_W(a, b), (short)0, (int)(uint32_t)(a.strideWS * 8), 0x00020000);
  auto offW = [&](int i, int l) { return (uint32_t)(((int64_t)i * CB * Mp + (int64_t)l * CB) * 8); };
  auto offB = [&](int i, int c) { return (uint32_t)((Mp * Mp + (int64_t)i * CB * Mp + (int64_t)c * CB) * 8); };
  auto offD = [&](int j) { return (uint32_t)((2 * Mp * Mp + (int64_t)j * CB * CB) * 8); };
  float* LinvT = a.LinvT + (int64_t)b * a.strideL;
  float* lt_max = a.lt_absmax[0];
#pragma unroll
  for (int q = 1; q < kMaxBatch; ++q)
    if (b == q) lt_max = a.lt_absmax[q];
  auto store_linvT = [&](int c, int j, const double* sx) {  // X_jc -> LinvT block (c, j)
    const int64_t gr = (int64_t)c * CB, gc = (int64_t)j * CB;
    const float m = tile_store_f32_v4(LinvT + gr * a.ldl + gc, a.ldl, sx, true, (int)min<int64_t>(CB, a.M - gr),
                                      (int)min<int64_t>(CB, a.M - gc));
    if (lt_max) wave_absmax_atomic(m, lt_max);
  };
  auto store_L = [&](int i, int j, const double* s) {     // L block (i, j), float32
    if (!a.L) return;
    const int64_t gr = (int64_t)i * CB, gc = (int64_t)j * CB;
    tile_store_f32_v4(a.L + (int64_t)b * a.strideL + gr * a.ldl + gc, a.ldl, s, false,
                      (int)min<int64_t>(CB, a.M - gr), (int)min<int64_t>(CB, a.M - gc));
  };
  auto give_up = [&]() {
    if (threadIdx.x == 0) atomicCAS(a.info + b, 0, -1);
  };

  if (blockIdx.x == 0) {
    // ---------------------------------------------------------------- chain
    double *sD = bufA, *s1 = bufB, *s2 = bufC;
    {
      TileRegs rD;
      tile_fetch_c(rD, R, offD(0), CB);
      tile_put(sD, rD);
      __syncthreads();
      store_linvT(0, 0, sD);                             // X_00 = D_0
    }
    for (int j = 0; j + 1 < nb; ++j) {
      PSTAMP(b, j, 0);
      const int* p[4] = {Wver + (j + 1) * nb + j, Wver + (j + 1) * nb + j + 1, Wver, Wver};
      const int v[4] = {j, j, 0, 0};
      if (!wait_all(p, v, 2, err, &s_flag)) { give_up(); return; }
      PSTAMP(b, j, 1);
      TileRegs r1, r2;
      tile_fetch_c(r1, R, offW(j + 1, j), Mp);
      tile_fetch_c(r2, R, offW(j + 1, j + 1), Mp);
      tile_put(s1, r1);
      tile_put(s2, r2);
      __syncthreads();
      PSTAMP(b, j, 2);
      Blk4 pi = blk4_zero();
      row_mma<true, 1>(pi, s1, sD, 1.0);                 // L_{j+1,j} = W_{j+1,j} D_j^T
      row_to_global_c(R, offW(j + 1, j), Mp, pi);        // handed to the U tasks of column j + 1
      __syncthreads();
      blk4_to_lds<true>(s1, pi);
      __syncthreads();
      // column block 0 of W_{j+1,j+1} -= P P^T (one 16x16 block per wave); the rest
      // beside the first panel sweep (factor_diag_tile's pending update).  The
      // L_{j+1,j} stores drain meanwhile.
      sub_outer_blk<4>(s2, 16 * (threadIdx.x >> 6), 0, s1, s1);
      publish(Wver + (j + 1) * nb + j, j + 1);
      __syncthreads();
      PSTAMP(b, j, 3);
      store_L(j + 1, j, s1);
      factor_diag_tile(s2, s1, col, a.info + b, (int64_t)(j + 1) * CB, s1);
      __syncthreads();
      PSTAMP(b, j, 4);
      tile_store_c(R, offD(j + 1), CB, s1);              // D_{j+1}, handed to the workers
      publish(Dready + j + 1, 1);
      PSTAMP(b, j, 5);
      store_L(j + 1, j + 1, s2);
      store_linvT(j + 1, j + 1, s1);                     // X_{j+1,j+1} = D_{j+1}
      __syncthreads();
      PSTAMP(b, j, 6);
      double* t = sD; sD = s1; s1 = t;                   // D_{j+1} stays in LDS
    }
    return;
  }

  // ------------------------------------------------------------------ workers
  // Software-pipelined: the next task is dequeued while the current one's tiles load,
  // and its tiles are loaded (when its inputs are already published) while the
  // current one computes.  A task's operands: tile 1 -> s1, tile 2 -> s2 (optional),
  // the read-modify-write tile in registers (optional), D_j -> sD (cached per step).
  double *s1 = bufA, *s2 = bufB, *sD = bufC;
  int dcur = -1;                                         // the step whose D is in sD
  struct Plan { int kind, j, i, l; uint32_t o1, o2, ou; bool t2, u, d; };
  auto decode = [&](int t, Plan& P) {
    const int code = a.tasks[t];
    P.kind = code >> 24; P.j = (code >> 16) & 255; P.i = (code >> 8) & 255; P.l = code & 255;
    const int j = P.j, i = P.i, l = P.l;
    P.t2 = P.u = P.d = false;
    P.o2 = P.ou = 0;
    if (P.kind == kTaskPan) { P.o1 = offW(i, j); P.d = true; }
    else if (P.kind == kTaskU) {
      P.o1 = offW(i, j); P.t2 = true;
      if (l != i) { P.o2 = offW(l, j); P.u = true; P.ou = offW(i, l); }
      else P.o2 = offW(i, i);
    } else if (P.kind == kTaskXR) { P.o1 = offB(j, l); P.d = true; }
    else {
      P.o1 = offW(i, j);
      if (l < j) { P.t2 = true; P.o2 = offB(j, l); P.u = true; P.ou = offB(i, l); }
      else P.d = true;
    }
  };
  auto deps = [&](const Plan& P, const int* (&p)[4], int (&v)[4]) {
    const int j = P.j, i = P.i, l = P.l;
    for (int k = 0; k < 4; ++k) { p[k] = Wver; v[k] = 0; }
    if (P.kind == kTaskPan) {
      p[0] = Dready + j; v[0] = 1; p[1] = Wver + i * nb + j; v[1] = j;
      return 2;
    }
    if (P.kind == kTaskU) {
      p[0] = Wver + i * nb + j; v[0] = j + 1; p[1] = Wver + i * nb + l; v[1] = j;
      p[2] = Wver + l * nb + j; v[2] = j + 1;
      return (l != i) ? 3 : 2;
    }
    if (P.kind == kTaskXR) {
      p[0] = Dready + j; v[0] = 1; p[1] = Bver + j * nb + l; v[1] = j - l;
      return 2;
    }
    p[0] = Wver + i * nb + j; v[0] = j + 1;
    if (l < j) {
      p[1] = Bver + j * nb + l; v[1] = j - l + 1; p[2] = Bver + i * nb + l; v[2] = j - l;
      return 3;
    }
    p[1] = Dready + j; v[1] = 1;
    return 2;
  };
  struct Regs { TileRegs r1, r2; Blk4 u; };
  auto issue = [&](const Plan& P, Regs& G) {
    tile_fetch_c(G.r1, R, P.o1, Mp);
    if (P.t2) tile_fetch_c(G.r2, R, P.o2, Mp);
    if (P.u) row_from_global_c(G.u, R, P.ou, Mp);
  };
  auto dequeue = [&]() {
    if (threadIdx.x == 0) s_task = atomicAdd(head, 1);
    __syncthreads();
    const int t = s_task;
    __syncthreads();
    return t;
  };

  int tc = dequeue();
  if (tc >= a.ntask) return;
  Plan P;
  decode(tc, P);
  Regs G;
  {
    const int* p[4];
    int v[4];
    const int n = deps(P, p, v);
    if (!wait_all(p, v, n, err, &s_flag)) { give_up(); return; }
    issue(P, G);
  }
  const int wid = blockIdx.x;
  for (;;) {
    unsigned long long c0 = PNOW();
    const int tn = dequeue();                            // overlaps the loads in flight
    unsigned long long c1 = PNOW();
    PWACC(b, wid, 0, c1 - c0);
    if (P.d && dcur != P.j) {
      TileRegs rD;
      tile_fetch_c(rD, R, offD(P.j), CB);
      tile_put(sD, rD);
      dcur = P.j;
      PWACC(b, wid, 7, 1);
    }
    tile_put(s1, G.r1);
    if (P.t2) tile_put(s2, G.r2);
    Blk4 u = P.u ? G.u : blk4_zero();
    __syncthreads();
    unsigned long long c2 = PNOW();
    PWACC(b, wid, 2, c2 - c1);
    // the next task's operands, in flight during this task's MFMAs (when published)
    Plan Q;
    bool have = tn < a.ntask, issued = false;
    const int* pq[4];
    int vq[4], nq = 0;
    if (have) {
      decode(tn, Q);
      nq = deps(Q, pq, vq);
      if (poll_all(pq, vq, nq, &s_flag)) { issue(Q, G); issued = true; }
    }
    unsigned long long c3 = PNOW();
    PWACC(b, wid, 3, c3 - c2);
    PWACC(b, wid, 6, issued ? 1 : 0);
    PWACC(b, wid, 5, 1);
    const int j = P.j, i = P.i, l = P.l;
    if (P.kind == kTaskPan) {                            // L_ij = W_ij D_j^T in place
      Blk4 pi = blk4_zero();
      row_mma<true, 1>(pi, s1, sD, 1.0);
      row_to_global_c(R, offW(i, j), Mp, pi);
      __syncthreads();
      blk4_to_lds<true>(s1, pi);
      publish(Wver + i * nb + j, j + 1);
      __syncthreads();
      store_L(i, j, s1);
    } else if (P.kind == kTaskU && l != i) {             // W_il -= L_ij L_lj^T
      row_mma<true, 0>(u, s1, s2, -1.0);
      row_to_global_c(R, offW(i, l), Mp, u);
      publish(Wver + i * nb + l, j + 1);
    } else if (P.kind == kTaskU) {                       // lower blocks of W_ii -= L_ij L_ij^T
      diag_lower_update(s2, s1);
      __syncthreads();
      tile_store_c(R, offW(i, i), Mp, s2);
      publish(Wver + i * nb + i, j + 1);
    } else if (P.kind == kTaskXR) {                      // X_jc = D_j B_jc in place, LinvT block (c, j)
      Blk4 x = blk4_zero();
      col_mma_lower(x, sD, s1);
      __syncthreads();
      blk4_to_lds<false>(s1, x);
      __syncthreads();
      tile_store_c(R, offB(j, l), Mp, s1);
      publish(Bver + j * nb + l, j - l + 1);
      store_linvT(l, j, s1);
    } else {                                             // FU: B_ic -= L_ij X_jc (X_jj = D_j)
      if (l < j) row_mma<false, 0>(u, s1, s2, -1.0);
      else row_mma<false, 2>(u, s1, sD, -1.0);
      row_to_global_c(R, offB(i, l), Mp, u);
      publish(Bver + i * nb + l, j - l + 1);
    }
    __syncthreads();
    unsigned long long c4 = PNOW();
    PWACC(b, wid, 4, c4 - c3);
    if (!have) break;
    if (!issued) {
      if (!wait_all(pq, vq, nq, err, &s_flag)) { give_up(); return; }
      issue(Q, G);
    }
    PWACC(b, wid, 1, PNOW() - c4);
    P = Q;
  }
}

// ------------------------------------------------------------------ Cholesky backward
// Reverse mode of Lm = chol(Kuu) (GPflow base_conditional's cholesky,
// models.py:141), as in PyTorch / Murray (2016):
//   P = Phi(Lm^T gL)  (lower triangle, diagonal halved),  S = Lm^-T P Lm^-1,
//   gKuu = (S + S^T) / 2,
// all in float64 (M^3 work; Kuu is badly conditioned).  dgemm: C = op(A) op(B)
// on v_mfma_f64_16x16x4_f64: 64 x 64 tile per workgroup (4 waves x 32 x 32 =
// 2 x 2 MFMA blocks each), 16-deep LDS chunks.  tri (the triangular operands of
// the three products; every term outside the range is an exact zero):
//   kTriNone: k over [0, M);
//   kTriUpperK: k over [max(i0, j0), M)  (op(A) upper, op(B) lower: L^T gL, Linv^T G);
//   kTriBand: k over [j0, i0 + 64)       (A lower, B lower: P Linv);
//   | kTriLowerOut: tiles wholly above the diagonal are not computed (their
//     consumer reads only the lower triangle / never reaches them).
constexpr int kTriNone = 0, kTriUpperK = 1, kTriBand = 2, kTriLowerOut = 4;
template <bool TA, bool TB, int BN = 64, int KC = 16>
__global__ __launch_bounds__(256) void dgemm_kernel(const double* __restrict__ A, int64_t lda,
                                                    const double* __restrict__ B, int64_t ldb,
                                                    double* __restrict__ C, int64_t ldc, int64_t M, int tri) {
  // 64 x BN tile; wave w: rows wi .. wi + 31, columns wj .. wj + BN / 2 - 1 (NB 16-wide blocks);
  // KC-deep chunks (KC / 4 MFMA k-steps per barrier pair)
  constexpr int NB = BN / 32, LA = 64 * KC / 256, LB = KC * BN / 256;  // loads per thread
  __shared__ double sa[64][KC + 1], sb[KC][BN + 1];  // sa[i][k] = op(A), sb[k][j] = op(B)
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wi = (w >> 1) * 32, wj = (w & 1) * (BN / 2);
  const int64_t i0 = (int64_t)blockIdx.y * 64, j0 = (int64_t)blockIdx.x * BN;
  if ((tri & kTriLowerOut) && j0 > i0 + 63) return;
  const int64_t klo = (tri & kTriUpperK) ? (i0 > j0 ? i0 : j0) : (tri & kTriBand) ? j0 : 0;
  const int64_t khi = (tri & kTriBand) ? (i0 + 64 < M ? i0 + 64 : M) : M;
  doublex4 acc[2][NB];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < NB; ++b) acc[a][b] = doublex4{0.0, 0.0, 0.0, 0.0};
  // chunk k0 .. k0 + KC - 1: thread loads LA elements of op(A) and LB of op(B)
  // (coalesced along the contiguous index), one chunk ahead in registers
  double ra[LA], rb[LB];
  auto load = [&](int64_t k0) {
#pragma unroll
    for (int q = 0; q < LA; ++q) {
      const int idx = tid + 256 * q;
      const int r_a = TA ? idx % 64 : idx / KC, k_a = TA ? idx / 64 : idx % KC;
      const int64_t ia = i0 + r_a, kA = k0 + k_a;
      ra[q] = (ia < M && kA < M) ? (TA ? A[kA * lda + ia] : A[ia * lda + kA]) : 0.0;
    }
#pragma unroll
    for (int q = 0; q < LB; ++q) {
      const int idx = tid + 256 * q;
      const int c_b = TB ? idx / KC : idx % BN, k_b = TB ? idx % KC : idx / BN;
      const int64_t jb = j0 + c_b, kB = k0 + k_b;
      rb[q] = (jb < M && kB < M) ? (TB ? B[jb * ldb + kB] : B[kB * ldb + jb]) : 0.0;
    }
  };
  auto store = [&]() {
#pragma unroll
    for (int q = 0; q < LA; ++q) {
      const int idx = tid + 256 * q;
      sa[TA ? idx % 64 : idx / KC][TA ? idx / 64 : idx % KC] = ra[q];
    }
#pragma unroll
    for (int q = 0; q < LB; ++q) {
      const int idx = tid + 256 * q;
      sb[TB ? idx % KC : idx / BN][TB ? idx / KC : idx % BN] = rb[q];
    }
  };
  if (klo < khi) load(klo);
  for (int64_t k0 = klo; k0 < khi; k0 += KC) {
    store();
    __syncthreads();
    if (k0 + KC < khi) load(k0 + KC);
#pragma unroll
    for (int ks = 0; ks < KC / 4; ++ks) {
      double av[2], bv[NB];
#pragma unroll
      for (int t = 0; t < 2; ++t) av[t] = sa[wi + 16 * t + (lane & 15)][4 * ks + (lane >> 4)];
#pragma unroll
      for (int t = 0; t < NB; ++t) bv[t] = sb[4 * ks + (lane >> 4)][wj + 16 * t + (lane & 15)];
#pragma unroll
      for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < NB; ++b) acc[a][b] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[a], bv[b], acc[a][b], 0, 0, 0);
    }
    __syncthreads();
  }
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < NB; ++b)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int64_t i = i0 + wi + 16 * a + (lane >> 4) + 4 * r, j = j0 + wj + 16 * b + (lane & 15);
        if (i < M && j < M) C[i * ldc + j] = acc[a][b][r];
      }
}

// mode 0: dst = f64(src) (src f32);  1: dst = f64(src^T);  2: Phi (tril, diag / 2) in place on f64;
// 3: out32 = (S + S^T) / 2 -> f32 and out64 (optional)
__global__ __launch_bounds__(256) void chol_bwd_elem_kernel(int mode, const float* __restrict__ src32,
                                                            int64_t lds, double* __restrict__ d, int64_t M,
                                                            float* __restrict__ out32, int64_t ldo) {
  const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (idx >= M * M) return;
  const int64_t i = idx / M, j = idx % M;
  if (mode == 0) d[idx] = (double)src32[i * lds + j];
  else if (mode == 1) d[idx] = (double)src32[j * lds + i];
  else if (mode == 2) d[idx] = (j < i) ? d[idx] : (j == i ? 0.5 * d[idx] : 0.0);
  else out32[i * ldo + j] = (float)(0.5 * (d[i * M + j] + d[j * M + i]));
}

}  // namespace mgp

using namespace mgp;

static int64_t chol_mp(int64_t M) { return (M + CB - 1) / CB * CB; }
static int64_t chol_ws_doubles_per_batch(int64_t M) {
  const int64_t Mp = chol_mp(M);
  return 2 * Mp * Mp + (Mp / CB) * CB * CB;
}

#ifdef MGP_DBG_STAMPS
extern "C" int mgp_dbg_chol_stamps(unsigned long long* host) {
  return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(g_stamps), sizeof(g_stamps));
}
extern "C" int mgp_dbg_persist_stamps(unsigned long long* chain, unsigned long long* work, int reset) {
  if (reset) {
    static unsigned long long zeros[2 * 128 * 8] = {};
    hipMemcpyToSymbol(HIP_SYMBOL(g_pchain), zeros, sizeof(zeros));
    return (int)hipMemcpyToSymbol(HIP_SYMBOL(g_pwork), zeros, sizeof(zeros));
  }
  hipMemcpyFromSymbol(chain, HIP_SYMBOL(g_pchain), sizeof(g_pchain));
  return (int)hipMemcpyFromSymbol(work, HIP_SYMBOL(g_pwork), sizeof(g_pwork));
}
#endif

static int64_t chol_task_ints(int nb) { return ((int64_t)task_count(nb) + 63) / 64 * 64; }

// doubles of every batch entry, then the persistent path's sync words (per batch)
// and its task table (shared)
extern "C" size_t mgp_chol_workspace_bytes(int64_t M, int32_t batch) {
  if (M <= 0 || batch <= 0) return 0;
  const int nb = (int)(chol_mp(M) / CB);
  return (size_t)chol_ws_doubles_per_batch(M) * (size_t)batch * sizeof(double) +
         (size_t)(chol_sync_words(nb) * batch + chol_task_ints(nb)) * sizeof(int);
}

// Persistent launch (chol_persist) with MGP_CHOL_PERSIST=1 (measured at c3: 0.27-0.28 ms
// standalone at 48-64 workers per layer against 0.28 ms for the per-step launches, 445 vs
// 434 us in the ELBO step -- the chain -> worker -> chain hand-offs of every step cost what
// the launch boundaries did); sizes it supports: task codes hold 8-bit tile
// indices, the per-batch buffer resource 31-bit offsets.
static bool chol_persist_ok(int nb, int64_t strideWS) {
  const char* e = getenv("MGP_CHOL_PERSIST");   // read per call (tuning runs switch it in-process)
  const int env = e ? atoi(e) : 0;
  return env != 0 && nb >= 3 && nb <= 128 && strideWS * 8 < ((int64_t)1 << 31);
}
// Worker workgroups per batch entry (MGP_CHOL_WORKERS overrides)
static int chol_persist_workers(int nb) {
  const char* e = getenv("MGP_CHOL_WORKERS");
  const int env = e ? atoi(e) : 0;
  if (env > 0) return env;
  return std::min(48, std::max(2, 2 * nb));
}

// Per-step launches on tile pairs (chol_step_pair, default) or one tile per workgroup
// (chol_step, MGP_CHOL_PAIR=0; read per call).
static bool chol_pair_enabled() {
  const char* e = getenv("MGP_CHOL_PAIR");
  return e ? atoi(e) != 0 : true;
}

static int chol_run(CholArgs& a, int batch, void* workspace, size_t workspace_bytes, hipStream_t s,
                    hipEvent_t prep_done = nullptr) {
  if (!workspace || workspace_bytes < mgp_chol_workspace_bytes(a.M, batch)) return MGP_ERR_WORKSPACE;
  if (!aligned16(workspace)) return MGP_ERR_ALIGN;
  // the diagonal tiles of L and L^-T are written with 16-byte stores
  const bool lay4 = a.ldl % 4 == 0 && (batch <= 1 || a.strideL % 4 == 0);
  if ((a.L && !aligned16(a.L)) || (a.LinvT && !aligned16(a.LinvT)) || !lay4) return MGP_ERR_ALIGN;
  a.Mp = chol_mp(a.M);
  a.nb = (int)(a.Mp / CB);
  a.strideWS = chol_ws_doubles_per_batch(a.M);
  a.ws = (double*)workspace;
  const bool persist = chol_persist_ok(a.nb, a.strideWS);
  if (persist) {
    a.strideSync = chol_sync_words(a.nb);
    a.sync = (int*)((char*)workspace + (size_t)a.strideWS * batch * sizeof(double));
    a.tasks = a.sync + a.strideSync * batch;
    a.ntask = task_count(a.nb);
  }
  const dim3 block(kCholThreads);
  hipLaunchKernelGGL(chol_prep, dim3(a.nb * a.nb + 1, batch), block, 0, s, a);
  int st = launch_status();
  if (st) return st;
  if (prep_done) {
    st = hip_status(hipEventRecord(prep_done, s));
    if (st) return st;
  }
  if (persist) {
    hipLaunchKernelGGL(chol_persist, dim3(1 + chol_persist_workers(a.nb), batch), block, 0, s, a);
    return launch_status();
  }
  const bool pair = chol_pair_enabled();
  for (int j = 0; j < a.nb; ++j) {
    const int T = a.nb - j - 1;
    if (pair && T > 0) {
      hipLaunchKernelGGL(chol_step_pair, dim3(1 + step_pair_count(a.nb, j), batch), dim3(kPairThreads), 0, s, a, j);
      st = launch_status();
      if (st) return st;
      continue;
    }
    const int n = (T == 0) ? a.nb : T * (T + 1) / 2 + T * (j + 1);
    hipLaunchKernelGGL(chol_step, dim3(n, batch), block, 0, s, a, j);
    st = launch_status();
    if (st) return st;
  }
  return MGP_OK;
}

extern "C" int mgp_potrf_trtri(const float* A, int64_t lda, int64_t strideA, int64_t M, int32_t batch,
                               float* L, float* LinvT, int64_t ldl, int64_t strideL, int32_t* info,
                               void* workspace, size_t workspace_bytes, mgp_stream_t stream) {
  if (!A) return -1;
  if (lda < M) return -2;
  if (batch > 1 && strideA < lda * M) return -3;
  if (M < 0) return -4;
  if (batch < 0) return -5;
  if (!LinvT) return -7;
  if (ldl < M) return -8;
  if (batch > 1 && strideL < ldl * M) return -9;
  if (!info) return -10;
  if (M == 0 || batch == 0) return MGP_OK;
  CholArgs a = {};
  a.A = A; a.lda = lda; a.strideA = strideA;
  a.L = L; a.LinvT = LinvT; a.ldl = ldl; a.strideL = strideL;
  a.info = info; a.M = M;
  return chol_run(a, batch, workspace, workspace_bytes, (hipStream_t)stream);
}

static int kuu_potrf_trtri_impl(const float* const* Z, int64_t ldz, int64_t M, int32_t D,
                                   const float* const* variance, const float* const* lengthscales,
                                   const int32_t* n_ls, float jitter, int32_t batch, float* L,
                                   float* LinvT, int64_t ldl, int64_t strideL, int32_t* info,
                                   void* workspace, size_t workspace_bytes, hipEvent_t prep_done,
                                   float* const* lt_absmax, mgp_stream_t stream) {
  if (!Z) return -1;
  if (ldz < D) return -2;
  if (M < 0) return -3;
  if (D < 1) return -4;
  if (!variance) return -5;
  if (!lengthscales) return -6;
  if (!n_ls) return -7;
  if (!(jitter >= 0.f)) return -8;
  if (batch < 0 || batch > kMaxBatch) return -9;
  if (!LinvT) return -11;
  if (ldl < M) return -12;
  if (batch > 1 && strideL < ldl * M) return -13;
  if (!info) return -14;
  if (M == 0 || batch == 0) return MGP_OK;
  CholArgs a = {};
  for (int b = 0; b < batch; ++b) {
    if (!Z[b] || !variance[b] || !lengthscales[b]) return -1;
    if (n_ls[b] != 1 && n_ls[b] != D) return -7;
    a.Z[b] = Z[b]; a.var[b] = variance[b]; a.ls[b] = lengthscales[b]; a.n_ls[b] = n_ls[b];
    a.lt_absmax[b] = lt_absmax ? lt_absmax[b] : nullptr;
  }
  a.ldz = ldz; a.D = D; a.jitter = (double)jitter;
  a.L = L; a.LinvT = LinvT; a.ldl = ldl; a.strideL = strideL;
  a.info = info; a.M = M;
  return chol_run(a, batch, workspace, workspace_bytes, (hipStream_t)stream, prep_done);
}

extern "C" int mgp_kuu_potrf_trtri(const float* const* Z, int64_t ldz, int64_t M, int32_t D,
                                   const float* const* variance, const float* const* lengthscales,
                                   const int32_t* n_ls, float jitter, int32_t batch, float* L,
                                   float* LinvT, int64_t ldl, int64_t strideL, int32_t* info,
                                   void* workspace, size_t workspace_bytes, mgp_stream_t stream) {
  return kuu_potrf_trtri_impl(Z, ldz, M, D, variance, lengthscales, n_ls, jitter, batch, L, LinvT, ldl, strideL,
                              info, workspace, workspace_bytes, nullptr, nullptr, stream);
}

extern "C" int mgp_kuu_potrf_trtri_ev(const float* const* Z, int64_t ldz, int64_t M, int32_t D,
                                      const float* const* variance, const float* const* lengthscales,
                                      const int32_t* n_ls, float jitter, int32_t batch, float* L,
                                      float* LinvT, int64_t ldl, int64_t strideL, int32_t* info,
                                      void* workspace, size_t workspace_bytes, void* prep_done,
                                      mgp_stream_t stream) {
  return kuu_potrf_trtri_impl(Z, ldz, M, D, variance, lengthscales, n_ls, jitter, batch, L, LinvT, ldl, strideL,
                              info, workspace, workspace_bytes, (hipEvent_t)prep_done, nullptr, stream);
}

extern "C" int mgp_kuu_potrf_trtri_ex(const float* const* Z, int64_t ldz, int64_t M, int32_t D,
                                      const float* const* variance, const float* const* lengthscales,
                                      const int32_t* n_ls, float jitter, int32_t batch, float* L,
                                      float* LinvT, int64_t ldl, int64_t strideL, int32_t* info,
                                      void* workspace, size_t workspace_bytes, void* prep_done,
                                      float* const* linvt_absmax, mgp_stream_t stream) {
  return kuu_potrf_trtri_impl(Z, ldz, M, D, variance, lengthscales, n_ls, jitter, batch, L, LinvT, ldl, strideL,
                              info, workspace, workspace_bytes, (hipEvent_t)prep_done, linvt_absmax, stream);
}

extern "C" size_t mgp_chol_backward_workspace_bytes(int64_t M) {
  return (size_t)(M > 0 ? M : 1) * (size_t)(M > 0 ? M : 1) * 4 * sizeof(double);
}

extern "C" int mgp_chol_backward(const float* L, int64_t ldl, const float* LinvT, int64_t ldli, const float* gL,
                                 int64_t ldg, int64_t M, float* gKuu, int64_t ldo, void* workspace,
                                 size_t workspace_bytes, mgp_stream_t stream) {
  if (!L) return -1;
  if (ldl < M) return -2;
  if (!LinvT) return -3;
  if (ldli < M) return -4;
  if (!gL) return -5;
  if (ldg < M) return -6;
  if (M < 0) return -7;
  if (!gKuu) return -8;
  if (ldo < M) return -9;
  if (M == 0) return MGP_OK;
  if (!workspace || workspace_bytes < mgp_chol_backward_workspace_bytes(M)) return MGP_ERR_WORKSPACE;
  hipStream_t s = (hipStream_t)stream;
  constexpr int KCB = 32;  // chunk depth of the products (32: half the barriers of 16)
  double* Ld = (double*)workspace;
  double* Li = Ld + M * M;   // Linv = LinvT^T
  double* G = Li + M * M;
  double* T = G + M * M;
  const dim3 eg((unsigned)((M * M + 255) / 256)), gg((unsigned)((M + 31) / 32), (unsigned)((M + 63) / 64));  // 64 x 32 tiles: 2 x the workgroups of 64 x 64 (measured faster at M = 1024)
  hipLaunchKernelGGL(chol_bwd_elem_kernel, eg, dim3(256), 0, s, 0, L, ldl, Ld, M, nullptr, (int64_t)0);
  hipLaunchKernelGGL(chol_bwd_elem_kernel, eg, dim3(256), 0, s, 1, LinvT, ldli, Li, M, nullptr, (int64_t)0);
  hipLaunchKernelGGL(chol_bwd_elem_kernel, eg, dim3(256), 0, s, 0, gL, ldg, G, M, nullptr, (int64_t)0);
  // L, gL, Linv are lower triangular (exact zeros above), so are P and P Linv: the
  // products skip the zero terms and the tiles Phi / the next product never read
  hipLaunchKernelGGL((dgemm_kernel<true, false, 32, KCB>), gg, dim3(256), 0, s, Ld, M, G, M, T, M, M,
                     kTriUpperK | kTriLowerOut);                                                      // L^T gL
  hipLaunchKernelGGL(chol_bwd_elem_kernel, eg, dim3(256), 0, s, 2, nullptr, (int64_t)0, T, M, nullptr, (int64_t)0);
  hipLaunchKernelGGL((dgemm_kernel<false, false, 32, KCB>), gg, dim3(256), 0, s, T, M, Li, M, G, M, M,
                     kTriBand | kTriLowerOut);                                                        // P Linv
  hipLaunchKernelGGL((dgemm_kernel<true, false, 32, KCB>), gg, dim3(256), 0, s, Li, M, G, M, T, M, M,
                     kTriUpperK);                                                                     // Linv^T (.)
  hipLaunchKernelGGL(chol_bwd_elem_kernel, eg, dim3(256), 0, s, 3, nullptr, (int64_t)0, T, M, gKuu, ldo);
  return launch_status();
}
