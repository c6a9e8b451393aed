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
// matrices (chol_prep: blockIdx.y; the step launches: step_pair_count).  nb + 1
// launches per factorisation.
#include <math.h>
#include <stdlib.h>

#include <algorithm>
#include <atomic>
#include <cstddef>
#include <vector>

#include "kuf_image.hpp"
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
#define STAMP(j, k) do { if (threadIdx.x == 0 && blockIdx.x == 0 && blockIdx.y == 0) g_stamps[(j) * 16 + (k)] = __builtin_amdgcn_s_memtime(); } while (0)
// 100 MHz reference clock (one time base for every CU): slots 14 / 15
#define RSTAMP(j, k) do { if (threadIdx.x == 0 && blockIdx.x == 0 && blockIdx.y == 0) g_stamps[(j) * 16 + (k)] = __builtin_amdgcn_s_memrealtime(); } while (0)
// one pair workgroup per step (the first pair of the last tile row, batch 0): phase stamps
__device__ unsigned long long g_pair_stamps[64 * 8];
#define PAIRSTAMP(on, j, k) do { if ((on) && threadIdx.x == 0) g_pair_stamps[(j) * 8 + (k)] = __builtin_amdgcn_s_memtime(); } while (0)
// the time at kernel entry (held in a register until the workgroup knows whether it stamps)
#define ENTRYTIME(t) const unsigned long long t = __builtin_amdgcn_s_memtime()
#define PAIRSTAMP_AT(on, j, k, t) do { if ((on) && threadIdx.x == 0) g_pair_stamps[(j) * 8 + (k)] = (t); } while (0)
#else
#define ENTRYTIME(t) do {} while (0)
#define PAIRSTAMP_AT(on, j, k, t) do {} while (0)
#define STAMP(j, k) do {} while (0)
#define RSTAMP(j, k) do {} while (0)
#define PAIRSTAMP(on, j, k) do {} while (0)
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
  double* ws; int64_t strideWS;                   // per batch: W, B tile-major [nb][nb][64][64], D [nb][64][64]
  int64_t M, Mp; int nb;
  // optional Kuf side job (mgp_kuu_potrf_trtri_kuf): the Kuf image of every batch entry,
  // K(Z_b, X) (kuf_image.hpp blocks), written by extra workgroups of the step launches
  const float* kx; int64_t kldx, kN;
  bf16x8* kfr[kMaxBatch]; float* kbound[kMaxBatch];
  int kf16, knmk, krow_blocks; int64_t kblocks;   // blocks per batch entry
};

__device__ __forceinline__ double* ws_W(const CholArgs& a, int b) { return a.ws + (int64_t)b * a.strideWS; }
__device__ __forceinline__ double* ws_B(const CholArgs& a, int b) { return ws_W(a, b) + a.Mp * a.Mp; }
// W and B are tile-major: tile (bi, bl) is 64 x 64 contiguous doubles (leading dimension
// CB) at ((bi nb + bl) 64 64).  A row-major tile's 64 rows sit Mp doubles apart (8 KiB at
// M = 1024), so every step launch's concurrent tile loads hit the same few HBM channels.
__device__ __forceinline__ double* ws_tile(const CholArgs& a, double* base, int bi, int bl) {
  return base + ((int64_t)bi * a.nb + bl) * (CB * CB);
}
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
// tile_fetch of a block-lower-triangular tile (D_j = L_jj^-1): the 16 x 16 blocks above the
// block diagonal are not loaded (their lanes are masked off) and come back as zeros
__device__ __forceinline__ void tile_fetch_lower(TileRegs& t, const double* __restrict__ g, int64_t ld) {
#pragma unroll
  for (int it = 0; it < 8; ++it) {
    const int idx = ctid() + kCholThreads * it, r = idx >> 5, c = (idx & 31) * 2;
    t.v[it] = (c >> 4) <= (r >> 4) ? *reinterpret_cast<const double2*>(g + (int64_t)r * ld + c) : double2{0.0, 0.0};
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
// The LDS operands of k-step s + 1 are read before the MFMAs of k-step s (two register
// sets; round 4): the compiler had issued each k-step's reads right in front of its own
// MFMAs and waited for them (lgkmcnt(0) after one MFMA of cover).  The sign is applied
// at the MFMA, so the reads need no VALU op behind them; per accumulator the MFMAs run
// in the same k order (same bits).
template <bool TB, int TRI, int BLK = 0xF>
__device__ __forceinline__ void row_mma(Blk4& r, const double* __restrict__ sa, const double* __restrict__ sb,
                                        double sign) {
  const int lane = ctid() & 63, w = ctid() >> 6, l16 = lane & 15, kq = lane >> 4;
  auto on = [](int tj, int k0) {
    return ((BLK >> tj) & 1) && !(TRI == 1 && k0 >= 16 * (tj + 1)) && !(TRI == 2 && k0 < 16 * tj);
  };
  double av[2], bv[2][4];
  auto load = [&](int buf, int k0) {
    const int k = k0 + kq;
    av[buf] = sa[(16 * w + l16) * LDT + k];
#pragma unroll
    for (int tj = 0; tj < 4; ++tj)
      if (on(tj, k0)) bv[buf][tj] = TB ? sb[(16 * tj + l16) * LDT + k] : sb[k * LDT + 16 * tj + l16];
  };
  load(0, 0);
#pragma unroll
  for (int st = 0; st < CB / 4; ++st) {
    const int k0 = 4 * st, cur = st & 1;
    if (st + 1 < CB / 4) load(cur ^ 1, k0 + 4);
    __builtin_amdgcn_sched_barrier(0);
    const double a = sign * av[cur];
#pragma unroll
    for (int tj = 0; tj < 4; ++tj)
      if (on(tj, k0)) r.c[tj] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, bv[cur][tj], r.c[tj], 0, 0, 0);
    __builtin_amdgcn_sched_barrier(0);
  }
}

// Column stripe: C[16ti + i][16w + j] += sum_k D[16ti + i][k] sb[k][16w + j] with
// D lower triangular (k < 16 (ti + 1)): X_jc = D_j B_jc.  Operands one k-step ahead
// as row_mma.
__device__ __forceinline__ void col_mma_lower(Blk4& r, const double* __restrict__ sD, const double* __restrict__ sb) {
  const int lane = ctid() & 63, w = ctid() >> 6, l16 = lane & 15, kq = lane >> 4;
  double bv[2], av[2][4];
  auto load = [&](int buf, int k0) {
    const int k = k0 + kq;
    bv[buf] = sb[k * LDT + 16 * w + l16];
#pragma unroll
    for (int ti = 0; ti < 4; ++ti)
      if (k0 < 16 * (ti + 1)) av[buf][ti] = sD[(16 * ti + l16) * LDT + k];
  };
  load(0, 0);
#pragma unroll
  for (int st = 0; st < CB / 4; ++st) {
    const int k0 = 4 * st, cur = st & 1;
    if (st + 1 < CB / 4) load(cur ^ 1, k0 + 4);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int ti = 0; ti < 4; ++ti)
      if (k0 < 16 * (ti + 1)) r.c[ti] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[cur][ti], bv[cur], r.c[ti], 0, 0, 0);
    __builtin_amdgcn_sched_barrier(0);
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
  double av[4], bv[4];   // all operands read before the first MFMA (one LDS wait, not four)
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    av[q] = sa[i * LDT + 4 * q + kq];
    bv[q] = TB ? sb[i * LDT + 4 * q + kq] : sb[(4 * q + kq) * LDT + i];
  }
#pragma unroll
  for (int q = 0; q < 4; ++q) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(sign * av[q], bv[q], acc, 0, 0, 0);
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
    // operands of the next four k-steps read before the current four MFMAs
    double av[2][4], bv[2][4];
    auto load = [&](int buf, int c) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        av[buf][q] = sP[(16 * bi + l16) * LDT + 16 * c + 4 * q + kq];
        bv[buf][q] = sP[(16 * bj + l16) * LDT + 16 * c + 4 * q + kq];
      }
    };
    load(0, 0);
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      if (c + 1 < 4) load((c + 1) & 1, c + 1);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int q = 0; q < 4; ++q) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(-av[c & 1][q], bv[c & 1][q], acc, 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
    }
    blk_store(s + 16 * bi * LDT + 16 * bj, acc);
  }
}

// s[R0 .. R0+15][C1 .. C1+15] -= sum over 16 NK columns k of sa[R0 + i][k] sb[C1 + j][k]
// (one wave, f64 MFMA; rows of sa / sb at leading dimension LDT).
template <int NK>
__device__ __forceinline__ void sub_outer_blk(double* __restrict__ s, int R0, int C1, const double* __restrict__ sa,
                                              const double* __restrict__ sb) {
  const int lane = ctid() & 63, i = lane & 15, kq = lane >> 4;
  doublex4 acc = blk_load(s + R0 * LDT + C1);
  // the 16-deep chunks' operands one chunk ahead (two register sets), same MFMA order
  double av[2][4], bv[2][4];
  auto load = [&](int buf, int kk) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      av[buf][q] = sa[(R0 + i) * LDT + 16 * kk + 4 * q + kq];
      bv[buf][q] = sb[(C1 + i) * LDT + 16 * kk + 4 * q + kq];
    }
  };
  load(0, 0);
#pragma unroll
  for (int kk = 0; kk < NK; ++kk) {
    if (kk + 1 < NK) load((kk + 1) & 1, kk + 1);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int q = 0; q < 4; ++q)
      acc = __builtin_amdgcn_mfma_f64_16x16x4f64(-av[kk & 1][q], bv[kk & 1][q], acc, 0, 0, 0);
    __builtin_amdgcn_sched_barrier(0);
  }
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
// col[16P + c] = 1 / L[16P + c][16P + c].  No pivot check in the sweep (each
// check is a VALU compare feeding scalar selects, 0.7 K cycles per panel,
// r05z_panel_probe.log): a non-positive (or NaN) pivot leaves a NaN or zero L
// diagonal, which factor_diag_tile's check_pivots finds after the last panel.
template <int P>
__device__ __forceinline__ void panel_factor(double* __restrict__ sF, double* __restrict__ col, int r) {
  constexpr int C0 = 16 * P;
  double a[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) a[j] = sF[r * LDT + C0 + j];
  double rs[16];
  // software pipeline: column c's pivot chain is issued before column c - 1's
  // remaining FMAs (only a[c] had to be updated first)
  double piv = read_lane_f64(a[0], C0);
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
                                                 const double* sPend = nullptr, bool active = true) {
  // active = false: the caller's idle waves take part in every barrier and do no work
  // (w = 4 matches no role), so the barrier sequence is the same for all waves
  const int w = active ? (ctid() >> 6) : 4, lane = ctid() & 63;
  const int js = (int)(gcol0 / CB) - 1;
  if (w == 0) {
    panel_factor<0>(sF, col, lane);
  } else if (w < 4 && sPend) {  // blocks (1,1), (2,1) | (3,1), (2,2) | (3,2), (3,3)
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
  } else if (w == 3) {
    for (int q = 0; q < 6; ++q) {  // upper blocks (i < j) of X are zero
      const int i = q < 3 ? 0 : (q < 5 ? 1 : 2), j = q < 3 ? q + 1 : (q < 5 ? q - 1 : 3);
      blk_store(sX + 16 * i * LDT + 16 * j, doublex4{0.0, 0.0, 0.0, 0.0});
    }
  }
  __syncthreads();
  STAMP(js, 9);
  if (w == 0) {
    panel_factor<1>(sF, col, lane);
  } else if (w == 1) {
    inv_diag_block(sF, sX, col, 0, lane);
  } else if (w == 2) {
    sub_outer_blk<1>(sF, 32, 32, P0, P0);  // update 0 of (2,2), (3,2)
    sub_outer_blk<1>(sF, 48, 32, P0, P0);
  } else if (w == 3) {
    sub_outer_blk<1>(sF, 48, 48, P0, P0);  // update 0 of (3,3)
  }
  STAMP(js, 10);
  __syncthreads();
  if (w < 2) sub_outer_blk<1>(sF, 32 + 16 * w, 32, sF + 16, sF + 16);  // update 1 of (2,2), (3,2)
  __syncthreads();
  STAMP(js, 11);
  if (w == 0) panel_factor<2>(sF, col, lane);
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
    panel_factor<3>(sF, col, lane);
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
  } else if (w == 3) {
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
  } else if (w == 3) {
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
  } else if (w == 3) {
    // pivot check (LAPACK info: the first column, 1-based, + gcol0): pivot c is
    // positive iff L_cc = piv * rsq(piv) is (NaN for a negative or NaN pivot, 0 * inf
    // for a zero one; an infinite pivot is reported too)
    const double d = sF[lane * LDT + lane];
    const unsigned long long nonpos = __ballot(!(d > 0.0));
    if (nonpos && lane == 0) atomicCAS(info, 0, (int32_t)(gcol0 + __ffsll(nonpos)));
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

// ------------------------------------------------------------------ prep launch
// MGP_K3_PREP_NT: the prep's Kuu tiles and zero fills stored non-temporal (fewer dirty L2
// lines for the write-back at the prep's end, in front of the first step launch)
#ifndef MGP_K3_PREP_NT
#define MGP_K3_PREP_NT 0
#endif
template <class T>
__device__ __forceinline__ void prep_store(T* p, T v) {
#if MGP_K3_PREP_NT
  __builtin_nontemporal_store(v, p);
#else
  *p = v;
#endif
}
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
  // The 64 x 64 Kuu tile (r0, c0) into dst (leading dimension ld): with Z in LDS
  // (rows r0.. as zr[64][D], columns c0.. transposed as zc[D][64], staged in the
  // scratch space `stage`, >= 2 * 64 * D floats) -- the same float64 arithmetic as
  // kuu_elem, without its 2 D dependent global loads per element.
  auto build_tile = [&](double* dst, int64_t ld, int64_t r0, int64_t c0, float* stage) {
    if (a.A || a.D > 32) {
      for (int idx = threadIdx.x; idx < CB * CB; idx += kCholThreads) {
        const int r = idx >> 6, c = idx & 63;
        prep_store(dst + (int64_t)r * ld + c, elem(r0 + r, c0 + c));
      }
      return;
    }
    const int D = a.D;
    float* zr = stage;
    float* zc = stage + CB * D;
    for (int idx = threadIdx.x; idx < CB * D; idx += kCholThreads) {
      const int r = idx / D, d = idx % D;
      zr[idx] = (r0 + r < a.M) ? Zb[(r0 + r) * a.ldz + d] : 0.f;
      zc[d * CB + r] = (c0 + r < a.M) ? Zb[(c0 + r) * a.ldz + d] : 0.f;
    }
    __syncthreads();
    for (int idx = threadIdx.x; idx < CB * CB; idx += kCholThreads) {
      const int r = idx >> 6, c = idx & 63;
      const int64_t gr = r0 + r, gc = c0 + c;
      double v;
      if (gr >= a.M || gc >= a.M) {
        v = gr == gc ? 1.0 : 0.0;
      } else {
        double sacc = 0.0;
        for (int d = 0; d < D; ++d) {
          const double diff = ((double)zr[r * D + d] - (double)zc[d * CB + c]) * sil[d];
          sacc = fma(diff, diff, sacc);
        }
        v = varb * exp(-0.5 * sacc);
        if (gr == gc) v += a.jitter;
      }
      prep_store(dst + (int64_t)r * ld + c, v);
    }
    __syncthreads();
  };
  if (blockIdx.x == 0) {  // factor tile (0, 0) straight from the input (dispatched first)
    STAMP(63, 0);
    RSTAMP(63, 14);
    if (threadIdx.x == 0) {
      a.info[b] = 0;
      float* lt = a.lt_absmax[0];
#pragma unroll
      for (int i = 1; i < kMaxBatch; ++i)
        if (b == i) lt = a.lt_absmax[i];
      if (lt) *lt = 0.f;
    }
    build_tile(s1, LDT, 0, 0, reinterpret_cast<float*>(s2));
    __syncthreads();
    STAMP(63, 1);
    factor_diag_tile(s1, s2, col, a.info + b, 0);
    __syncthreads();
    STAMP(63, 2);
    write_diag(a, b, 0, s1, s2);
    STAMP(63, 3);
    RSTAMP(63, 15);
    return;
  }
  const int bi = (blockIdx.x - 1) / a.nb, bl = (blockIdx.x - 1) % a.nb;
  const int64_t r0 = (int64_t)bi * CB, c0 = (int64_t)bl * CB;
  if (bl <= bi) build_tile(ws_tile(a, ws_W(a, b), bi, bl), CB, r0, c0, reinterpret_cast<float*>(s2));
  // zero L above / LinvT below the block diagonal (within M x M)
  if (bl != bi && (bl < bi || a.L)) {
    float* dst = (bl > bi ? a.L : a.LinvT) + (int64_t)b * a.strideL;
    for (int idx = threadIdx.x; idx < CB * CB; idx += kCholThreads) {
      const int r = idx >> 6, c = idx & 63;
      const int64_t gr = r0 + r, gc = c0 + c;
      if (gr < a.M && gc < a.M) prep_store(dst + gr * a.ldl + gc, 0.f);
    }
  }
}

// ------------------------------------------------------------------ step launch j
// The look-ahead's factorisation of tile (j+1, j+1): s1 holds P = L_{j+1,j}, s2 the
// tile with column block 0 of -P P^T still to apply.
__device__ __forceinline__ void lookahead_factor(const CholArgs& a, int b, int j, double* s1, double* s2,
                                                 double* col, bool active) {
  // column block 0 of W_ii -= P_i P_i^T (one block per wave); the other six
  // lower blocks are applied beside the first panel sweep
  if (active) sub_outer_blk<4>(s2, 16 * (ctid() >> 6), 0, s1, s1);
  __syncthreads();
  STAMP(j, 3);
  STAMP(j, 4);
  factor_diag_tile(s2, s1, col, a.info + b, (int64_t)(j + 1) * CB, s1, active);
  STAMP(j, 6);
  __syncthreads();
  if (active) write_diag(a, b, j + 1, s2, s1);
  __syncthreads();
  STAMP(j, 7);
  RSTAMP(j, 15);
}

// Last step (j = nb - 1, no trailing matrix): row block j of X = L^-1, X_jc = D_j B_jc
// (c < j) and X_jj = D_j, written transposed into L^-T; one workgroup per tile c.
__global__ __launch_bounds__(kCholThreads) void chol_last_step(CholArgs a, int j) {
  __shared__ double s1[CB * LDT], sD[CB * LDT];
  const int b = blockIdx.y;
  const int c = blockIdx.x;
  double* Bm = ws_B(a, b);
  float* LinvT = a.LinvT + (int64_t)b * a.strideL;
  float* lt_max = a.lt_absmax[0];  // this batch entry's max |L^-T| (no dynamic indexing of the arguments)
#pragma unroll
  for (int q = 1; q < kMaxBatch; ++q)
    if (b == q) lt_max = a.lt_absmax[q];
  auto store_linvT = [&](const double* sx) {  // X_jc -> LinvT block (c, j)
    const int64_t gr = (int64_t)c * CB, gc = (int64_t)j * CB;
    const float m = tile_store_f32_max(LinvT + gr * a.ldl + gc, a.ldl, sx, true, (int)min<int64_t>(CB, a.M - gr),
                                       (int)min<int64_t>(CB, a.M - gc));
    if (lt_max) wave_absmax_atomic(m, lt_max);
  };
  tile_load(sD, ws_D(a, b, j), CB);
  if (c < j) tile_load(s1, ws_tile(a, Bm, j, c), CB);
  __syncthreads();
  if (c < j) {   // (uniform per workgroup)
    Blk4 x = blk4_zero();
    col_mma_lower(x, sD, s1);
    __syncthreads();
    blk4_to_lds<false>(s1, x);
    __syncthreads();
    store_linvT(s1);
  } else {
    store_linvT(sD);
  }
}

// ------------------------------------------------------------------ step launch arguments
// chol_step_pair's leading scalar arguments are the ones its first tile loads need (the
// workspace, its strides, the step and the pair count); they come ahead of the CholArgs
// block so that the dispatch preloads them into SGPRs (chol.hip is compiled with
// -amdgpu-kernarg-preload-count, modulatedgps_amd/build.py).  Every other field is read
// from the kernel-argument segment behind the tile loads.  The layout below mirrors the
// kernel's parameter list (kernel arguments follow their natural alignment in order),
// giving the offset of the CholArgs block for the side job's dynamic-index reads.
struct StepPairKernargs {
  double* ws; int64_t strideWS, Mp; int nb, j, batch, Pb;
  CholArgs a;
};
constexpr size_t kStepArgsOffset = offsetof(StepPairKernargs, a);

// ------------------------------------------------------------------ Kuf side job
#ifndef MGP_KUF_SIDE_POLICY
#define MGP_KUF_SIDE_POLICY 1   // the side job's image stores (kuf_image.hpp img_store): non-temporal
#endif
// Kuf image blocks [k0, k1) (batch-major: block b * kblocks + bid is block bid of entry b's
// image) run by the `nkwg` extra workgroups of a step launch, two blocks per pass (one per
// 256-thread group).  The step kernel's LDS holds one of its workgroups per CU, so these
// workgroups take CUs the launch's tile workgroups leave idle; the blocks are the ones
// rbf_kuf_x6_kernel runs (same function, same bits).  Every pass is uniform across the
// workgroup (a group without a block joins the barriers).
template <int DM>
__device__ __forceinline__ void kuf_side_blocks(const CholArgs& a, int w, int64_t k0, int64_t k1, int nkwg,
                                                float* lds) {
  const int g = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 8));
  const int t = (int)(threadIdx.x & 255);
  const int64_t per = 2 * (int64_t)nkwg;
  const int64_t passes = (k1 - k0 + per - 1) / per;
  for (int64_t it = 0; it < passes; ++it) {
    const int64_t item = k0 + it * per + 2 * w + g;
    const bool active = item < k1;
    const int b = __builtin_amdgcn_readfirstlane(active ? (int)(item / a.kblocks) : 0);
    // this batch entry's operands: scalar loads from the kernel-argument segment at a
    // dynamic index (`a` is the by-value kernel argument at its offset 0; indexing `a`
    // itself would copy the whole struct to scratch)
    typedef const CholArgs __attribute__((address_space(4))) KernargCholArgs;
    const KernargCholArgs& ag = *(const KernargCholArgs*)(
        (const char __attribute__((address_space(4)))*)__builtin_amdgcn_kernarg_segment_ptr() + kStepArgsOffset);
    const KufImageArgs ka = {a.kx, a.kldx, ag.Z[b], a.ldz, a.kN, a.M, a.D, ag.var[b], ag.ls[b], ag.n_ls[b],
                             a.knmk, a.krow_blocks, ag.kfr[b], ag.kbound[b]};
    const int64_t bid = item - b * a.kblocks;
    if (a.kf16) kuf_image_block<DM, true, MGP_KUF_SIDE_POLICY>(ka, bid, t, active, lds);
    else kuf_image_block<DM, false, MGP_KUF_SIDE_POLICY>(ka, bid, t, active, lds);
  }
}

__device__ __forceinline__ void kuf_side_job(const CholArgs& a, int w, int64_t k0, int64_t k1, int nkwg, float* lds0,
                                          float* lds1) {
  float* lds = (threadIdx.x >> 8) ? lds1 : lds0;
  if (a.D <= 1) kuf_side_blocks<1>(a, w, k0, k1, nkwg, lds);
  else if (a.D <= 2) kuf_side_blocks<2>(a, w, k0, k1, nkwg, lds);
  else if (a.D <= 4) kuf_side_blocks<4>(a, w, k0, k1, nkwg, lds);
  else if (a.D <= 8) kuf_side_blocks<8>(a, w, k0, k1, nkwg, lds);
  else if (a.D <= 16) kuf_side_blocks<16>(a, w, k0, k1, nkwg, lds);
  else kuf_side_blocks<32>(a, w, k0, k1, nkwg, lds);
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
// Barriers are uniform: every __syncthreads of the kernel is reached by all eight waves of
// the workgroup on every path (the look-ahead's idle group joins each barrier of the
// factorisation with no work, lookahead_factor's `active`; after P_i the pair's two groups
// run their tiles' products barrier-free, and the diagonal tile's LDS hand-off barrier sits
// outside the tile-kind branches), so no barrier depends on which waves are still live.
// Row i's tiles in order: the heavy tiles first -- the off-diagonal update tiles (i, l),
// l = j + 1 .. i - 1 (rows i > j + 1), then the forward-substitution tiles (i, c), c < j --,
// then the two light ones, the diagonal tile (i, i) (rows i > j + 1) and (i, j) (X_jj = D_j,
// one triangular product).  A heavy tile runs three products (two of them full), a light
// one a triangular product only: with the light tiles adjacent they share a pair (a short
// workgroup) on every row whose tile count is even, instead of each holding a heavy tile's
// workgroup to the heavy tile's length with one group idle.
constexpr int kPairThreads = 2 * kCholThreads;
__host__ __device__ inline int step_row_tiles(int i, int j) { return i == j + 1 ? j + 1 : i + 1; }
__host__ __device__ inline int step_row_pairs(int i, int j) { return (step_row_tiles(i, j) + 1) / 2; }
__host__ __device__ inline int step_pair_count(int nb, int j) {  // per batch entry
  int n = 0;
  for (int i = j + 1; i < nb; ++i) n += step_row_pairs(i, j);
  return n;
}
// Workgroups of a step launch (one dimension, batch (1 + step_pair_count) of them): the
// batch's look-ahead workgroups first (workgroup b: batch entry b), then one per pair.
// The pairs, in the order (batch entry, tile row, pair), are cut into 8 consecutive runs,
// and run x goes to the workgroups w with (w - batch) % 8 == x, which share an XCD under
// the round-robin placement (speed only, nothing depends on it): a row's pairs then load
// its panel tile W_ij into one L2 and a run's rows (of one batch entry where the run
// does not straddle two) share the panel tiles W_lj, B_jc there.  No idle workgroups.
// Workgroups past batch (1 + Pb) (when the launch carries a Kuf side job): kuf_side_job
// over the image blocks [k0, k1), nkwg of them.
__global__ __launch_bounds__(kPairThreads) void chol_step_pair(double* pws, int64_t pstrideWS, int64_t pMp, int pnb,
                                                               int j, int batch, int Pb, CholArgs ain, int64_t k0,
                                                               int64_t k1, int nkwg) {
  __shared__ double s1[CB * LDT], sD[CB * LDT], s2[2][CB * LDT], col[CB];
  CholArgs a = ain;   // (fields read in place; the hot ones from the preloaded arguments)
  a.ws = pws;
  a.strideWS = pstrideWS;
  a.Mp = pMp;
  a.nb = pnb;
  if ((int)blockIdx.x >= batch * (1 + Pb)) {   // uniform per workgroup
    kuf_side_job(a, (int)blockIdx.x - batch * (1 + Pb), k0, k1, nkwg, reinterpret_cast<float*>(s1),
                 reinterpret_cast<float*>(sD));
    return;
  }
  ENTRYTIME(t_entry);
  // the other kernel arguments a workgroup reads, as one batch of scalar loads whose wait
  // sits behind the tile loads' issue (the compiler had placed each load at its first use:
  // dependent kernel-argument round trips, ~1 us each, in front of the first tile load)
  auto kernargs_in = [&]() {
    asm volatile("" ::"s"(a.M), "s"(a.L), "s"(a.LinvT), "s"(a.ldl), "s"(a.strideL), "s"(a.info));
    asm volatile("" ::"s"(a.lt_absmax[0]), "s"(a.lt_absmax[1]), "s"(a.lt_absmax[2]), "s"(a.lt_absmax[3]),
                 "s"(a.lt_absmax[4]), "s"(a.lt_absmax[5]), "s"(a.lt_absmax[6]), "s"(a.lt_absmax[7]));
  };
  const int g = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 8));  // tile group
  const int wg = blockIdx.x;
  // workgroup -> (batch entry, tile row, pair of the row): step_pair_count
  int b = wg, i = j + 1, q = 0;
  if (wg >= batch) {
    // Pb = step_pair_count(nb, j) from the host; position k in the pair order: run x
    // starts after the runs y < x, (P - y + 7) / 8 pairs each (m + 1 for y < P % 8, else m)
    const int P = batch * Pb, m = P >> 3, x = (wg - batch) & 7;
    int k = ((wg - batch) >> 3) + x * m + min(x, P & 7);
    b = k / Pb;
    k -= b * Pb;
    for (;; ++i) {
      const int np = step_row_pairs(i, j);
      if (k < np) break;
      k -= np;
    }
    q = k;
  }
  double* W = ws_W(a, b);
  double* Bm = ws_B(a, b);
  float* LinvT = a.LinvT + (int64_t)b * a.strideL;
  auto Wt = [&](int bi, int bl) { return ws_tile(a, W, bi, bl); };
  auto Bt = [&](int bi, int bl) { return ws_tile(a, Bm, bi, bl); };
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
  if (wg < batch) {
    // look-ahead: tile (j+1, j+1).  Both groups load and form P = W_{j+1,j} D_j^T (group 0
    // column blocks 0 and 3, group 1 blocks 1 and 2: equal MFMA counts, as the pairs'
    // P_i); the factorisation then runs on group 0 while group 1's waves take part in
    // every barrier and do no work (uniform barrier sequence)
    const bool act = g == 0;
    RSTAMP(j, 14);
    STAMP(j, 0);
    TileRegs r1, rD, r2;
    if (act) {
      tile_fetch(r1, Wt(i, j), CB);
      tile_fetch_lower(rD, ws_D(a, b, j), CB);
    } else {
      tile_fetch(r2, Wt(i, i), CB);
    }
    kernargs_in();
    if (act) {
      tile_put(s1, r1);
      tile_put(sD, rD);
    } else {
      tile_put(s2[0], r2);
    }
    __syncthreads();
    STAMP(j, 1);
    Blk4 pi = blk4_zero();
    if (act) row_mma<true, 1, 0x9>(pi, s1, sD, 1.0);
    else row_mma<true, 1, 0x6>(pi, s1, sD, 1.0);
    __syncthreads();
    if (act) blk4_to_lds<true, 0x9>(s1, pi);
    else blk4_to_lds<true, 0x6>(s1, pi);
    __syncthreads();
    STAMP(j, 2);
    lookahead_factor(a, b, j, s1, s2[0], col, act);
    return;
  }
  // pair q of row i: tiles e = 2 q, 2 q + 1 of the row
  const int nt = step_row_tiles(i, j);
  const int e = 2 * q + g;
  const bool has = e < nt;  // an odd row's last pair: group 1 has no tile (it forms its half of P_i)
  const bool pst = i == a.nb - 1 && q == 0 && b == 0;   // debug stamps only
  PAIRSTAMP_AT(pst, j, 7, t_entry);
  PAIRSTAMP(pst, j, 0);
  const int nh = (i == j + 1) ? 0 : i - j - 1;  // off-diagonal update tiles of the row
  int l = -1, c = -1;                              // update tile (i, l) or B tile (i, c)
  if (e < nh) l = j + 1 + e;
  else if (e < nh + j) c = e - nh;
  else if (i > j + 1 && e == nh + j) l = i;
  else c = j;
  const bool upd = has && l >= 0;
  const bool fwd = has && c >= 0 && c < j;  // forward-substitution tile reading B_jc
  const bool first = (upd && l != i) || fwd;  // P_l / X_jc before the update
  double* sT = s2[g];
  // this tile's operands: sT's tile (when it reads one) and the updated tile (u)
  TileRegs r1, rD, r2;
  Blk4 u = blk4_zero();  // B_ij is zero before step j
  if (g == 0) {
    tile_fetch(r1, Wt(i, j), CB);
    tile_fetch_lower(rD, ws_D(a, b, j), CB);
  }
  // one fetch site per operand, its source chosen by tile kind (one site per kind had the
  // compiler merge the kinds' pending loads and wait for most of group 0's loads before a
  // forward-substitution tile issued its own)
  const double* src2 = upd ? Wt(l != i ? l : i, l != i ? j : i) : fwd ? Bt(j, c) : nullptr;
  const double* srcu = (upd && l != i) ? Wt(i, l) : fwd ? Bt(i, c) : nullptr;
  if (src2) tile_fetch(r2, src2, CB);
  if (srcu) row_from_global(u, srcu, CB);
  kernargs_in();
#ifdef MGP_DBG_STAMPS
  __builtin_amdgcn_sched_barrier(0);
  PAIRSTAMP(pst, j, 6);  // every load issued
  __builtin_amdgcn_sched_barrier(0);
#endif
  if (g == 0) {
    tile_put(s1, r1);
    tile_put(sD, rD);
  }
  if (upd || fwd) tile_put(sT, r2);
  __syncthreads();
  PAIRSTAMP(pst, j, 1);
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
  PAIRSTAMP(pst, j, 2);
  if (g == 0) blk4_to_lds<true, 0x9>(s1, pi);
  else blk4_to_lds<true, 0x6>(s1, pi);
  if (first) upd ? blk4_to_lds<true>(sT, t) : blk4_to_lds<false>(sT, t);
  __syncthreads();
  PAIRSTAMP(pst, j, 3);
  if (g == 0 && q == 0 && a.L) {  // L_ij, once per row
    const int64_t gr = (int64_t)i * CB, gc = (int64_t)j * CB;
    tile_store_f32(a.L + (int64_t)b * a.strideL + gr * a.ldl + gc, a.ldl, s1, false,
                   (int)min<int64_t>(CB, a.M - gr), (int)min<int64_t>(CB, a.M - gc));
  }
  // the final products; the diagonal tile's LDS hand-off barrier is taken by every wave
  // of both groups (uniform barrier sequence; the other paths have no barrier here)
  const bool diag = upd && l == i;
  if (upd && l != i) {
    row_mma<true, 0>(u, s1, sT, -1.0);    // W_il -= P_i P_l^T
    row_to_global(Wt(i, l), CB, u);
  } else if (diag) {                       // diagonal tile (i, i): lower blocks of W_ii -= P_i P_i^T
    diag_lower_update(sT, s1);
  } else if (fwd) {
    if (i == j + 1) store_linvT(c, sT);
    row_mma<false, 0>(u, s1, sT, -1.0);    // B_ic -= P_i X_jc
    row_to_global(Bt(i, c), CB, u);
  } else if (has) {                        // X_jj = D_j (lower triangular)
    if (i == j + 1) store_linvT(c, sD);
    row_mma<false, 2>(u, s1, sD, -1.0);
    row_to_global(Bt(i, c), CB, u);
  }
  PAIRSTAMP(pst, j, 4);
  __syncthreads();
  if (diag) tile_store_f64(Wt(i, i), CB, sT);
  PAIRSTAMP(pst, j, 5);
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
//     consumer reads only the lower triangle / never reaches them);
//   | kPhiOut: C = Phi(op(A) op(B)) (lower triangle, diagonal halved, zeros above).
// blockIdx.z: the layer; A, B and C advance by zs doubles per layer.
constexpr int kTriNone = 0, kTriUpperK = 1, kTriBand = 2, kTriLowerOut = 4, kPhiOut = 8;
template <bool TA, bool TB, int BN = 64, int KC = 16>
__global__ __launch_bounds__(256) void dgemm_kernel(const double* __restrict__ A, int64_t lda,
                                                    const double* __restrict__ B, int64_t ldb,
                                                    double* __restrict__ C, int64_t ldc, int64_t M, int tri,
                                                    int64_t zs) {
  A += blockIdx.z * zs;
  B += blockIdx.z * zs;
  C += blockIdx.z * zs;
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
        const double v = acc[a][b][r];
        if (i < M && j < M) C[i * ldc + j] = !(tri & kPhiOut) ? v : (j < i ? v : (j == i ? 0.5 * v : 0.0));
      }
}

// The float32 operands and outputs of up to kMaxBatch layers; the float64 workspace
// holds per layer b, at b * 4 M^2 doubles: Ld = L, Li = Linv = LinvT^T, G = gL, T.
struct CholBwdIO {
  const float* L[kMaxBatch]; const float* LinvT[kMaxBatch]; const float* gL[kMaxBatch]; float* gKuu[kMaxBatch];
  int64_t ldl, ldli, ldg, ldo;
};

// grid (ceil(M^2 / 256), 3, batch): y = 0 Ld = f64(L), 1 Li = f64(LinvT^T), 2 G = f64(gL)
__global__ __launch_bounds__(256) void chol_bwd_convert_kernel(CholBwdIO io, double* __restrict__ ws, int64_t M) {
  const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (idx >= M * M) return;
  const int64_t i = idx / M, j = idx % M;
  const int b = blockIdx.z, y = blockIdx.y;
  double* d = ws + (int64_t)b * 4 * M * M + (int64_t)y * M * M;
  if (y == 0) d[idx] = (double)io.L[b][i * io.ldl + j];
  else if (y == 1) d[idx] = (double)io.LinvT[b][j * io.ldli + i];
  else d[idx] = (double)io.gL[b][i * io.ldg + j];
}

// gKuu = (S + S^T) / 2 -> f32, S = T of layer blockIdx.y
__global__ __launch_bounds__(256) void chol_bwd_sym_kernel(CholBwdIO io, const double* __restrict__ ws, int64_t M) {
  const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (idx >= M * M) return;
  const int64_t i = idx / M, j = idx % M;
  const double* T = ws + (int64_t)blockIdx.y * 4 * M * M + 3 * M * M;
  io.gKuu[blockIdx.y][i * io.ldo + j] = (float)(0.5 * (T[i * M + j] + T[j * M + i]));
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
extern "C" int mgp_dbg_pair_stamps(unsigned long long* host) {
  return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(g_pair_stamps), sizeof(g_pair_stamps));
}
#endif

// the doubles of every batch entry (W, B, D; chol_ws_doubles_per_batch)
extern "C" size_t mgp_chol_workspace_bytes(int64_t M, int32_t batch) {
  if (M <= 0 || batch <= 0) return 0;
  return (size_t)chol_ws_doubles_per_batch(M) * (size_t)batch * sizeof(double);
}

// The Kuf side job of a factorisation (mgp_kuu_potrf_trtri_kuf): X [N][ldx] and one image per
// batch entry (split-f16 when f16, else split-bf16), each of at least mgp_x6_cols_bytes(M, N).
struct KufSideJob {
  const float* X; int64_t ldx, N;
  void* const* Kfr; bool f16;
};

extern "C" size_t mgp_x6_cols_bytes(int64_t M, int64_t N);

// Share of the image blocks per step launch j: proportional to the CUs the launch's tile
// workgroups leave idle (one workgroup per CU: the step kernel's LDS), at least an eighth
// of the CUs each.
// CU count of the device the stream runs on, cached per device (the attribute query
// costs a driver call on every K3 launch otherwise).
static int stream_device_cus(hipStream_t s) {
  static std::atomic<int> cache[64];
  int dev = 0;
  if (hipStreamGetDevice(s, &dev) != hipSuccess && hipGetDevice(&dev) != hipSuccess) return 256;
  if (dev < 0 || dev >= 64) dev = 0;
  int cus = cache[dev].load(std::memory_order_relaxed);
  if (cus > 0) return cus;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) cus = 256;
  cache[dev].store(cus, std::memory_order_relaxed);
  return cus;
}

static void kuf_side_split(int nb, int batch, int64_t total, std::vector<int64_t>& beg, std::vector<int>& nwg,
                           hipStream_t s) {
  const int cus = stream_device_cus(s);
  const int steps = nb - 1;
  std::vector<double> idle(steps);
  double sum = 0.0;
  for (int j = 0; j < steps; ++j) {
    idle[j] = std::max<double>(cus - batch * (1 + step_pair_count(nb, j)), cus / 8.0);
    sum += idle[j];
  }
  beg.assign(steps + 1, 0);
  nwg.assign(steps, 0);
  double acc = 0.0;
  for (int j = 0; j < steps; ++j) {
    acc += idle[j];
    beg[j + 1] = j + 1 == steps ? total : std::min<int64_t>(total, (int64_t)(total * (acc / sum) + 0.5));
    const int64_t cnt = beg[j + 1] - beg[j];
    // at least one workgroup for a step that was given image blocks (idle[j] can be
    // < 1 on a device or partition with fewer than 8 CUs)
    nwg[j] = cnt > 0 ? (int)std::max<int64_t>(1, std::min<int64_t>((cnt + 1) / 2, (int64_t)idle[j])) : 0;
  }
}

static int chol_run(CholArgs& a, int batch, void* workspace, size_t workspace_bytes, hipStream_t s,
                    hipEvent_t prep_done = nullptr, const KufSideJob* kj = nullptr) {
  if (!workspace || workspace_bytes < mgp_chol_workspace_bytes(a.M, batch)) return MGP_ERR_WORKSPACE;
  if (!aligned16(workspace)) return MGP_ERR_ALIGN;
  // the diagonal tiles of L and L^-T are written with 16-byte stores
  const bool lay4 = a.ldl % 4 == 0 && (batch <= 1 || a.strideL % 4 == 0);
  if ((a.L && !aligned16(a.L)) || (a.LinvT && !aligned16(a.LinvT)) || !lay4) return MGP_ERR_ALIGN;
  a.Mp = chol_mp(a.M);
  a.nb = (int)(a.Mp / CB);
  a.strideWS = chol_ws_doubles_per_batch(a.M);
  a.ws = (double*)workspace;
  const dim3 block(kCholThreads);
  std::vector<int64_t> kbeg;
  std::vector<int> knwg;
  if (kj && kj->N > 0 && a.M > 0) {
    a.kx = kj->X; a.kldx = kj->ldx; a.kN = kj->N; a.kf16 = kj->f16 ? 1 : 0;
    const int64_t mp = (a.M + 127) / 128 * 128;
    a.knmk = (int)(mp / 16);
    a.krow_blocks = kuf_row_blocks(a.M);
    a.kblocks = kuf_blocks(a.M, kj->N);
    for (int b = 0; b < batch; ++b) {
      a.kfr[b] = (bf16x8*)kj->Kfr[b];
      a.kbound[b] = (float*)((char*)kj->Kfr[b] + mgp_x6_cols_bytes(a.M, kj->N) - 256);  // image trailer
    }
    if (a.nb >= 2) kuf_side_split(a.nb, batch, batch * a.kblocks, kbeg, knwg, s);
  }
  hipLaunchKernelGGL(chol_prep, dim3(a.nb * a.nb + 1, batch), block, 0, s, a);
  int st = launch_status();
  if (st) return st;
  if (prep_done) {
    st = hip_status(hipEventRecord(prep_done, s));
    if (st) return st;
  }
  if (kj && kj->N > 0 && a.M > 0 && a.nb < 2) {   // no step launches to carry the job: K1's own launches
    for (int b = 0; b < batch; ++b) {
      st = kj->f16 ? mgp_rbf_kuf_f16(kj->X, kj->ldx, a.Z[b], a.ldz, kj->N, a.M, a.D, a.var[b], a.ls[b], a.n_ls[b],
                                     kj->Kfr[b], mgp_x6_cols_bytes(a.M, kj->N), s)
                   : mgp_rbf_kuf_x6(kj->X, kj->ldx, a.Z[b], a.ldz, kj->N, a.M, a.D, a.var[b], a.ls[b], a.n_ls[b],
                                    kj->Kfr[b], mgp_x6_cols_bytes(a.M, kj->N), s);
      if (st) return st;
    }
  }
  for (int j = 0; j < a.nb; ++j) {
    const int T = a.nb - j - 1;
    if (T > 0) {
      const int Pb = step_pair_count(a.nb, j);
      const bool side = !kbeg.empty() && knwg[j] > 0;
      const int nkwg = side ? knwg[j] : 0;
      hipLaunchKernelGGL(chol_step_pair, dim3(batch * (1 + Pb) + nkwg), dim3(kPairThreads), 0, s, a.ws, a.strideWS,
                         a.Mp, a.nb, j, batch, Pb, a, side ? kbeg[j] : (int64_t)0, side ? kbeg[j + 1] : (int64_t)0,
                         nkwg);
    } else {
      hipLaunchKernelGGL(chol_last_step, dim3(a.nb, batch), block, 0, s, a, j);
    }
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
                                   float* const* lt_absmax, mgp_stream_t stream,
                                   const KufSideJob* kj = nullptr) {
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
  return chol_run(a, batch, workspace, workspace_bytes, (hipStream_t)stream, prep_done, kj);
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

extern "C" int mgp_kuu_potrf_trtri_kuf(const float* const* Z, int64_t ldz, int64_t M, int32_t D,
                                       const float* const* variance, const float* const* lengthscales,
                                       const int32_t* n_ls, float jitter, int32_t batch, float* L,
                                       float* LinvT, int64_t ldl, int64_t strideL, int32_t* info,
                                       void* workspace, size_t workspace_bytes, void* prep_done,
                                       float* const* linvt_absmax, const float* X, int64_t ldx, int64_t N,
                                       void* const* Kfr, size_t kfr_bytes, int32_t kfr_format,
                                       mgp_stream_t stream) {
  if (!X) return -19;
  if (ldx < D) return -20;
  if (N < 0) return -21;
  if (!Kfr) return -22;
  if (kfr_format != 0 && kfr_format != 1) return -24;
  if (D > 32) return MGP_ERR_UNSUPPORTED;
  if (M > 0 && N > 0 && batch > 0 && batch <= kMaxBatch) {
    if (kfr_bytes < mgp_x6_cols_bytes(M, N)) return -23;
    for (int b = 0; b < batch; ++b) {
      if (!Kfr[b]) return -22;
      if (!aligned16(Kfr[b])) return MGP_ERR_ALIGN;
    }
  }
  const KufSideJob kj = {X, ldx, N, Kfr, kfr_format == 1};
  return kuu_potrf_trtri_impl(Z, ldz, M, D, variance, lengthscales, n_ls, jitter, batch, L, LinvT, ldl, strideL,
                              info, workspace, workspace_bytes, (hipEvent_t)prep_done, linvt_absmax, stream, &kj);
}

extern "C" size_t mgp_chol_backward_workspace_bytes(int64_t M) {
  return (size_t)(M > 0 ? M : 1) * (size_t)(M > 0 ? M : 1) * 4 * sizeof(double);
}

// both layers' Cholesky backward in five launches: the conversions, the three
// products (blockIdx.z = layer, Phi folded into the first one's store) and the
// symmetrisation -- the same float64 operations in the same order as per layer
static int chol_backward_impl(const CholBwdIO& io, int batch, int64_t M, void* workspace, hipStream_t s) {
  constexpr int KCB = 32;  // chunk depth of the products (32: half the barriers of 16)
  double* Ld = (double*)workspace;
  double* Li = Ld + M * M;  // Linv = LinvT^T
  double* G = Li + M * M;
  double* T = G + M * M;
  const int64_t zs = 4 * M * M;
  const unsigned ne = (unsigned)((M * M + 255) / 256);
  const dim3 gg((unsigned)((M + 31) / 32), (unsigned)((M + 63) / 64), (unsigned)batch);  // 64 x 32 tiles: 2 x the workgroups of 64 x 64 (measured faster at M = 1024)
  hipLaunchKernelGGL(chol_bwd_convert_kernel, dim3(ne, 3, (unsigned)batch), dim3(256), 0, s, io, Ld, M);
  // L, gL, Linv are lower triangular (exact zeros above), so are P and P Linv: the
  // products skip the zero terms and the tiles Phi / the next product never read
  hipLaunchKernelGGL((dgemm_kernel<true, false, 32, KCB>), gg, dim3(256), 0, s, Ld, M, G, M, T, M, M,
                     kTriUpperK | kTriLowerOut | kPhiOut, zs);                                          // Phi(L^T gL)
  hipLaunchKernelGGL((dgemm_kernel<false, false, 32, KCB>), gg, dim3(256), 0, s, T, M, Li, M, G, M, M,
                     kTriBand | kTriLowerOut, zs);                                                    // P Linv
  hipLaunchKernelGGL((dgemm_kernel<true, false, 32, KCB>), gg, dim3(256), 0, s, Li, M, G, M, T, M, M,
                     kTriUpperK, zs);                                                                 // Linv^T (.)
  hipLaunchKernelGGL(chol_bwd_sym_kernel, dim3(ne, (unsigned)batch), dim3(256), 0, s, io, Ld, M);
  return launch_status();
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
  CholBwdIO io = {};
  io.L[0] = L, io.LinvT[0] = LinvT, io.gL[0] = gL, io.gKuu[0] = gKuu;
  io.ldl = ldl, io.ldli = ldli, io.ldg = ldg, io.ldo = ldo;
  return chol_backward_impl(io, 1, M, workspace, (hipStream_t)stream);
}

extern "C" int mgp_chol_backward_batch(int32_t batch, const float* const* L, int64_t ldl, const float* const* LinvT,
                                       int64_t ldli, const float* const* gL, int64_t ldg, int64_t M,
                                       float* const* gKuu, int64_t ldo, void* workspace, size_t workspace_bytes,
                                       mgp_stream_t stream) {
  if (batch < 1 || batch > kMaxBatch) return -1;
  if (!L) return -2;
  if (ldl < M) return -3;
  if (!LinvT) return -4;
  if (ldli < M) return -5;
  if (!gL) return -6;
  if (ldg < M) return -7;
  if (M < 0) return -8;
  if (!gKuu) return -9;
  if (ldo < M) return -10;
  CholBwdIO io = {};
  for (int b = 0; b < batch; ++b) {
    if (!L[b]) return -2;
    if (!LinvT[b]) return -4;
    if (!gL[b]) return -6;
    if (!gKuu[b]) return -9;
    io.L[b] = L[b], io.LinvT[b] = LinvT[b], io.gL[b] = gL[b], io.gKuu[b] = gKuu[b];
  }
  if (M == 0) return MGP_OK;
  if (!workspace || workspace_bytes < (size_t)batch * mgp_chol_backward_workspace_bytes(M)) return MGP_ERR_WORKSPACE;
  io.ldl = ldl, io.ldli = ldli, io.ldg = ldg, io.ldo = ldo;
  return chol_backward_impl(io, batch, M, workspace, (hipStream_t)stream);
}
