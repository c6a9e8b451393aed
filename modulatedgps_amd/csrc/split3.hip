// K5 on the bf16 matrix cores at f32 accuracy ("split-bf16 x6").
//
// Reference: the same contraction as trigemm.hip's K5 -- for every expert k,
// fvar[k][n] += sum_m' (L_k^T A)[m'][n]^2 with L_k = band_part(q_sqrt[k], -1, 0)
// (GPflow base_conditional, reached from MixtureGPs/models.py:141-143).
//
// Every f32 operand x is split exactly into three bf16 planes,
//     x = hi + mid + lo (+ |x| 2^-25 at most),   hi = bf16(x), mid = bf16(x - hi),
//     lo = bf16(x - hi - mid)
// (each difference is exact in f32).  A product is formed from the six plane
// products whose weight is >= 2^-16 of the leading one,
//     a b ~ a_hi b_hi + a_hi b_mid + a_mid b_hi + a_hi b_lo + a_mid b_mid + a_lo b_hi,
// so the per-product error is a few f32 ulps and the sum is accumulated in the
// f32 MFMA accumulator -- the accuracy class of an f32 GEMM.  Six
// v_mfma_f32_32x32x16_bf16 (32 cycles each for 32x32x16) replace eight
// v_mfma_f32_32x32x2_f32 (64 cycles each for 32x32x2): 192 vs 512 cycles per
// 32x32x16 block, 2.7x the f32 matrix rate on the same silicon.
//
// Data layout ("fragment images", built once per step, 6 B per element):
//   Lfr[k][mb][mk][p][lane][8]  A-operand of (L_k)^T: lane (r = lane&31,
//       h = lane>>5), element j holds L_k[m][m'] with m' = 32 mb + r and
//       m = 16 mk + kperm(h, j), kperm(h, j) = (j&3) + 8 (j>>2) + 4 h; zero above
//       the diagonal (m < m') and outside M.
//   Afr[nb][mk][p][lane][8]     B-operand of A: element j holds
//       A[16 mk + kperm(h, j)][32 nb + r]; zero outside M x N.
// kperm is the row order in which a 32x32 MFMA accumulator holds its rows
// (register 8s + j of lane half h is row 16 s + kperm(h, j)), so K4's epilogue
// can emit A's image straight from its accumulators; both operands use the
// same k order, which leaves the contraction unchanged.
// Each fragment is 1 KiB contiguous per plane: a wave reads it with one
// coalesced 16-B-per-lane load (global for A, LDS for L), no transposes.
//
// K5x6 kernel: one 256-thread workgroup per item (expert k, row tile t of 128
// rows m', column tile of 256 n).  Wave w owns all 128 rows x 64 columns
// (4 x 2 accumulators of 32x32).  Per k-step (16 rows of m): the workgroup
// stages the 12 KiB of L fragments of its 4 row sub-tiles in LDS (double
// buffered, one barrier per k-step); each wave loads its 6 A fragments (6 KiB)
// straight from global into registers one k-step ahead; 48 MFMAs per wave.
// The triangle is exploited at row-tile granularity (k-steps start at 128 t);
// the zero blocks inside the diagonal tile come from Lfr's zero fill.
#include <stdlib.h>

#include <algorithm>
#include <type_traits>

#include "mgp_common.hpp"
#include "qsqrt_jobs.hpp"

#ifndef MGP_K4_STORE_NT
#define MGP_K4_STORE_NT 1   // K4's A-image stores non-temporal (0: plain, for A/B builds)
#endif

namespace mgp {

// Debug builds only (-DMGP_DBG_STAMPS, tools/k4_stamps.py): K4 phase times per
// workgroup on the 100 MHz reference clock (one time base for every CU).
#ifdef MGP_DBG_STAMPS
__device__ unsigned long long g_k4_stamps[4096 * 8];
#define K4STAMP(i, k) do { if (threadIdx.x == 0 && (i) >= 0 && (i) < 4096) g_k4_stamps[(i) * 8 + (k)] = __builtin_amdgcn_s_memrealtime(); } while (0)
#else
#define K4STAMP(i, k) do {} while (0)
#endif

constexpr int kX6BM = 128;   // rows m' per item
constexpr int kX6BN = 256;   // columns n per item
constexpr int kFragBytes = 1024;

// A-operand image of a batch of triangular matrices: element (k-row m, row m')
// = S_b[m][m'] kept where m >= m' (LOWER: L_k = tril(q_sqrt[k]), K5) or m <= m'
// (upper: LinvT, K4's T[k][i] = L^-T[k][i]).  One wave per fragment block
// (b, mb, mk): grid.x = batch * nmb * nmk / 4.
// TRANS: the source is stored transposed (element (m, m') read at S[m' ld + m]).
// bound != nullptr: split-f16 image, scaled by 2^img_exp(*bound).
template <bool LOWER, bool TRANS = false, bool FULL = false>
__global__ __launch_bounds__(256) void split_tri_kernel(const float* __restrict__ src, int64_t ld,
                                                        int64_t stride, int64_t M, int nmb, int nmk,
                                                        int64_t nfrag, bf16x8* __restrict__ img,
                                                        const float* __restrict__ bound = nullptr) {
  // (a grid of fewer than nfrag / 4 workgroups walks the fragments with a stride)
  for (int64_t f = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); f < nfrag; f += (int64_t)gridDim.x * 4)
    split_tri_frag<LOWER, TRANS, FULL>(src, ld, stride, M, nmb, nmk, f, threadIdx.x & 63, img, bound);
}

// ------------------------------------------------------------------ tril(q_sqrt) work of two layers
// mgp_qsqrt_images_kl_f16_batch: the split-f16 images of tril(q_sqrt) and the whitened KL
// terms of both SMGP layers in three launches (blockIdx.y / x = the layer) instead of five
// per layer (bound memset, absmax, split, KL partials, KL final): the KL partial sums also
// fold the images' scale bounds (the maxima of the lower triangles they read), the final
// launch writes both KL terms and both bounds, the split launch follows.  Same sums in the
// same order and the same bound as the per-layer launches: bit-identical results.
struct QLayer {
  const float* q_mu;
  const float* q_sqrt;
  bf16x8* Lfr;
  float* bound;     // Lfr's trailer
  double* kl_out;
  double* part;     // [nblk][3] partial sums
  float* bmax;      // [nblk] block maxima
};

// The tril(q_sqrt) work runs on the side stream beside K3's chain: with MGP_QS_GRID > 0 its
// two wide launches (the KL partials and the image split) walk their blocks / fragments in a
// grid-stride loop over at most MGP_QS_GRID workgroups per layer, so that they hold fewer CUs
// while the chain's step launches dispatch (same per-block and per-fragment work: the same bits;
// 256 against the full grids: ELBO step 3.186-3.234 vs 3.229-3.238 ms and c4r 0.696-0.700 vs
// 0.702-0.706 ms on one box, even on another, profiles/r06v_qsqrt_side_grid_ab.log, r06w_*;
// 16 or 64 put the side work on the critical path).
#ifndef MGP_QS_GRID
#define MGP_QS_GRID 256
#endif
constexpr int kQsGrid = MGP_QS_GRID;

__global__ __launch_bounds__(256) void kl_absmax2_kernel(QLayer l0, QLayer l1, int64_t ldq, int64_t ldqs,
                                                         int64_t strideq, int64_t M, int K, int nrb, int nblk) {
  __shared__ double scratch[16];
  __shared__ float smax[4];
  const QLayer& l = blockIdx.y ? l1 : l0;
  for (int blk = blockIdx.x; blk < nblk; blk += gridDim.x) {   // (uniform per workgroup)
    const KlPartial r = kl_partials_thread(l.q_mu, ldq, l.q_sqrt, ldqs, strideq, M, K, nrb, blk, threadIdx.x, 256);
    const float m = wave_max_f32(r.amax);
    if ((threadIdx.x & 63) == 0) smax[threadIdx.x >> 6] = m;
    const double a = block_sum<double>((double)r.tr, scratch);   // (its barriers publish smax)
    const double b = block_sum<double>((double)r.ld, scratch);
    const double c = block_sum<double>((double)r.mh, scratch);
    if (threadIdx.x == 0) {
      l.part[3 * blk + 0] = a;
      l.part[3 * blk + 1] = b;
      l.part[3 * blk + 2] = c;
      l.bmax[blk] = fmaxf(fmaxf(smax[0], smax[1]), fmaxf(smax[2], smax[3]));
    }
    __syncthreads();   // smax / scratch reused by the next block
  }
}

// One 1024-thread block per layer: kl_final_kernel's sums, and the image bound.
__global__ __launch_bounds__(1024) void kl_final2_kernel(QLayer l0, QLayer l1, int nblk, double MK) {
  __shared__ double scratch[16];
  __shared__ float smax[16];
  const QLayer& l = blockIdx.x ? l1 : l0;
  double tr, ld, mh;
  kl_final_thread(l.part, nblk, threadIdx.x, 1024, tr, ld, mh);
  float m = 0.f;
  for (int i = threadIdx.x; i < nblk; i += 1024) m = fmaxf(m, l.bmax[i]);
  m = wave_max_f32(m);
  if ((threadIdx.x & 63) == 0) smax[threadIdx.x >> 6] = m;
  tr = block_sum<double>(tr, scratch);   // (its barriers publish smax)
  ld = block_sum<double>(ld, scratch);
  mh = block_sum<double>(mh, scratch);
  if (threadIdx.x == 0) {
    *l.kl_out = 0.5 * (mh - MK - ld + tr);
    float b = 0.f;
    for (int i = 0; i < 16; ++i) b = fmaxf(b, smax[i]);
    *l.bound = b;
  }
}

__global__ __launch_bounds__(256) void split_lower2_kernel(QLayer l0, QLayer l1, int64_t ldqs, int64_t strideq,
                                                           int64_t M, int nmb, int nmk, int64_t nfrag) {
  const QLayer& l = blockIdx.y ? l1 : l0;
  for (int64_t f = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); f < nfrag; f += (int64_t)gridDim.x * 4)
    split_tri_frag<true>(l.q_sqrt, ldqs, strideq, M, nmb, nmk, f, threadIdx.x & 63, l.Lfr, l.bound);
}

// split_tri_kernel<false> (the split-f16 L^-T images) for two matrices at src and
// src + stride into two images in one launch: blockIdx.y = the matrix (same fragments,
// same arithmetic as two launches: bit-identical).
__global__ __launch_bounds__(256) void split_upper2_kernel(const float* __restrict__ src, int64_t ld, int64_t stride,
                                                           int64_t M, int nmb, int nmk, int64_t nfrag,
                                                           bf16x8* __restrict__ img0, const float* __restrict__ bound0,
                                                           bf16x8* __restrict__ img1,
                                                           const float* __restrict__ bound1) {
  const int64_t f = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (f >= nfrag) return;
  const bool second = blockIdx.y != 0;
  bf16x8* img = second ? img1 : img0;
  const float* bound = second ? bound1 : bound0;
  const int lane = threadIdx.x & 63, r = lane & 31, h = lane >> 5;
  const int mk = (int)(f % nmk);
  const int mb = (int)((f / nmk) % nmb);
  const int64_t mc = 32 * (int64_t)mb + r;
  const float* S = src + (second ? stride : 0);
  float v[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int64_t m = 16 * (int64_t)mk + kperm(h, j);
    v[j] = (m < M && mc < M && m <= mc) ? S[m * ld + mc] : 0.f;
  }
  store_split_f16<true>(img + f * 3 * 64 + lane, v, ldexpf(1.f, img_exp(*bound)));
}

// One wave per fragment block (nb, mk): grid.x = nnb * nmk / 4.
__global__ __launch_bounds__(256) void split_cols_kernel(const float* __restrict__ A, int64_t lda, int64_t M,
                                                         int64_t N, int nmk, int64_t nfrag,
                                                         bf16x8* __restrict__ Afr,
                                                         const float* __restrict__ bound = nullptr) {
  const int64_t f = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (f >= nfrag) return;
  const int lane = threadIdx.x & 63, r = lane & 31, h = lane >> 5;
  const int mk = (int)(f % nmk);
  const int64_t n = 32 * (f / nmk) + r;
  float v[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int64_t m = 16 * (int64_t)mk + kperm(h, j);
    v[j] = (m < M && n < N) ? A[m * lda + n] : 0.f;
  }
  if (bound)
    store_split_f16<true>(Afr + f * 3 * 64 + lane, v, ldexpf(1.f, img_exp(*bound)));
  else
    store_split(Afr + f * 3 * 64 + lane, v);
}

// max |x| over a batch of row-major matrices (rows x cols; TRI 0: all entries,
// 1: column <= row, 2: column >= row) -> *out as float bits through atomicMax
// (non-negative floats order as their bit patterns; *out zeroed beforehand).
// Waves stride over rows; one atomic per workgroup after an LDS reduction (a
// same-address atomic per wave serialises at the L2: 96 us at K M = 8192 rows).
template <int TRI>
__global__ __launch_bounds__(256) void absmax_kernel(const float* __restrict__ src, int64_t ld, int64_t stride,
                                                     int64_t rows, int64_t cols, int64_t nrows_total,
                                                     unsigned int* __restrict__ out) {
  __shared__ float red[4];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  // TRI 0: blockIdx.y strides over column chunks of kAbsChunk (few long rows)
  constexpr int64_t kAbsChunk = 8192;
  float m = 0.f;
  for (int64_t gr = (int64_t)blockIdx.x * 4 + w; gr < nrows_total; gr += (int64_t)gridDim.x * 4) {
    const int64_t b = gr / rows, r = gr % rows;
    const float* row = src + b * stride + r * ld;
    int64_t c0 = TRI == 2 ? r : 0;
    int64_t c1 = TRI == 1 ? (r + 1 < cols ? r + 1 : cols) : cols;
    if (TRI == 0) {
      c0 = (int64_t)blockIdx.y * kAbsChunk;
      c1 = c0 + kAbsChunk < cols ? c0 + kAbsChunk : cols;
    }
    if (TRI != 2 && (ld & 3) == 0 && ((uintptr_t)row & 15) == 0) {  // float4 loads (c0 % 4 == 0), scalar tail
      const int64_t c4 = c0 + ((c1 - c0) & ~(int64_t)3);
#pragma unroll 4
      for (int64_t c = c0 + 4 * lane; c < c4; c += 256) {
        const float4 v = *reinterpret_cast<const float4*>(row + c);
        m = fmaxf(m, fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w))));
      }
      for (int64_t c = c4 + lane; c < c1; c += 64) m = fmaxf(m, fabsf(row[c]));
    } else {
      for (int64_t c = c0 + lane; c < c1; c += 64) m = fmaxf(m, fabsf(row[c]));
    }
  }
  m = fmaxf(m, __shfl_xor(m, 32, 64));
  m = fmaxf(m, __shfl_xor(m, 16, 64));
  m = fmaxf(m, __shfl_xor(m, 8, 64));
  m = fmaxf(m, __shfl_xor(m, 4, 64));
  m = fmaxf(m, __shfl_xor(m, 2, 64));
  m = fmaxf(m, __shfl_xor(m, 1, 64));
  if (lane == 0) red[w] = m;
  __syncthreads();
  if (threadIdx.x == 0) atomicMax(out, __float_as_uint(fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]))));
}

// Launch shape of absmax_kernel<TRI>: <= 1024 row groups (one atomic per workgroup; 256
// left the reduction of K q_sqrt triangles latency-bound at 34 us for 32 MB, round 4);
// TRI 0 adds column chunks so a few long rows still fill the chip.
template <int TRI>
static void launch_absmax(const float* src, int64_t ld, int64_t stride, int64_t rows, int64_t cols,
                          int64_t nrows_total, float* out, hipStream_t s) {
  const int64_t gx = std::min<int64_t>((nrows_total + 3) / 4, TRI == 0 ? 64 : 1024);
  const int64_t gy = TRI == 0 ? std::min<int64_t>((cols + 8191) / 8192, 64) : 1;
  hipLaunchKernelGGL(absmax_kernel<TRI>, dim3((unsigned)gx, (unsigned)gy), dim3(256), 0, s, src, ld, stride, rows,
                     cols, nrows_total, (unsigned int*)out);
}

__device__ __forceinline__ bf16x8 ld_frag(__amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff) {
  return __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(r, voff, soff, 0));
}

// Item b -> (row tile t heavy-first, column tile tn, expert k); the K experts of
// a column tile are 8 block ids apart (one XCD) when nTn % 8 == 0.
// TN_OUTER: per XCD, one column tile at a time with all its row tiles (heavy first)
// and experts, so A's column slab is fetched about once instead of once per row tile
// (the 32x32x16 C-writing K5 of round 2: 1.60 -> 1.51 ms; without the C writes the
// row-tile-outer order was faster, 1.33 vs 1.36 ms).  The 16x16x32 kernels use the
// row-tile-outer order for both (MGP_K5C_TN_OUTER).
template <bool TN_OUTER = false>
__device__ __forceinline__ void x6_item(int b, int nTn, int K, int& t, int& tn, int& k, int grid = -1) {
  if (TN_OUTER && nTn % 8 == 0) {
    const int nT = (grid < 0 ? (int)gridDim.x : grid) / (nTn * K);
    const int x = b & 7, j = b >> 3;
    const int per_g = nT * K;
    t = (j % per_g) / K;
    tn = (j / per_g) * 8 + x;
    k = j % K;
    return;
  }
#ifndef MGP_K5_GROUP
#define MGP_K5_GROUP 4
#endif
  // MGP_K5_GROUP = G > 0 (the default, 4): per XCD, groups of G column tiles, row tiles in
  // the middle (group outer, then t, then the group's tiles x experts), so that a group's A
  // slabs are re-read per row tile from L2 / MALL instead of re-streamed from HBM: K5 pair
  // 4.31 -> 3.71 GB fetched per launch, ELBO step 3.347-3.353 -> 3.322-3.332 ms, training
  // 14.52-14.58 -> 14.49-14.51 ms (profiles/r06zc_*, r06zd_*; G = 2 slower, 8 between).
  // Items are unchanged, so the results are bit-identical; at c4's per-rank N (one group per
  // XCD) the order is the row-tile-outer one.
  if (MGP_K5_GROUP > 0 && nTn % 8 == 0 && (nTn / 8) % MGP_K5_GROUP == 0) {
    constexpr int G = MGP_K5_GROUP > 0 ? MGP_K5_GROUP : 1;
    const int nT = (grid < 0 ? (int)gridDim.x : grid) / (nTn * K);
    const int x = b & 7, j = b >> 3;
    const int g = j / (nT * G * K);
    t = (j / (G * K)) % nT;
    const int i = (j / K) % G;
    k = j % K;
    tn = (g * G + i) * 8 + x;
    return;
  }
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
}

// Item b -> (row tile t, column tile tn) for the one-matrix products (K4,
// gA, gKuf): the nT row tiles of a column tile are adjacent block ids on one
// XCD (b % 8), heaviest first, so the column slab of the B image they all read
// is served from that XCD's L2.
__device__ __forceinline__ void col_major_item(int b, int nT, int nTn, int& t, int& tn) {
  if (nTn % 8 == 0) {
    const int x = b & 7, j = b >> 3;
    t = nT - 1 - j % nT;
    tn = (j / nT) * 8 + x;
  } else {
    t = nT - 1 - b % nT;
    tn = b / nT;
  }
}

// Main loop shared by K4 and K5: acc[i][c] (row sub-tile i = 0..3 of the
// 128-row tile, column sub-tile c = 0..1 of this wave's 64 columns) +=
// sum over k-steps mk in [mk_begin, mk_end) (even count) of T-image blocks
// (4 t + i, mk) x B-image blocks (nb0 + c, mk).  T fragments are staged in LDS
// (shared by the 4 waves), B fragments go global -> registers one k-step ahead.
//   tbase: byte offset of T block (mb = 4 t, mk = 0) of this matrix
//   sB0:   byte offset of B block (nb0, mk = 0)
template <int V>
using ic = std::integral_constant<int, V>;

// DIAG_FIRST (K5, T lower: block (mb, mk) zero for 16 mk + 15 < 32 mb): the
// first 8 k-steps meet the diagonal and only sub-tiles i <= p of k-step pair p
// are non-zero.  Otherwise (K4, T upper: zero for 16 mk > 32 mb + 31) the last
// 8 k-steps do, with sub-tiles i >= p of pair p.  Those MFMAs are skipped
// (8% of the work), everything else is unchanged.
// DIAG: 1 = diagonal first (lower T), 2 = diagonal last (upper T), 0 = full T.
// NC: column sub-tiles (32 wide) per wave (B blocks nb0 .. nb0 + NC - 1).
// NPL: planes used (3 = x6 products; 2, 1 = K5's reduced modes, mfma_planes):
// only those planes are loaded and staged.
// F16: the images are split-f16 (mfma_fmt), NPL must be 2.
// X8 (with F16): image planes 0 (f16 hi) and 2 (e4m3 cross terms) are loaded;
// per k-step pair, two f16 hi products and one e4m3 MFMA for both pairs of
// cross terms (mfma_f8x): 2 + 2 f16-product-equivalents instead of 6.
// HOIST: all T fragment reads of a k-step issued before its MFMAs (trsm_bwd: 457 ->
// 438 us; K4 +2.5 %, K5 unchanged -- so only there).
// BH: called as bh(b, mk) on k-step mk's B fragments right before their MFMAs
// (trsm_bwd16_kernel's per-column rescale of the gA image); NoBHook: nothing.
struct NoBHook {
  template <class B>
  __device__ __forceinline__ void operator()(B&, int) const {}
};
template <int DIAG, int NC = 2, int NPL = 3, bool F16 = false, bool X8 = false, bool HOIST = false,
          typename BH = NoBHook>
__device__ __forceinline__ void x6_mainloop(floatx16 (&acc)[4][NC], bf16x8 (*sL)[4 * 3 * 64],
                                            __amdgpu_buffer_rsrc_t rT, uint32_t tbase,
                                            __amdgpu_buffer_rsrc_t rB, uint32_t sB0, int mk_begin,
                                            int mk_end, int nmk, bool init = true, BH bhook = BH{}) {
  static_assert(!X8 || (F16 && NPL == 2), "X8 reads split-f16 images");
  auto PL = [](int p) { return (X8 && p == 1) ? 2 : p; };  // LDS / register plane -> image plane
  const int tid = threadIdx.x, lane = tid & 63;
  const uint32_t vB = 16u * lane;
  const uint32_t sBc = (uint32_t)nmk * 3u * kFragBytes;  // B block nb0 + c at sB0 + c sBc
  // T stage: 256 NPL 16-B units per k-step, NPL per thread: unit e = tid + 256 s ->
  //   row sub-tile i = e / (64 NPL), plane p = (e / 64) % NPL, lane e % 64
  //   byte offset tbase + ((i * nmk + mk) * 192 + p * 64 + lane) * 16; LDS unit (3 i + p) * 64 + lane
  uint32_t vT[NPL];
  int dT[NPL];
#pragma unroll
  for (int s = 0; s < NPL; ++s) {
    const int e = tid + 256 * s, i = e / (64 * NPL), p = (e / 64) % NPL;
    vT[s] = (uint32_t)((i * nmk * 192 + PL(p) * 64 + (e & 63)) * 16);
    dT[s] = (3 * i + p) * 64 + (e & 63);
  }
  if (init) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int c = 0; c < NC; ++c)
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[i][c][e] = 0.f;
  }

  auto load_b = [&](bf16x8 (&b)[NC][3], int mk) {
    const uint32_t o = (uint32_t)mk * 3u * kFragBytes;
#pragma unroll
    for (int p = 0; p < NPL; ++p)
#pragma unroll
      for (int c = 0; c < NC; ++c) b[c][p] = ld_frag(rB, vB, sB0 + c * sBc + o + PL(p) * kFragBytes);
  };
  auto load_t = [&](u32x4v (&st)[NPL], int mk) {
    const uint32_t o = tbase + (uint32_t)mk * 192u * 16u;
#pragma unroll
    for (int s = 0; s < NPL; ++s) st[s] = __builtin_amdgcn_raw_buffer_load_b128(rT, vT[s], o, 0);
  };
  auto store_t = [&](int buf, const u32x4v (&st)[NPL]) {
#pragma unroll
    for (int s = 0; s < NPL; ++s) reinterpret_cast<u32x4v*>(sL[buf])[dT[s]] = st[s];
  };
  auto compute = [&](int buf, const bf16x8 (&b)[NC][3], auto ilo, auto ihi) {
    constexpr int ILO = decltype(ilo)::value, IHI = decltype(ihi)::value;
    if constexpr (HOIST) {  // every T fragment read of the k-step before its first MFMA
    bf16x8 a[4][3];
#pragma unroll
    for (int i = ILO; i < IHI; ++i)
#pragma unroll
      for (int p = 0; p < NPL; ++p) a[i][p] = sL[buf][(i * 3 + p) * 64 + lane];
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int i = ILO; i < IHI; ++i)
#pragma unroll
      for (int c = 0; c < NC; ++c) acc[i][c] = mfma_fmt<NPL, F16>(a[i], b[c], acc[i][c]);
    } else {
#pragma unroll
    for (int i = ILO; i < IHI; ++i) {
      bf16x8 a[3];
#pragma unroll
      for (int p = 0; p < NPL; ++p) a[p] = sL[buf][(i * 3 + p) * 64 + lane];
#pragma unroll
      for (int c = 0; c < NC; ++c) acc[i][c] = mfma_fmt<NPL, F16>(a, b[c], acc[i][c]);
    }
    }
  };

  // X8: the first k-step of a pair keeps its cross-term fragments for the second
  bf16x8 ax_s[4], bx_s[NC];
  auto compute_x8 = [&](int buf, const bf16x8 (&b)[NC][3], auto ilo, auto ihi, auto second) {
    constexpr int ILO = decltype(ilo)::value, IHI = decltype(ihi)::value;
    constexpr bool SECOND = decltype(second)::value;
#pragma unroll
    for (int i = ILO; i < IHI; ++i) {
      const bf16x8 a_hi = sL[buf][(i * 3) * 64 + lane], a_x = sL[buf][(i * 3 + 1) * 64 + lane];
#pragma unroll
      for (int c = 0; c < NC; ++c) {
        if constexpr (SECOND) acc[i][c] = mfma_f8x(ax_s[i], a_x, bx_s[c], b[c][1], acc[i][c]);
        acc[i][c] = mfma_f16(a_hi, b[c][0], acc[i][c]);
      }
      if constexpr (!SECOND) ax_s[i] = a_x;
    }
    if constexpr (!SECOND) {
#pragma unroll
      for (int c = 0; c < NC; ++c) bx_s[c] = b[c][1];
    }
  };

  bf16x8 b0[NC][3], b1[NC][3];
  u32x4v st[NPL];
  load_t(st, mk_begin);
  load_b(b0, mk_begin);
  store_t(0, st);
  __syncthreads();
  // two k-steps per iteration: LDS buffers and fragment sets alternate
  // one pair of k-steps (mk, mk + 1) on sub-tiles [ilo, ihi); sched_barrier(0)
  // pins the prefetch loads ahead of the MFMA block
  auto pair = [&](int mk, auto ilo, auto ihi) {
    load_t(st, mk + 1);
    load_b(b1, mk + 1);
    __builtin_amdgcn_sched_barrier(0);
    bhook(b0, mk);
    if constexpr (X8)
      compute_x8(0, b0, ilo, ihi, std::false_type{});
    else
      compute(0, b0, ilo, ihi);
    __builtin_amdgcn_sched_barrier(0);
    store_t(1, st);
    __syncthreads();
    const int m2 = mk + 2 < nmk ? mk + 2 : nmk - 1;  // after the last pair: harmless reload
    load_t(st, m2);
    load_b(b0, m2);
    __builtin_amdgcn_sched_barrier(0);
    bhook(b1, mk + 1);
    if constexpr (X8)
      compute_x8(1, b1, ilo, ihi, std::true_type{});
    else
      compute(1, b1, ilo, ihi);
    __builtin_amdgcn_sched_barrier(0);
    store_t(0, st);
    __syncthreads();
  };
  if constexpr (DIAG == 1) {
    pair(mk_begin, ic<0>{}, ic<1>{});
    pair(mk_begin + 2, ic<0>{}, ic<2>{});
    pair(mk_begin + 4, ic<0>{}, ic<3>{});
    pair(mk_begin + 6, ic<0>{}, ic<4>{});
#pragma nounroll
    for (int mk = mk_begin + 8; mk < mk_end; mk += 2) pair(mk, ic<0>{}, ic<4>{});
  } else if constexpr (DIAG == 0) {
#pragma nounroll
    for (int mk = mk_begin; mk < mk_end; mk += 2) pair(mk, ic<0>{}, ic<4>{});
  } else {
#pragma nounroll
    for (int mk = mk_begin; mk < mk_end - 8; mk += 2) pair(mk, ic<0>{}, ic<4>{});
    pair(mk_end - 8, ic<0>{}, ic<4>{});
    pair(mk_end - 6, ic<1>{}, ic<4>{});
    pair(mk_end - 4, ic<2>{}, ic<4>{});
    pair(mk_end - 2, ic<3>{}, ic<4>{});
  }
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t img_rsrc(const void* p, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc((void*)p, (short)0, (int)bytes, 0x00020000);
}

// ------------------------------------------------------------------ K5 (x6)
// F16: split-f16 images (NPL = 2) scaled by 2^img_exp(*a_bound), 2^img_exp(*l_bound).
// X8: their hi planes on f16 MFMA and cross terms on e4m3 MFMA (mfma_f8x).
template <int NPL, bool F16 = false, bool X8 = false>
__global__ __launch_bounds__(256, 2) void expert_cond_x6_kernel(const bf16x8* __restrict__ Afr,
                                                                const bf16x8* __restrict__ Lfr,
                                                                uint32_t afr_bytes, uint32_t lfr_bytes,
                                                                int nmk, int nmb, int nTn, int K,
                                                                int64_t N, float* __restrict__ part,
                                                                int64_t ldp, const float* __restrict__ a_bound,
                                                                const float* __restrict__ l_bound) {
  __shared__ bf16x8 sL[2][4 * 3 * 64];  // 2 x 12 KiB: [row sub-tile][plane][lane]
  int t, tn, k;
  x6_item(blockIdx.x, nTn, K, t, tn, k);
  const int nTp = nmb / 4;
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  floatx16 acc[4][2];
  x6_mainloop<1, 2, NPL, F16, X8>(acc, sL, img_rsrc(Lfr, lfr_bytes), (uint32_t)(((int64_t)k * nmb + 4 * t) * nmk) * 3u * kFragBytes,
              img_rsrc(Afr, afr_bytes), (uint32_t)((8 * tn + 2 * w) * nmk) * 3u * kFragBytes, 8 * t, nmk, nmk);

  // sum over the 128 rows of C^2 per column: 4 sub-tiles x 16 registers, then the lane halves
  const int64_t nbase = (int64_t)tn * kX6BN + 64 * w + (lane & 31);
  float* dst = part + ((int64_t)k * nTp + t) * ldp;
  float unscale = 1.f;
  if constexpr (F16) unscale = ldexpf(1.f, -2 * (img_exp(*a_bound) + img_exp(*l_bound)));
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int e = 0; e < 16; ++e) s = fmaf(acc[i][c][e], acc[i][c][e], s);
    s += __shfl_xor(s, 32, 64);
    if constexpr (F16) s *= unscale;
    const int64_t n = nbase + 32 * c;
    if (lane < 32 && n < N) dst[n] = s;
  }
}

// ------------------------------------------------------------------ K5 (split-f16) on 16x16x32 MFMAs
// The same contraction, items and split-f16 images as expert_cond_x6_kernel<2, true>,
// on v_mfma_f32_16x16x32_f16 (16 cycles per 16x16x32 block: the same cycles per flop
// as 32x32x16; the chip can hold a different clock per shape under load,
// MI355X_MICROARCH.md, DVFS give-back item 7).  No new image format: one k-step PAIR
// (32 deep) of the existing fragments is one MFMA k-step; lane l (i = l % 16,
// q = l / 16) takes the 16 bytes of fragment k-step 2 ks + q / 2 at lane position
// 16 (row block % 2) + i + 32 (q % 2) -- its 8 elements are 8 of the 32 m of the pair,
// the same 8 for the A operand (L_k^T, rows m') and the B operand (A, columns n), so
// the contraction is unchanged.  Wave w: 128 rows x 64 columns = 8 x 4 blocks of
// 16 x 16; per pair the L fragments of the item's 4 row sub-tiles (16 KiB) are staged
// in LDS (double buffered, one barrier per pair), the wave's B fragments go global ->
// registers one pair ahead; 96 MFMAs per wave and pair.
typedef float floatx4v __attribute__((ext_vector_type(4)));
typedef _Float16 halfx2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ floatx4v mfma16_f16(bf16x8 a, bf16x8 b, floatx4v c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(halfx8, a), __builtin_bit_cast(halfx8, b), c,
                                                0, 0, 0);
}
__device__ __forceinline__ floatx4v mfma16_bf16(bf16x8 a, bf16x8 b, floatx4v c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
// one 16x16 block: the plane products of mfma_fmt (x6: six bf16, split-f16: three f16)
template <int NPL, bool F16>
__device__ __forceinline__ floatx4v mfma16_fmt(const bf16x8 (&a)[3], const bf16x8 (&b)[3], floatx4v acc) {
  if constexpr (F16) {
    acc = mfma16_f16(a[1], b[0], acc);
    acc = mfma16_f16(a[0], b[1], acc);
    return mfma16_f16(a[0], b[0], acc);
  } else if constexpr (NPL == 3) {
    acc = mfma16_bf16(a[2], b[0], acc);
    acc = mfma16_bf16(a[1], b[1], acc);
    acc = mfma16_bf16(a[0], b[2], acc);
    acc = mfma16_bf16(a[1], b[0], acc);
    acc = mfma16_bf16(a[0], b[1], acc);
    return mfma16_bf16(a[0], b[0], acc);
  } else if constexpr (NPL == 2) {
    acc = mfma16_bf16(a[1], b[0], acc);
    acc = mfma16_bf16(a[0], b[1], acc);
    return mfma16_bf16(a[0], b[0], acc);
  } else {
    return mfma16_bf16(a[0], b[0], acc);
  }
}

// Main loop of the 16x16x32 kernels: acc[ib][cb] (16-row block ib = 0..7 of the 128-row
// item, 16-column block cb = 0..3 of this wave's 64 columns) += sum over k-step PAIRS
// ks in [ks_begin, ks_end) (even count) of T-image rows x B-image columns.  T fragments
// of the item's 4 row sub-tiles, both k-steps of a pair and NPL planes are staged in LDS
// (double buffered, one barrier per pair); B fragments go global -> registers one pair
// ahead.  DIAG = 1: T lower (K5): the first 4 pairs meet the diagonal, pair p has row
// blocks ib <= 2 p + 1; DIAG = 2: T upper (K4): the last 4 pairs do, pair p of them has
// ib >= 2 p; 0: full.  (The zero sub-blocks inside come from the images' zero fill.)
//   tbase: byte offset of T fragment (mb = 4 t, mk = 0); sB0: of B fragment (nb0, mk = 0)
template <int DIAG, int NPL, bool F16>
__device__ __forceinline__ void x6_mainloop16(floatx4v (&acc)[8][4], bf16x8 (*sL)[4 * 2 * 3 * 64],
                                              __amdgpu_buffer_rsrc_t rT, uint32_t tbase, __amdgpu_buffer_rsrc_t rB,
                                              uint32_t sB0, int ks_begin, int ks_end, int nmk) {
  const int tid = threadIdx.x, lane = tid & 63, li = lane & 15, q = lane >> 4;
  // T staging: unit e = tid + 256 s (NPL 2: 4 units, 3: 6 units per thread): sub-tile
  // i = e / (128 NPL), k-step kk = (e / (64 NPL)) % 2, plane p = (e / 64) % NPL, position e % 64
  constexpr int NU = 2 * NPL;
  uint32_t vT[NU];
#pragma unroll
  for (int s = 0; s < NU; ++s) {
    const int e = tid + 256 * s, i = e / (128 * NPL), kk = (e / (64 * NPL)) % 2, p = (e / 64) % NPL;
    vT[s] = (uint32_t)((((i * nmk + kk) * 3 + p) * 64 + (e & 63)) * 16);
  }
  // B: column block cb, plane p, pair ks: fragment nb0 + cb / 2, k-step 2 ks + q / 2,
  // position 16 (cb % 2) + li + 32 (q % 2)
  const uint32_t vB = (uint32_t)((((q >> 1) * 3) * 64 + li + 32 * (q & 1)) * 16);
  auto boff = [&](int cb, int p, int ks) {
    return sB0 + (uint32_t)(cb >> 1) * (uint32_t)nmk * 3u * kFragBytes + (uint32_t)((2 * ks) * 3 + p) * kFragBytes +
           (uint32_t)(16 * (cb & 1)) * 16u;
  };
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int c = 0; c < 4; ++c) acc[i][c] = floatx4v{0.f, 0.f, 0.f, 0.f};
  auto load_b = [&](bf16x8 (&b)[4][3], int ks) {
#pragma unroll
    for (int cb = 0; cb < 4; ++cb)
#pragma unroll
      for (int p = 0; p < NPL; ++p) b[cb][p] = ld_frag(rB, vB, boff(cb, p, ks));
  };
  auto load_t = [&](u32x4v (&st)[NU], int ks) {
    const uint32_t o = tbase + (uint32_t)(2 * ks) * 3u * kFragBytes;
#pragma unroll
    for (int s = 0; s < NU; ++s) st[s] = __builtin_amdgcn_raw_buffer_load_b128(rT, vT[s], o, 0);
  };
  auto store_t = [&](int buf, const u32x4v (&st)[NU]) {
#pragma unroll
    for (int s = 0; s < NU; ++s) reinterpret_cast<u32x4v*>(sL[buf])[tid + 256 * s] = st[s];
  };
  // A operand of row block ib, plane p: sub-tile ib / 2, k-step q / 2, position 16 (ib % 2) + li + 32 (q % 2)
  const int aoff = (q >> 1) * 64 * NPL + li + 32 * (q & 1);
  auto compute = [&](int buf, const bf16x8 (&b)[4][3], auto ilo, auto ihi) {
    constexpr int ILO = decltype(ilo)::value, IHI = decltype(ihi)::value;
#pragma unroll
    for (int ib = ILO; ib < IHI; ++ib) {
      const int base = (ib >> 1) * 128 * NPL + 16 * (ib & 1) + aoff;
      bf16x8 a[3];
#pragma unroll
      for (int p = 0; p < NPL; ++p) a[p] = sL[buf][base + 64 * p];
#pragma unroll
      for (int cb = 0; cb < 4; ++cb) acc[ib][cb] = mfma16_fmt<NPL, F16>(a, b[cb], acc[ib][cb]);
    }
  };
  bf16x8 b0[4][3], b1[4][3];
  u32x4v st[NU];
  load_t(st, ks_begin);
  load_b(b0, ks_begin);
  store_t(0, st);
  __syncthreads();
  auto two = [&](int ks, auto ilo0, auto ihi0, auto ilo1, auto ihi1) {
    load_t(st, ks + 1);
    load_b(b1, ks + 1);
    __builtin_amdgcn_sched_barrier(0);
    compute(0, b0, ilo0, ihi0);
    __builtin_amdgcn_sched_barrier(0);
    store_t(1, st);
    __syncthreads();
    const int k2 = ks + 2 < ks_end ? ks + 2 : ks_end - 1;  // after the last pair: harmless reload
    load_t(st, k2);
    load_b(b0, k2);
    __builtin_amdgcn_sched_barrier(0);
    compute(1, b1, ilo1, ihi1);
    __builtin_amdgcn_sched_barrier(0);
    store_t(0, st);
    __syncthreads();
  };
  if constexpr (DIAG == 1) {
    two(ks_begin, ic<0>{}, ic<2>{}, ic<0>{}, ic<4>{});
    two(ks_begin + 2, ic<0>{}, ic<6>{}, ic<0>{}, ic<8>{});
#pragma nounroll
    for (int ks = ks_begin + 4; ks < ks_end; ks += 2) two(ks, ic<0>{}, ic<8>{}, ic<0>{}, ic<8>{});
  } else if constexpr (DIAG == 0) {
#pragma nounroll
    for (int ks = ks_begin; ks < ks_end; ks += 2) two(ks, ic<0>{}, ic<8>{}, ic<0>{}, ic<8>{});
  } else {
#pragma nounroll
    for (int ks = ks_begin; ks < ks_end - 4; ks += 2) two(ks, ic<0>{}, ic<8>{}, ic<0>{}, ic<8>{});
    two(ks_end - 4, ic<0>{}, ic<8>{}, ic<2>{}, ic<8>{});
    two(ks_end - 2, ic<4>{}, ic<8>{}, ic<6>{}, ic<8>{});
  }
}

// ------------------------------------------------------------------ K5 (split-f16) on 16x16x32 MFMAs
// The same contraction, items and split-f16 images as expert_cond_x6_kernel<2, true>,
// on v_mfma_f32_16x16x32_f16 (16 cycles per 16x16x32 block: the same cycles per flop
// as 32x32x16; the chip can hold a different clock per shape under load,
// MI355X_MICROARCH.md, DVFS give-back item 7).  No new image format: one k-step PAIR
// (32 deep) of the existing fragments is one MFMA k-step; lane l (i = l % 16,
// q = l / 16) takes the 16 bytes of fragment k-step 2 ks + q / 2 at lane position
// 16 (row block % 2) + i + 32 (q % 2) -- its 8 elements are 8 of the 32 m of the pair,
// the same 8 for the A operand (L_k^T, rows m') and the B operand (A, columns n), so
// the contraction is unchanged (x6_mainloop16).  Wave w: 128 rows x 64 columns =
// 8 x 4 blocks of 16 x 16; 96 MFMAs per wave and pair.
// COUT (training): C_k = L_k^T A is also written as a split-f16 B-layout image per expert,
// (the B-layout of the images K4 writes); a fragment's lane position takes
// 8 rows from two lanes of the 16x16 accumulator layout (one exchange across the lane halves).
// One item (workgroup index b of a launch of `grid` items) of the split-f16 K5.
// C_k images (training) with non-temporal stores (MGP_C_NT)
#ifndef MGP_C_NT
#define MGP_C_NT 1
#endif
constexpr bool kCntStores = MGP_C_NT;
// C-writing K5 (training) in the column-tile-outer item order (x6_item TN_OUTER): measured
// against the forward's row-tile-outer order on the 16x16x32 kernel, training step 14.18-14.22
// vs 14.11-14.18 ms (profiles/r06o_train_ab.log) -- so the row-tile-outer order (0) is kept
#ifndef MGP_K5C_TN_OUTER
#define MGP_K5C_TN_OUTER 0
#endif
constexpr bool kK5cTnOuter = MGP_K5C_TN_OUTER;
#ifndef MGP_K5_TN_OUTER
#define MGP_K5_TN_OUTER 0   // the forward K5's item order (0: row tile outer)
#endif
constexpr bool kK5TnOuter = MGP_K5_TN_OUTER;
template <bool COUT>
__device__ __forceinline__ void expert_cond16_item(bf16x8 (*sL)[4 * 2 * 3 * 64], int b, int grid,
                                                   const bf16x8* __restrict__ Afr, const bf16x8* __restrict__ Lfr,
                                                   uint32_t afr_bytes, uint32_t lfr_bytes, int nmk, int nmb, int nTn,
                                                   int K, int64_t N, float* __restrict__ part, int64_t ldp,
                                                   const float* __restrict__ a_bound,
                                                   const float* __restrict__ l_bound, bf16x8* __restrict__ Cfr,
                                                   int64_t cexp, const float* __restrict__ colmax) {
  int t, tn, k;
  x6_item<COUT ? kK5cTnOuter : kK5TnOuter>(b, nTn, K, t, tn, k, grid);
  const int nTp = nmb / 4;
  const int lane = threadIdx.x & 63, li = lane & 15, q = lane >> 4;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  floatx4v acc[8][4];
  x6_mainloop16<1, 2, true>(acc, sL, img_rsrc(Lfr, lfr_bytes), (uint32_t)(((int64_t)k * nmb + 4 * t) * nmk) * 3u * kFragBytes,
                            img_rsrc(Afr, afr_bytes), (uint32_t)((8 * tn + 2 * w) * nmk) * 3u * kFragBytes, 4 * t,
                            nmk / 2, nmk);
  if constexpr (COUT) {
    const float cmul = ldexpf(1.f, img_exp(*colmax * *a_bound * 1.0009765625f) -
                                       (img_exp(*a_bound) + img_exp(*l_bound)));
    bf16x8* Ck = Cfr + (int64_t)k * cexp;
    const bool lo_half = lane < 32;
    const int pos = lo_half ? li + 32 * q : 16 + li + 32 * (q - 2);
#pragma unroll
    for (int ib = 0; ib < 8; ++ib)
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        float v[8];
#pragma unroll
        for (int r = 0; r < 4; ++r) {  // lanes 0-31: (own 2c, lane + 32's 2c); 32-63: (lane - 32's 2c + 1, own)
          float x0 = acc[ib][2 * c][r], x1 = acc[ib][2 * c + 1][r];
          lane_half_swap(x0, x1);
          v[r] = x0 * cmul;
          v[4 + r] = x1 * cmul;
        }
        bf16x8* dst = Ck + ((((int64_t)8 * tn + 2 * w + c) * nmk + 8 * t + ib) * 3) * 64 + pos;
        if constexpr (kCntStores) {  // read back only by the backward, long after: past L2
          halfx8 h, l;
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const _Float16 hi = (_Float16)v[j];
            h[j] = hi;
            l[j] = (_Float16)(v[j] - (float)hi);
          }
          __builtin_nontemporal_store(__builtin_bit_cast(bf16x8, h), dst);
          __builtin_nontemporal_store(__builtin_bit_cast(bf16x8, l), dst + 64);
        } else {
          store_split_f16(dst, v, 1.f);
        }
      }
  }
  // sum over the 128 rows of C^2 per column: 8 blocks x 4 registers, then the 4 lane groups
  const float unscale = ldexpf(1.f, -2 * (img_exp(*a_bound) + img_exp(*l_bound)));
  float* dst = part + ((int64_t)k * nTp + t) * ldp;
#pragma unroll
  for (int cb = 0; cb < 4; ++cb) {
    float s = 0.f;
#pragma unroll
    for (int ib = 0; ib < 8; ++ib)
#pragma unroll
      for (int r = 0; r < 4; ++r) s = fmaf(acc[ib][cb][r], acc[ib][cb][r], s);
    s += lane_xor16(s);
    s += lane_xor32(s);
    const int64_t n = (int64_t)tn * kX6BN + 64 * w + 16 * cb + li;
    if (lane < 16 && n < N) dst[n] = s * unscale;
  }
}

template <bool COUT = false>
__global__ __launch_bounds__(256, 2) void expert_cond16_kernel(const bf16x8* __restrict__ Afr,
                                                               const bf16x8* __restrict__ Lfr, uint32_t afr_bytes,
                                                               uint32_t lfr_bytes, int nmk, int nmb, int nTn, int K,
                                                               int64_t N, float* __restrict__ part, int64_t ldp,
                                                               const float* __restrict__ a_bound,
                                                               const float* __restrict__ l_bound,
                                                               bf16x8* __restrict__ Cfr = nullptr, int64_t cexp = 0,
                                                               const float* __restrict__ colmax = nullptr) {
  __shared__ bf16x8 sL[2][4 * 2 * 3 * 64];  // [row sub-tile][k-step of pair][plane][lane position] (2 planes used)
  expert_cond16_item<COUT>(sL, blockIdx.x, gridDim.x, Afr, Lfr, afr_bytes, lfr_bytes, nmk, nmb, nTn, K, N, part, ldp,
                           a_bound, l_bound, Cfr, cexp, colmax);
}

// One layer's operands of the batched K5.
struct K5Layer {
  const bf16x8* Afr;
  const bf16x8* Lfr;
  float* part;
  const float* a_bound;
  const float* l_bound;
  bf16x8* Cfr;
  const float* colmax;
};

// expert_cond16_kernel over two layers in one launch: workgroups [0, per) run layer 0's
// items, [per, 2 per) layer 1's (same items, same arithmetic: bit-identical partials
// and C_k images); one kernel tail fewer between the layers.
template <bool COUT>
__global__ __launch_bounds__(256, 2) void expert_cond16_pair_kernel(K5Layer l0, K5Layer l1, int per,
                                                                    uint32_t afr_bytes, uint32_t lfr_bytes, int nmk,
                                                                    int nmb, int nTn, int K, int64_t N, int64_t ldp,
                                                                    int64_t cexp) {
  __shared__ bf16x8 sL[2][4 * 2 * 3 * 64];
  const bool second = (int)blockIdx.x >= per;
  const K5Layer& l = second ? l1 : l0;
  expert_cond16_item<COUT>(sL, (int)blockIdx.x - (second ? per : 0), per, l.Afr, l.Lfr, afr_bytes, lfr_bytes, nmk,
                           nmb, nTn, K, N, l.part, ldp, l.a_bound, l.l_bound, l.Cfr, cexp, l.colmax);
}

// ------------------------------------------------------------------ backward (x6)
// Store a 128 x 256 item's accumulators (wave w: 128 rows x 64 columns) as f32
// rows [i0 + .][n0 + .] of out (M rows, leading dimension ld), each column n
// scaled by colscale[n] (if given).  Buffer stores with 32-bit offsets: rows
// beyond M fall outside the resource and are dropped.
__device__ __forceinline__ void store_acc_f32(const floatx16 (&acc)[4][2], float* __restrict__ out, int64_t ld,
                                              int64_t i0, int64_t n0, int64_t M, int64_t N,
                                              const float* __restrict__ colscale) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const __amdgpu_buffer_rsrc_t r =
      __builtin_amdgcn_make_buffer_rsrc((void*)out, (short)0, (int)(uint32_t)(M * ld * 4), 0x00020000);
  const uint32_t soff = (uint32_t)((i0 * ld + n0) * 4);
  const uint32_t ld32 = (uint32_t)ld;
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    const int nl = 64 * w + 32 * c + (lane & 31);
    const int64_t n = n0 + nl;
    if (n < N) {
      const float cs = colscale ? colscale[n] : 1.f;
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const uint32_t rl = (uint32_t)(32 * i + acc_row(e, lane));
          __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, acc[i][c][e] * cs), r,
                                                (rl * ld32 + (uint32_t)nl) * 4u, soff, 0);
        }
    }
  }
}

// Store the accumulators as the split image [nb][mk] of the item's 128 x 256
// block (as K4 does for A), columns scaled by colscale[n] (0 beyond N).
__device__ __forceinline__ void store_acc_image(const floatx16 (&acc)[4][2], bf16x8* __restrict__ img, int nmk,
                                                int t, int tn, int64_t N, const float* __restrict__ colscale) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    const int64_t nb = 8 * (int64_t)tn + 2 * w + c;
    const int64_t n = 32 * nb + (lane & 31);
    const float cs = colscale ? (n < N ? colscale[n] : 0.f) : 1.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int64_t mk = 8 * (int64_t)t + 2 * i;
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        float v[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = acc[i][c][8 * s + j] * cs;
        store_split(img + ((nb * nmk + mk + s) * 3) * 64 + lane, v);
      }
    }
  }
}

// gA0[m][n] = sum_k q_mu[m][k] G_mu[k][n] - 2 A[m][n] sum_k Gv[k][n]: the part
// of the A gradient that needs no GEMM (one thread per column n, looping rows).
template <int KMAX>
__global__ __launch_bounds__(256) void grad_a_base_kernel(const float* __restrict__ A, int64_t lda,
                                                          const float* __restrict__ q_mu, int64_t ldq,
                                                          const float* __restrict__ Gmu,
                                                          const float* __restrict__ Gv, int64_t ldg, int64_t M,
                                                          int64_t N, int K, int rows_per_block,
                                                          float* __restrict__ out, int64_t ldo) {
  __shared__ float sq[64][KMAX];
  const int64_t n = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t r0 = (int64_t)blockIdx.y * rows_per_block;
  float gmu[KMAX], gvs = 0.f;
#pragma unroll
  for (int k = 0; k < KMAX; ++k) {
    gmu[k] = (k < K && n < N) ? Gmu[(int64_t)k * ldg + n] : 0.f;
    if (k < K && n < N) gvs += Gv[(int64_t)k * ldg + n];
  }
  for (int64_t rb = r0; rb < r0 + rows_per_block && rb < M; rb += 64) {
    __syncthreads();
    for (int i = threadIdx.x; i < 64 * KMAX; i += 256) {
      const int rr = i / KMAX, k = i % KMAX;
      sq[rr][k] = (rb + rr < M && k < K) ? q_mu[(rb + rr) * ldq + k] : 0.f;
    }
    __syncthreads();
    if (n < N) {
      const int rows = (int)((M - rb) < 64 ? (M - rb) : 64);
      for (int rr = 0; rr < rows; ++rr) {
        float v = -2.f * A[(rb + rr) * lda + n] * gvs;
#pragma unroll
        for (int k = 0; k < KMAX; ++k) v = fmaf(sq[rr][k], gmu[k], v);
        out[(rb + rr) * ldo + n] = v;
      }
    }
  }
}

// Steps 2, 5 (A's row image) and 6 (g_q_mu) of the split-f16 conditional backward
// in ONE pass over A (three kernels read A before: grad_a_base, split_rows_f16,
// gram_narrow).  Workgroup: one slab of 8 k-steps (128 n) x kPrepRB 32-row blocks;
// G_mu and sum_k Gv over the slab's columns are staged in LDS once.  Per row block:
//   (1) coalesced: thread t takes rows t / 32 + 8 i (i < 4), columns 4 (t % 32) + e
//       of A (16-B loads, two 512-B rows per wave instruction) and writes
//       gA0[m][n] = sum_k q_mu[m][k] G_mu[k][n] - 2 A[m][n] sum_k Gv[k][n] the same
//       way, and puts the tile into LDS (pitch 132 floats: conflict-free reads below);
//   (2) fragments: lane (r, h) of wave w takes row r, k-steps w and w + 4
//       (n = 16 ns + 8 h + j), stores split_rows_f16(A)'s image (same layout and
//       scale 2^img_exp(*bound)) and sums A[m][n] G_mu[k][n] for g_q_mu:
//       part[slab][m][k] (f32 per slab; folded in float64 by prep_fold_kernel).
// The tile and the row sums are double-buffered: one barrier per row block.
// c3 (MI355X, rocprofv3): 205 us per layer against 126 + 90 + 111 + 12 us for
// grad_a_base, split_rows_f16, gram_narrow and its fold (profiles/r03_grad_a_prep_probe.log).
// Measured, not kept: the next row block's A loads issued before (2) (287 vs 248 us),
// 4 instead of 8 row blocks per workgroup (same).
constexpr int kPrepRB = 8, kPrepPitch = 132;
template <int KMAX>
__global__ __launch_bounds__(256) void grad_a_prep_kernel(const float* __restrict__ A, int64_t lda,
                                                          const float* __restrict__ q_mu, int64_t ldq,
                                                          const float* __restrict__ Gmu,
                                                          const float* __restrict__ Gv, int64_t ldg, int64_t M,
                                                          int64_t N, int K, int nns, const float* __restrict__ bound,
                                                          float* __restrict__ gA0, int64_t ldo,
                                                          bf16x8* __restrict__ img, float* __restrict__ part, int rbs, int qvec,
                                                          float* __restrict__ amax = nullptr) {
  __shared__ __attribute__((aligned(16))) float sg[KMAX + 1][128];  // G_mu rows, then sum_k Gv
  __shared__ __attribute__((aligned(16))) float sA[2][32][kPrepPitch];
  __shared__ float sp[2][4][32][KMAX];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, r = lane & 31, h = lane >> 5;
  const int64_t nsb = 8 * (int64_t)blockIdx.x, n0 = 16 * nsb;
  const int64_t rb0 = (int64_t)blockIdx.y * rbs;
  const int nblk = (int)((M + 31) / 32);
  const int nit = nblk - rb0 < rbs ? (int)(nblk - rb0) : rbs;
  for (int i = tid; i < (KMAX + 1) * 32; i += 256) {  // 4 columns per item
    const int k = i >> 5, c = 4 * (i & 31);
    const int64_t n = n0 + c;
    floatx4 v = {0.f, 0.f, 0.f, 0.f};
    if (k < KMAX) {
      if (k < K) {
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = n + e < N ? Gmu[(int64_t)k * ldg + n + e] : 0.f;
      }
    } else {
#pragma unroll
      for (int kk = 0; kk < KMAX; ++kk)
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] += (kk < K && n + e < N) ? Gv[(int64_t)kk * ldg + n + e] : 0.f;
    }
    *reinterpret_cast<floatx4*>(&sg[k][c]) = v;
  }
  __syncthreads();
  const float scale = ldexpf(1.f, img_exp(*bound));
  const int ct_r = tid >> 5, ct_c = 4 * (tid & 31);
  const int64_t nc = n0 + ct_c;
  const bool colvec = nc + 3 < N;
  floatx4 gmu4[KMAX];
#pragma unroll
  for (int k = 0; k < KMAX; ++k) gmu4[k] = *reinterpret_cast<const floatx4*>(&sg[k][ct_c]);
  const floatx4 gvs4 = *reinterpret_cast<const floatx4*>(&sg[KMAX][ct_c]);
  auto flush = [&](int it, int b) {
    for (int i = tid; i < 32 * KMAX; i += 256) {
      const int rr = i / KMAX, k = i % KMAX;
      const int64_t m = 32 * (rb0 + it) + rr;
      if (m < M && k < K)
        part[((int64_t)blockIdx.x * M + m) * K + k] = (sp[b][0][rr][k] + sp[b][1][rr][k]) + (sp[b][2][rr][k] + sp[b][3][rr][k]);
    }
  };
  auto load_rows = [&](floatx4 (&a)[4], int64_t rb) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int64_t row = 32 * rb + ct_r + 8 * i;
      a[i] = floatx4{0.f, 0.f, 0.f, 0.f};
      if (row < M) {
        if (colvec) {
          a[i] = *reinterpret_cast<const floatx4*>(A + row * lda + nc);
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e) a[i][e] = nc + e < N ? A[row * lda + nc + e] : 0.f;
        }
      }
    }
  };
  floatx4 a[4];
  for (int it = 0; it < nit; ++it) {
    const int64_t rb = rb0 + it;
    const int b = it & 1;
    load_rows(a, rb);
    if (amax) {  // max |A[m][.]| over this slab per row -> amax[slab][m] (rowmax_fold_kernel)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float m =
            half_max_f32(fmaxf(fmaxf(fabsf(a[i][0]), fabsf(a[i][1])), fmaxf(fabsf(a[i][2]), fabsf(a[i][3]))));
        const int64_t row = 32 * rb + ct_r + 8 * i;
        if ((tid & 31) == 0 && row < M) amax[(int64_t)blockIdx.x * M + row] = m;
      }
    }
    // (1) coalesced rows: gA0, the LDS tile
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int64_t row = 32 * rb + ct_r + 8 * i;
      if (row < M) {
        floatx4 g = -2.f * a[i] * gvs4;
        if (qvec) {  // q_mu's row in 16-B loads (ldq % 4 == 0, K a multiple of 4)
#pragma unroll
          for (int k4 = 0; k4 < KMAX / 4; ++k4) {
            if (4 * k4 < K) {
              const floatx4 q = *reinterpret_cast<const floatx4*>(q_mu + row * ldq + 4 * k4);
#pragma unroll
              for (int e = 0; e < 4; ++e) g += q[e] * gmu4[4 * k4 + e];
            }
          }
        } else {
#pragma unroll
          for (int k = 0; k < KMAX; ++k)
            if (k < K) g += q_mu[row * ldq + k] * gmu4[k];
        }
        float* dst = gA0 + row * ldo + nc;
        if (colvec) {
          *reinterpret_cast<floatx4*>(dst) = g;
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e)
            if (nc + e < N) dst[e] = g[e];
        }
      }
      *reinterpret_cast<floatx4*>(&sA[b][ct_r + 8 * i][ct_c]) = a[i];
    }
    __syncthreads();
    if (it > 0) flush(it - 1, b ^ 1);
    // (2) fragments: the image and the g_q_mu row sums
    float pf[KMAX];
#pragma unroll
    for (int k = 0; k < KMAX; ++k) pf[k] = 0.f;
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      const int st = w + 4 * s2;
      const int64_t ns = nsb + st;
      if (ns >= nns) continue;
      const int c = 16 * st + 8 * h;
      const floatx4 lo = *reinterpret_cast<const floatx4*>(&sA[b][r][c]);
      const floatx4 hi = *reinterpret_cast<const floatx4*>(&sA[b][r][c + 4]);
      float v[8];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        v[j] = lo[j];
        v[4 + j] = hi[j];
      }
      store_split_f16(img + (rb * nns + ns) * 128 + lane, v, scale);
#pragma unroll
      for (int k = 0; k < KMAX; ++k)
#pragma unroll
        for (int j = 0; j < 8; ++j) pf[k] = fmaf(v[j], sg[k][c + j], pf[k]);
    }
#pragma unroll
    for (int k = 0; k < KMAX; ++k) pf[k] += __shfl_xor(pf[k], 32, 64);
    if (h == 0) {
#pragma unroll
      for (int k = 0; k < KMAX; ++k) sp[b][w][r][k] = pf[k];
    }
  }
  __syncthreads();
  if (nit > 0) flush(nit - 1, (nit - 1) & 1);
}

// out[m][k] = sum over the slabs of part[slab][m][k] in float64, fixed order:
// 16 outputs per workgroup, thread (o, g) sums slabs g, g + 16, ... (four running
// sums, slab c into sum (c / 16) % 4), then the 16 groups in order.
__global__ __launch_bounds__(256) void prep_fold_kernel(const float* __restrict__ part, int slabs, int64_t M, int K,
                                                        float* __restrict__ out, int64_t ldo) {
  __shared__ double sred[16][17];
  const int o = threadIdx.x & 15, g = threadIdx.x >> 4;
  const int64_t MK = M * K, idx = (int64_t)blockIdx.x * 16 + o;
  double v = 0.0;
  if (idx < MK) {
    double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0;
    int c = g;
    for (; c + 48 < slabs; c += 64) {
      a0 += (double)part[(int64_t)c * MK + idx];
      a1 += (double)part[(int64_t)(c + 16) * MK + idx];
      a2 += (double)part[(int64_t)(c + 32) * MK + idx];
      a3 += (double)part[(int64_t)(c + 48) * MK + idx];
    }
    for (int u = 0; c < slabs; c += 16, ++u) {
      const double x = (double)part[(int64_t)c * MK + idx];
      if (u == 0) a0 += x; else if (u == 1) a1 += x; else a2 += x;
    }
    v = (a0 + a1) + (a2 + a3);
  }
  sred[g][o] = v;
  __syncthreads();
  if (threadIdx.x < 16 && idx < MK) {
    double t = 0.0;
#pragma unroll
    for (int q = 0; q < 16; ++q) t += sred[q][o];
    out[(idx / K) * ldo + idx % K] = (float)t;
  }
}

// B-b: gA (image) = 2 sum_k (S_k A) diag(Gv_k) + gA0 with S_k = L_k L_k^T
// (full split images): item = (row tile t of 128 rows, column tile tn of
// 128), wave w owns the 32 columns of B block 4 tn + w.  Each expert's
// product runs through the K5 main loop (full T, one column sub-tile per
// wave) and is folded into the output registers with its column weights, so
// no per-expert intermediate is written.
// F16: Sfr and Afr are split-f16 images (scales 2^img_exp(*s_bound), 2^img_exp(*a_bound)):
// three f16 products per block; the unscale folds into the column weights.
// X8 (with F16): the S_k A products on f16 hi products + e4m3 cross terms
// (mfma_f8x; both images carry the e4m3 plane in the f16x8 training step).
template <bool F16 = false, bool X8 = false>
__global__ __launch_bounds__(256, 2) void grad_a_s_kernel(const bf16x8* __restrict__ Sfr, uint32_t s_bytes,
                                                          const bf16x8* __restrict__ Afr, uint32_t afr_bytes,
                                                          int nmk, int nTn, int K, int64_t M, int64_t N,
                                                          const float* __restrict__ Gv, int64_t ldg,
                                                          const float* __restrict__ gA0, int64_t ld0,
                                                          bf16x8* __restrict__ gAfr,
                                                          const float* __restrict__ s_bound = nullptr,
                                                          const float* __restrict__ a_bound = nullptr) {
  __shared__ bf16x8 sL[2][4 * 3 * 64];
  const int nT = nmk / 8, nmb = nmk / 2;
  int t, tn;
  col_major_item(blockIdx.x, nT, nTn, t, tn);
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t nb = 4 * (int64_t)tn + w;
  const int64_t n = 32 * nb + (lane & 31);
  floatx16 acc[4][1], out[4][1];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int e = 0; e < 16; ++e) out[i][0][e] = 0.f;
  const int64_t s_elems = (int64_t)nmb * nmk * 3 * 64;  // one expert's S image (bf16x8 units)
  float unscale = 1.f;
  if constexpr (F16) unscale = ldexpf(1.f, -(img_exp(*s_bound) + img_exp(*a_bound)));
  for (int k = 0; k < K; ++k) {
    x6_mainloop<0, 1, F16 ? 2 : 3, F16, X8>(acc, sL, img_rsrc(Sfr + k * s_elems, s_bytes),
                                        (uint32_t)(4 * t * nmk) * 3u * kFragBytes, img_rsrc(Afr, afr_bytes),
                                        (uint32_t)(nb * nmk) * 3u * kFragBytes, 0, nmk, nmk);
    const float g = n < N ? Gv[(int64_t)k * ldg + n] * unscale : 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int e = 0; e < 16; ++e) out[i][0][e] = fmaf(g, acc[i][0][e], out[i][0][e]);
  }
  const int64_t i0 = 128 * (int64_t)t;
  const __amdgpu_buffer_rsrc_t r0 =
      __builtin_amdgcn_make_buffer_rsrc((void*)gA0, (short)0, (int)(uint32_t)(M * ld0 * 4), 0x00020000);
  const uint32_t soff = (uint32_t)((i0 * ld0 + 128 * (int64_t)tn) * 4), ld32 = (uint32_t)ld0;
  const int nl = 32 * w + (lane & 31);
  const bool ok = n < N;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    float v[16];
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const uint32_t rl = (uint32_t)(32 * i + acc_row(e, lane));
      const float b0 = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r0, (rl * ld32 + (uint32_t)nl) * 4u, soff, 0));
      v[e] = ok ? fmaf(2.f, out[i][0][e], b0) : 0.f;   // rows >= M read 0 (outside the resource)
    }
    const int64_t mk = 8 * (int64_t)t + 2 * i;
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      float u[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) u[j] = v[8 * s2 + j];
      store_split(gAfr + ((nb * nmk + mk + s2) * 3) * 64 + lane, u);
    }
  }
}

// B-b on split-f16 images (grad_a_s_kernel<true> restated for LDS economy):
// gA = 2 sum_k (S_k A) diag(Gv_k) + gA0.  Item = (row tile t of 128, column tile
// tn of 128) as grad_a_s_kernel, but each wave owns a 64 x 64 quarter (row half
// wr = w / 2, column half wc = w % 2: 2 sub-tiles x 2 column blocks), so a T
// fragment read from LDS feeds two column blocks, and two experts run per pass
// of the main loop, sharing every B fragment (A's image).  Per wave and k-step:
// 8 LDS reads, 4 B loads, 24 MFMAs (grad_a_s_kernel: 8 LDS reads and 2 B loads
// per 12) -- half the LDS bytes per MFMA, which bound that kernel.  Odd K: the
// last pass pairs the last expert with itself at weight 0.
__global__ __launch_bounds__(256, 2) void grad_a_s_f16_kernel(const bf16x8* __restrict__ Sfr, uint32_t s_bytes,
                                                             const bf16x8* __restrict__ Afr, uint32_t afr_bytes,
                                                             int nmk, int nTn, int K, int64_t M, int64_t N,
                                                             const float* __restrict__ Gv, int64_t ldg,
                                                             const float* __restrict__ gA0, int64_t ld0,
                                                             bf16x8* __restrict__ gAfr,
                                                             const float* __restrict__ s_bound,
                                                             const float* __restrict__ a_bound) {
  __shared__ bf16x8 sL[2][2][4 * 3 * 64];  // [stage][expert of the pair][sub-tile][plane][lane]
  const int nT = nmk / 8, nmb = nmk / 2;
  int t, tn;
  col_major_item(blockIdx.x, nT, nTn, t, tn);
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = w >> 1, wc = w & 1;
  const int64_t nbw = 4 * (int64_t)tn + 2 * wc;  // the wave's first column block
  int64_t ncol[2];
#pragma unroll
  for (int c = 0; c < 2; ++c) ncol[c] = 32 * (nbw + c) + (lane & 31);
  const float unscale = ldexpf(1.f, -(img_exp(*s_bound) + img_exp(*a_bound)));
  const __amdgpu_buffer_rsrc_t rT = img_rsrc(Sfr, s_bytes), rB = img_rsrc(Afr, afr_bytes);
  const uint32_t sexp = (uint32_t)nmb * (uint32_t)nmk * 3u * kFragBytes;  // one expert's S image
  const uint32_t tb = (uint32_t)(4 * t * nmk) * 3u * kFragBytes;
  const uint32_t sB0 = (uint32_t)(nbw * nmk) * 3u * kFragBytes, sBc = (uint32_t)nmk * 3u * kFragBytes;
  const uint32_t vB = 16u * lane;
  // T stage units (both experts): e = tid + 256 s -> sub-tile e / 128, plane (e / 64) % 2
  uint32_t vT[2];
  int dT[2];
#pragma unroll
  for (int s2 = 0; s2 < 2; ++s2) {
    const int e = tid + 256 * s2, i = e / 128, p = (e / 64) % 2;
    vT[s2] = (uint32_t)((i * nmk * 192 + p * 64 + (e & 63)) * 16);
    dT[s2] = (3 * i + p) * 64 + (e & 63);
  }
  floatx16 out[2][2];
#pragma unroll
  for (int il = 0; il < 2; ++il)
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
      for (int e = 0; e < 16; ++e) out[il][c][e] = 0.f;

  for (int k = 0; k < K; k += 2) {
    const int k1 = k + 1 < K ? k + 1 : k;
    const uint32_t tb0 = (uint32_t)k * sexp + tb, tb1 = (uint32_t)k1 * sexp + tb;
    floatx16 acc0[2][2], acc1[2][2];
#pragma unroll
    for (int il = 0; il < 2; ++il)
#pragma unroll
      for (int c = 0; c < 2; ++c)
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          acc0[il][c][e] = 0.f;
          acc1[il][c][e] = 0.f;
        }
    auto load_b = [&](bf16x8 (&b)[2][3], int mk) {
      const uint32_t o = (uint32_t)mk * 3u * kFragBytes;
#pragma unroll
      for (int c = 0; c < 2; ++c)
#pragma unroll
        for (int p = 0; p < 2; ++p) b[c][p] = ld_frag(rB, vB, sB0 + c * sBc + o + p * kFragBytes);
    };
    auto load_t = [&](u32x4v (&st)[4], int mk) {
      const uint32_t o = (uint32_t)mk * 192u * 16u;
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        st[s2] = __builtin_amdgcn_raw_buffer_load_b128(rT, vT[s2], tb0 + o, 0);
        st[2 + s2] = __builtin_amdgcn_raw_buffer_load_b128(rT, vT[s2], tb1 + o, 0);
      }
    };
    auto store_t = [&](int buf, const u32x4v (&st)[4]) {
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        reinterpret_cast<u32x4v*>(sL[buf][0])[dT[s2]] = st[s2];
        reinterpret_cast<u32x4v*>(sL[buf][1])[dT[s2]] = st[2 + s2];
      }
    };
    auto compute = [&](int buf, const bf16x8 (&b)[2][3]) {
#pragma unroll
      for (int il = 0; il < 2; ++il) {
        const int i = 2 * wr + il;
        bf16x8 a0[3], a1[3];
#pragma unroll
        for (int p = 0; p < 2; ++p) {
          a0[p] = sL[buf][0][(i * 3 + p) * 64 + lane];
          a1[p] = sL[buf][1][(i * 3 + p) * 64 + lane];
        }
#pragma unroll
        for (int c = 0; c < 2; ++c) {
          acc0[il][c] = mfma_fmt<2, true>(a0, b[c], acc0[il][c]);
          acc1[il][c] = mfma_fmt<2, true>(a1, b[c], acc1[il][c]);
        }
      }
    };
    bf16x8 b0[2][3], b1[2][3];
    u32x4v st[4];
    load_t(st, 0);
    load_b(b0, 0);
    store_t(0, st);
    __syncthreads();
#pragma nounroll
    for (int mk = 0; mk < nmk; mk += 2) {
      load_t(st, mk + 1);
      load_b(b1, mk + 1);
      __builtin_amdgcn_sched_barrier(0);
      compute(0, b0);
      __builtin_amdgcn_sched_barrier(0);
      store_t(1, st);
      __syncthreads();
      const int m2 = mk + 2 < nmk ? mk + 2 : nmk - 1;  // after the last pair: harmless reload
      load_t(st, m2);
      load_b(b0, m2);
      __builtin_amdgcn_sched_barrier(0);
      compute(1, b1);
      __builtin_amdgcn_sched_barrier(0);
      store_t(0, st);
      __syncthreads();
    }
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      const float g0 = ncol[c] < N ? Gv[(int64_t)k * ldg + ncol[c]] * unscale : 0.f;
      const float g1 = (k + 1 < K && ncol[c] < N) ? Gv[(int64_t)(k + 1) * ldg + ncol[c]] * unscale : 0.f;
#pragma unroll
      for (int il = 0; il < 2; ++il)
#pragma unroll
        for (int e = 0; e < 16; ++e)
          out[il][c][e] = fmaf(g1, acc1[il][c][e], fmaf(g0, acc0[il][c][e], out[il][c][e]));
    }
  }

  // gA = 2 out + gA0, stored as the split image (bf16 x6, for B-d)
  const int64_t i0 = 128 * (int64_t)t;
  const __amdgpu_buffer_rsrc_t r0 =
      __builtin_amdgcn_make_buffer_rsrc((void*)gA0, (short)0, (int)(uint32_t)(M * ld0 * 4), 0x00020000);
  const uint32_t soff = (uint32_t)((i0 * ld0 + 128 * (int64_t)tn) * 4), ld32 = (uint32_t)ld0;
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    const int nl = 32 * (2 * wc + c) + (lane & 31);
    const bool ok = ncol[c] < N;
#pragma unroll
    for (int il = 0; il < 2; ++il) {
      const int i = 2 * wr + il;
      float v[16];
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const uint32_t rl = (uint32_t)(32 * i + acc_row(e, lane));
        const float a0 = __builtin_bit_cast(
            float, __builtin_amdgcn_raw_buffer_load_b32(r0, (rl * ld32 + (uint32_t)nl) * 4u, soff, 0));
        v[e] = ok ? fmaf(2.f, out[il][c][e], a0) : 0.f;  // rows >= M read 0 (outside the resource)
      }
      const int64_t mk = 8 * (int64_t)t + 2 * i;
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        float u[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) u[j] = v[8 * s2 + j];
        store_split(gAfr + (((nbw + c) * nmk + mk + s2) * 3) * 64 + lane, u);
      }
    }
  }
}

// B-b from the forward's C images (split-f16 training, mgp_conditional_backward_f16c):
// gA = 2 sum_k L_k (C_k diag(Gv_k)) + gA0 -- the triangular L_k instead of the full
// S_k = L_k L_k^T, so half of grad_a_s's products, and no S_k build.  T = L_k's
// image with rows m, k-steps over m' <= m (DIAG 2, mk < 8 t + 8), B = C_k's image
// (one column sub-tile per wave).  A workgroup takes the row-tile pair (nT - 1 - p,
// p) of a column tile for every expert in turn (K4's balancing): the pairs of a
// column tile then do equal work per expert and stay in step on one XCD, so each
// C_k column strip is read from HBM about once and served to the other pairs
// from L2 (one row tile per workgroup: the light tiles ran ahead through the
// experts and every strip came from HBM/MALL ~4.5 times).
// cexp != nullptr (MGP_TRSM_BWD16): the image is split-f16 instead of x6, each
// column of the 128-row tile t scaled by 2^e, e = img_exp(max over the tile's rows of
// |gA[., n]|) -- exact per (tile, column), so no bound can be loose -- and e goes to
// cexp[t][n] (kCexpZero for an all-zero tile) for trsm_bwd16_kernel.
constexpr float kCexpZero = 1000.f;
template <int NC>
__device__ __forceinline__ void grad_a_c_store(const floatx16 (&out)[4][NC], int c, int t, int tn, int w, int lane,
                                               int nmk, int64_t M, int64_t N, const float* __restrict__ gA0,
                                               int64_t ld0, bf16x8* __restrict__ gAfr, float* __restrict__ cexp,
                                               int64_t ldc) {
  const int64_t nb = 4 * (int64_t)tn + w;
  const int64_t n = 32 * nb + (lane & 31);
  const int64_t i0 = 128 * (int64_t)t;
  const __amdgpu_buffer_rsrc_t r0 =
      __builtin_amdgcn_make_buffer_rsrc((void*)gA0, (short)0, (int)(uint32_t)(M * ld0 * 4), 0x00020000);
  const uint32_t soff = (uint32_t)((i0 * ld0 + 128 * (int64_t)tn) * 4), ld32 = (uint32_t)ld0;
  const int nl = 32 * w + (lane & 31);
  const bool ok = n < N;
  if (cexp) {
    float v[4][16];
    float mx = 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const uint32_t rl = (uint32_t)(32 * i + acc_row(e, lane));
        const float b0 = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r0, (rl * ld32 + (uint32_t)nl) * 4u, soff, 0));
        v[i][e] = ok ? fmaf(2.f, out[i][c][e], b0) : 0.f;
        mx = fmaxf(mx, fabsf(v[i][e]));
      }
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64));  // the column's other 16 rows of each 32-row block
    // 2^ex as two factors: a tile of tiny values (|gA| < 2^-114) needs ex > 127
    const int ex = img_exp(mx), ex1 = ex / 2;
    const float sc1 = ldexpf(1.f, ex1), scale = ldexpf(1.f, ex - ex1);
    if (lane < 32 && ok) cexp[t * ldc + n] = mx > 0.f ? (float)ex : kCexpZero;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int64_t mk = 8 * (int64_t)t + 2 * i;
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        float u[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) u[j] = v[i][8 * s2 + j] * sc1;
        store_split_f16(gAfr + ((nb * nmk + mk + s2) * 3) * 64 + lane, u, scale);
      }
    }
    return;
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    float v[16];
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const uint32_t rl = (uint32_t)(32 * i + acc_row(e, lane));
      const float b0 = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r0, (rl * ld32 + (uint32_t)nl) * 4u, soff, 0));
      v[e] = ok ? fmaf(2.f, out[i][c][e], b0) : 0.f;  // rows >= M read 0 (outside the resource)
    }
    const int64_t mk = 8 * (int64_t)t + 2 * i;
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      float u[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) u[j] = v[8 * s2 + j];
      store_split(gAfr + ((nb * nmk + mk + s2) * 3) * 64 + lane, u);
    }
  }
}

template <int I, int N, typename F>
__device__ __forceinline__ void static_for_from(F&& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    static_for_from<I + 1, N>(f);
  }
}
template <int N, typename F>
__device__ __forceinline__ void static_for(F&& f) {
  static_for_from<0, N>(f);
}

// One continuous pipeline over the K L k-steps of a row tile (L = 8 t + 8 per
// expert), in blocks of 8 k-steps: for each 8-row-step block of m' (outer), for
// each expert k, its 8 k-steps.  T (L_k's row slab, via registers into the LDS
// double buffer), B (C_k's fragments, straight to registers) and g = Gv_k[n] are
// loaded PD k-steps ahead into a register ring of PD + 1 sets, across expert and
// block boundaries; every load of a k-step is issued before any of a later one
// (vector loads complete in order), so the wait for k-step s + 1's T slab never
// forces a younger prefetch.  Block order keeps the workgroups of a column tile in
// step: all start the first pass (row tile nT - 1 - p, nT - p blocks) at block 0 and
// advance one block per unit time, and the second pass (row tile p) runs its blocks
// downwards, which puts every workgroup at block nT - time in it -- so each C_k
// strip is fetched about twice per column tile, not once per workgroup.
// The per-column expert weights need no second accumulator set: acc holds the
// running sum in units of the current expert's g, sum (g_j / g_k) P_j, rescaled by
// g_k / g_k' at each expert switch (every 8 k-steps) and by the last g at the end
// -- each rescale is one f32 rounding relative to the running total, as for
// out += g acc.  |g| is clamped from below to 2^-40 max_k |g_k[n]| (the clamp moves
// the result by < 2^-40 of the largest contribution; the quotient stays < 2^82 of
// it).  DIAG masks are not applied: the zero blocks of the diagonal tile are
// zero-filled in the image (8 % more MFMAs, no branch in the pipeline).
// NC: 32-column sub-tiles per wave (workgroup = 128 rows x 128 NC columns).
// grad_a_c_kernel's prefetch distance and column sub-tiles per wave (c3, MI355X:
// PD 3 / NC 1 1.72 ms; PD 1 / NC 2 1.77 ms, 264 B of spill in its epilogue)
#ifndef MGP_GAC_PD
#define MGP_GAC_PD 3
#define MGP_GAC_NC 1
#endif
constexpr int kGacPD = MGP_GAC_PD, kGacNC = MGP_GAC_NC;
// the split-f16 C-images backward on grad_a_c16_kernel (0: grad_a_c_kernel; A/B)
#ifndef MGP_GAC16
#define MGP_GAC16 1
#endif
constexpr bool kGac16 = MGP_GAC16;
// grad_a_c16_kernel's row-tile groups per workgroup (1; 2: two row tiles at once, measured
// slower -- 3.0 vs 1.78 ms per launch for 3.2 vs 8.1 GB fetched, r06k_gac16_train_ab.log)
#ifndef MGP_GAC16_G
#define MGP_GAC16_G 1
#endif
constexpr int kGac16G = MGP_GAC16_G;

template <int PD, int NC>
__global__ __launch_bounds__(256, 2) void grad_a_c_kernel(const bf16x8* __restrict__ Ltfr, uint32_t lt_bytes,
                                                         const bf16x8* __restrict__ Cfr, int64_t cexp,
                                                         uint32_t c_bytes, int nmk, int nTn, int K, int64_t M,
                                                         int64_t N, const float* __restrict__ Gv, int64_t ldg,
                                                         const float* __restrict__ gA0, int64_t ld0,
                                                         bf16x8* __restrict__ gAfr,
                                                         const float* __restrict__ l_bound,
                                                         const float* __restrict__ a_bound,
                                                         const float* __restrict__ colmax,
                                                         float* __restrict__ gexp, int64_t ldc) {
  constexpr int U = PD + 1;
  static_assert(8 % U == 0, "the ring cycles within an expert's 8 k-steps (and the LDS double buffer)");
  __shared__ bf16x8 sL[2][4 * 3 * 64];
  const int nT = nmk / 8, nmb = nmk / 2, nP = (nT + 1) / 2;
  int p, tn;
  col_major_item(blockIdx.x, nP, nTn, p, tn);
  const int t1 = nT - 1 - p, t2 = p;  // t1 == t2: the middle tile of an odd nT, alone
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int64_t nb = 4 * NC * (int64_t)tn + NC * w;  // column blocks nb .. nb + NC - 1 (32 wide)
  const float unscale =
      ldexpf(1.f, -(img_exp(*l_bound) + img_exp(*colmax * *a_bound * 1.0009765625f)));
  const __amdgpu_buffer_rsrc_t rT = img_rsrc(Ltfr, lt_bytes);
  const __amdgpu_buffer_rsrc_t rG =
      __builtin_amdgcn_make_buffer_rsrc((void*)Gv, (short)0, (int)(uint32_t)(K * ldg * 4), 0x00020000);
  uint32_t vG[NC];
  float gmin[NC];
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const int64_t n = 32 * (nb + c) + (lane & 31);
    vG[c] = (uint32_t)(n < N ? n : 0) * 4u;
    float gmax = 0.f;
    for (int k = 0; k < K; ++k)
      gmax = fmaxf(gmax, fabsf(__builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                                                             rG, vG[c], (uint32_t)(k * ldg * 4), 0))));
    gmin[c] = fmaxf(gmax * 0x1p-40f, 0x1p-126f);
  }
  // T stage: thread tid moves units e = tid + 256 s (s = 0, 1): row sub-tile e / 128,
  // plane (e / 64) % 2, lane e % 64
  uint32_t vT[2];
  int dT[2];
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    const int e = tid + 256 * s, i = e / 128, pl = (e / 64) % 2;
    vT[s] = (uint32_t)((i * nmk * 192 + pl * 64 + (e & 63)) * 16);
    dT[s] = (3 * i + pl) * 64 + (e & 63);
  }
  const uint32_t vB = 16u * lane;
  for (int pass = 0; pass < (t2 != t1 ? 2 : 1); ++pass) {
    const int t = pass ? t2 : t1;
    const int L = 8 * t + 8, S = K * L;
    u32x4v st[U][2];
    bf16x8 bb[U][NC][3];
    // the load stream's k-step: 8-step block lmb (outer; the second pass runs it
    // downwards), expert lk, mk = 8 lmb + lj; index ls
    const int dmb = pass ? -1 : 1;
    int lk = 0, lmb = pass ? t : 0, lj = 0, ls = 0;
    auto issue = [&](auto jc) {
      constexpr int J = decltype(jc)::value;
      const int lmk = 8 * lmb + lj;
      const uint32_t ot = (uint32_t)(((int64_t)lk * nmb + 4 * t) * nmk + lmk) * 192u * 16u;
#pragma unroll
      for (int s = 0; s < 2; ++s) st[J][s] = __builtin_amdgcn_raw_buffer_load_b128(rT, vT[s], ot, 0);
      const __amdgpu_buffer_rsrc_t rB = img_rsrc(Cfr + (int64_t)lk * cexp, c_bytes);
#pragma unroll
      for (int c = 0; c < NC; ++c) {
        const uint32_t ob = (uint32_t)((nb + c) * nmk + lmk) * 3u * kFragBytes;
#pragma unroll
        for (int pl = 0; pl < 2; ++pl) bb[J][c][pl] = ld_frag(rB, vB, ob + pl * kFragBytes);
      }
      if (ls < S - 1) {  // advance (the stream stays on the last k-step once it is reached)
        ++ls;
        if (++lj == 8) {
          lj = 0;
          if (++lk == K) {
            lk = 0;
            lmb += dmb;
          }
        }
      }
    };
    auto loadg = [&](int k, float (&g)[NC]) {
#pragma unroll
      for (int c = 0; c < NC; ++c) {
        const float x =
            __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rG, vG[c], (uint32_t)(k * ldg * 4), 0));
        g[c] = __builtin_copysignf(fmaxf(fabsf(x), gmin[c]), x);
      }
    };
    floatx16 acc[4][NC];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int c = 0; c < NC; ++c)
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[i][c][e] = 0.f;
    // compute stream: expert ck; acc in units of gcur (= expert ck's g)
    int ck = 0;
    float gcur[NC], gnext[NC];
    loadg(0, gcur);
    static_for<PD>([&](auto jc) { issue(jc); });
#pragma unroll
    for (int s = 0; s < 2; ++s) reinterpret_cast<u32x4v*>(sL[0])[dT[s]] = st[0][s];
    __syncthreads();
    // the 8 k-steps of one (block, expert)
#pragma nounroll
    for (int s0 = 0; s0 < S; s0 += 8) {
      static_for<8>([&](auto jc) {
        constexpr int JJ = decltype(jc)::value, J = JJ % U;
        issue(std::integral_constant<int, (J + PD) % U>{});
        if constexpr (JJ == 0) loadg(ck + 1 < K ? ck + 1 : 0, gnext);  // needed at JJ = 7
        __builtin_amdgcn_sched_barrier(0);
        // NC = 1: all 8 LDS reads in flight before the first MFMA (3 MFMAs per
        // fragment pair would wait on each read); NC = 2: two sub-tiles at a time
        constexpr int RB = NC == 1 ? 4 : 2;
#pragma unroll
        for (int i0 = 0; i0 < 4; i0 += RB) {
          bf16x8 a[RB][3];
#pragma unroll
          for (int i = 0; i < RB; ++i)
#pragma unroll
            for (int pl = 0; pl < 2; ++pl) a[i][pl] = sL[J % 2][((i0 + i) * 3 + pl) * 64 + lane];
          if constexpr (RB == 4) __builtin_amdgcn_sched_barrier(0);
#pragma unroll
          for (int i = 0; i < RB; ++i)
#pragma unroll
            for (int c = 0; c < NC; ++c) acc[i0 + i][c] = mfma_fmt<2, true>(a[i], bb[J][c], acc[i0 + i][c]);
        }
        __builtin_amdgcn_sched_barrier(0);
        if constexpr (JJ == 7) {  // end of the expert's 8 k-steps: to units of the next one's g
#pragma unroll
          for (int c = 0; c < NC; ++c) {
            const float r = gcur[c] / gnext[c];
            gcur[c] = gnext[c];
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
              for (int e = 0; e < 16; ++e) acc[i][c][e] *= r;
          }
        }
#pragma unroll
        for (int s = 0; s < 2; ++s) reinterpret_cast<u32x4v*>(sL[(J + 1) % 2])[dT[s]] = st[(J + 1) % U][s];
        __syncthreads();
      });
      if (++ck == K) ck = 0;
    }
    // acc is in units of gcur (the wrapped-around expert 0's g after the last block)
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      const float gl = gcur[c] * unscale;
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[i][c][e] *= gl;
      // column block nb + c as (128-column tile, wave) of the one-block store
      grad_a_c_store(acc, c, t, (int)((nb + c) / 4), (int)((nb + c) % 4), lane, nmk, M, N, gA0, ld0, gAfr, gexp,
                     ldc);
    }
  }
}

// B-b from the C images on 16x16x32 MFMAs (round 6; replaces grad_a_c_kernel in the
// split-f16 training step): the same sum gA = 2 sum_k L_k (C_k diag(Gv_k)) + gA0 and the
// same per-(tile, column) exponent image, but with K5's main-loop shape instead of
// grad_a_c's 32x32x16 one -- wave tile 128 rows x 64 columns (8 x 4 blocks of 16 x 16),
// one LDS barrier per 32-deep k-step PAIR (96 MFMAs per wave) instead of per 16-deep
// k-step (12 MFMAs), and half the LDS bytes per MFMA (each staged L_k fragment feeds
// four column blocks instead of one).  grad_a_c measured 54-57 % MFMA busy with an
// LDS read per 1.5 MFMAs; K5's shape runs at ~80 %.
// Item = (row-tile pair (nT - 1 - p, p), 256-column tile tn), both passes as grad_a_c.
// The pair stream of a pass (row tile t): blocks of 4 pairs (8 k-steps) outer (the
// second pass runs them downwards, as grad_a_c, so the workgroups of a column tile
// stay in step on one XCD), experts inner; after an expert's 4 pairs the accumulator
// goes to units of the next expert's column weight (grad_a_c's rescale: one f32
// rounding per switch relative to the running sum, |g| clamped below at 2^-40 of the
// column's largest).  The column weights (K x 256) and their clamps sit in LDS.
// Zero blocks of the diagonal tile are zero-filled in the L_k image (no masks).
constexpr int kGac16KMax = 16;
// G = 1 (the default): two passes per 256-thread workgroup, as above.  G = 2 (measured,
// not kept): a 512-thread workgroup takes the row tiles (2j + 1, 2j) of a column tile AT
// ONCE, one per 4-wave group, over one stream of blocks ascending, so that both groups
// read the same C_k fragments between the same barriers.  With G = 1 the row-tile
// workgroups of a column tile share the C_k strips only through L2 when they happen to
// be in step (8.1 GB fetched per launch for 2.1 GB of images, profiles/
// r06i_pmc_cond_bwd_f16c.json); G = 2 fetches 3.2 GB but runs 3.0 ms instead of 1.78
// (one 8-wave workgroup per CU, a barrier over both groups, the short tile's group idle
// through the long tile's extra blocks) -- the fetched bytes are not what bounds it.
template <int G>
__global__ __launch_bounds__(256 * G, 2 / G) void grad_a_c16_kernel(const bf16x8* __restrict__ Ltfr, uint32_t lt_bytes,
                                                            const bf16x8* __restrict__ Cfr, int64_t cexp,
                                                            uint32_t c_bytes, int nmk, int nTn, int K, int64_t M,
                                                            int64_t N, const float* __restrict__ Gv, int64_t ldg,
                                                            const float* __restrict__ gA0, int64_t ld0,
                                                            bf16x8* __restrict__ gAfr,
                                                            const float* __restrict__ l_bound,
                                                            const float* __restrict__ a_bound,
                                                            const float* __restrict__ colmax,
                                                            float* __restrict__ gexp, int64_t ldc) {
  __shared__ bf16x8 sL[G][2][4 * 2 * 2 * 64];
  __shared__ float sG[kGac16KMax * 256];
  const int nT = nmk / 8, nmb = nmk / 2;
  const int nI = G == 1 ? (nT + 1) / 2 : (nT + 1) / 2;   // items per column tile
  int p, tn;
  col_major_item(blockIdx.x, nI, nTn, p, tn);
  const int grp = G == 2 ? __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 8)) : 0;
  // G = 1: passes over row tiles t1 = nT - 1 - p, then t2 = p (t1 == t2: the middle tile of
  // an odd nT, alone).  G = 2: one pass over blocks 0 .. th, th = min(2p + 1, nT - 1);
  // group 0 owns row tile th, group 1 row tile 2p (none when th == 2p)
  const int th = G == 2 ? (2 * p + 1 < nT ? 2 * p + 1 : nT - 1) : 0;
  const int own2 = grp == 0 ? th : (2 * p < th ? 2 * p : -1);
  const int tid = threadIdx.x & 255, lane = tid & 63, li = lane & 15, q = lane >> 4;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const float unscale =
      ldexpf(1.f, -(img_exp(*l_bound) + img_exp(*colmax * *a_bound * 1.0009765625f)));
  // column weights of the tile (column tid), clamped from below at 2^-40 of the column's largest
  if (grp == 0) {
    const int64_t n = 256 * (int64_t)tn + tid;
    float gmax = 0.f;
    for (int k = 0; k < K; ++k) {
      const float x = n < N ? Gv[(int64_t)k * ldg + n] : 0.f;
      sG[k * 256 + tid] = x;
      gmax = fmaxf(gmax, fabsf(x));
    }
    const float gmin = fmaxf(gmax * 0x1p-40f, 0x1p-126f);
    for (int k = 0; k < K; ++k) {
      const float x = sG[k * 256 + tid];
      sG[k * 256 + tid] = __builtin_copysignf(fmaxf(fabsf(x), gmin), x);
    }
  }
  // T staging (x6_mainloop16, NPL 2): unit e = tid + 256 s: sub-tile e / 256, k-step
  // (e / 128) % 2 of the pair, plane (e / 64) % 2
  uint32_t vT[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    const int e = tid + 256 * s, i = e / 256, kk = (e / 128) % 2, pl = (e / 64) % 2;
    vT[s] = (uint32_t)((((i * nmk + kk) * 3 + pl) * 64 + (e & 63)) * 16);
  }
  const uint32_t vB = (uint32_t)((((q >> 1) * 3) * 64 + li + 32 * (q & 1)) * 16);
  const uint32_t sB0 = (uint32_t)((8 * tn + 2 * w) * nmk) * 3u * kFragBytes;
  const int aoff = (q >> 1) * 64 * 2 + li + 32 * (q & 1);
  const int col0 = 64 * w + li;   // this lane's column of block cb: col0 + 16 cb (within the tile)
  bf16x8 (*sLg)[4 * 2 * 2 * 64] = sL[grp];
  __syncthreads();   // sG
  for (int pass = 0; pass < (G == 1 ? (nT - 1 - p != p ? 2 : 1) : 1); ++pass) {
    const int trun = G == 1 ? (pass ? p : nT - 1 - p) : th;   // the stream's blocks 0 .. trun
    const int t = G == 1 ? trun : own2;                      // this group's row tile (-1: none)
    const bool desc = G == 1 && pass;                        // G = 1, second pass: blocks downwards
    const int S = K * 4 * (trun + 1);                        // pairs of the stream (even)
    // pair s_ of the stream -> (expert k, pair ks, block b)
    auto at = [&](int s_, int& k, int& ks) {
      const int bi = s_ / (4 * K), r = s_ % (4 * K);
      k = r >> 2;
      ks = 4 * (desc ? trun - bi : bi) + (r & 3);
    };
    auto active = [&](int s_) {   // uniform per group: this group's tile needs the pair
      if (G == 1) return true;
      const int bi = s_ / (4 * K);
      return bi <= t;
    };
    auto load_t = [&](u32x4v (&st)[4], int s_) {
      if (!active(s_)) return;
      int k, ks;
      at(s_, k, ks);
      const uint32_t o = (uint32_t)(((int64_t)k * nmb + 4 * t) * nmk + 2 * ks) * 3u * kFragBytes;
#pragma unroll
      for (int u = 0; u < 4; ++u) st[u] = __builtin_amdgcn_raw_buffer_load_b128(img_rsrc(Ltfr, lt_bytes), vT[u], o, 0);
    };
    auto load_b = [&](bf16x8 (&b)[4][3], int s_) {
      if (!active(s_)) return;
      int k, ks;
      at(s_, k, ks);
      const __amdgpu_buffer_rsrc_t rB = img_rsrc(Cfr + (int64_t)k * cexp, c_bytes);
#pragma unroll
      for (int cb = 0; cb < 4; ++cb)
#pragma unroll
        for (int pl = 0; pl < 2; ++pl)
          b[cb][pl] = ld_frag(rB, vB, sB0 + (uint32_t)(cb >> 1) * (uint32_t)nmk * 3u * kFragBytes +
                                          (uint32_t)((2 * ks) * 3 + pl) * kFragBytes + (uint32_t)(16 * (cb & 1)) * 16u);
    };
    auto store_t = [&](int buf, const u32x4v (&st)[4], int s_) {
      if (!active(s_)) return;
#pragma unroll
      for (int u = 0; u < 4; ++u) reinterpret_cast<u32x4v*>(sLg[buf])[tid + 256 * u] = st[u];
    };
    floatx4v acc[8][4];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int c = 0; c < 4; ++c) acc[i][c] = floatx4v{0.f, 0.f, 0.f, 0.f};
    auto compute = [&](int buf, const bf16x8 (&b)[4][3], int s_) {
      if (!active(s_)) return;
#pragma unroll
      for (int ib = 0; ib < 8; ++ib) {
        const int base = (ib >> 1) * 128 * 2 + 16 * (ib & 1) + aoff;
        bf16x8 a[3];
#pragma unroll
        for (int pl = 0; pl < 2; ++pl) a[pl] = sLg[buf][base + 64 * pl];
#pragma unroll
        for (int cb = 0; cb < 4; ++cb) acc[ib][cb] = mfma16_fmt<2, true>(a, b[cb], acc[ib][cb]);
      }
    };
    // after expert k's 4 pairs of a block: to units of expert (k + 1) % K's weight
    auto rescale = [&](int s_) {
      if (!active(s_)) return;
      const int k = (s_ % (4 * K)) >> 2, kn = k + 1 < K ? k + 1 : 0;
#pragma unroll
      for (int cb = 0; cb < 4; ++cb) {
        const float r = sG[k * 256 + col0 + 16 * cb] / sG[kn * 256 + col0 + 16 * cb];
#pragma unroll
        for (int ib = 0; ib < 8; ++ib) acc[ib][cb] *= r;
      }
    };
    bf16x8 b0[4][3], b1[4][3];
    u32x4v st[4];
    load_t(st, 0);
    load_b(b0, 0);
    store_t(0, st, 0);
    __syncthreads();
#pragma nounroll
    for (int s_ = 0; s_ < S; s_ += 2) {
      load_t(st, s_ + 1);
      load_b(b1, s_ + 1);
      __builtin_amdgcn_sched_barrier(0);
      compute(0, b0, s_);
      __builtin_amdgcn_sched_barrier(0);
      store_t(1, st, s_ + 1);
      __syncthreads();
      const int s2 = s_ + 2 < S ? s_ + 2 : S - 1;  // after the last pair: harmless reload
      load_t(st, s2);
      load_b(b0, s2);
      __builtin_amdgcn_sched_barrier(0);
      compute(1, b1, s_ + 1);
      __builtin_amdgcn_sched_barrier(0);
      if ((s_ & 3) == 2) rescale(s_ + 1);   // pair s_ + 1 ended the expert's block
      store_t(0, st, s2);
      __syncthreads();
    }
    if (t < 0) continue;   // (G = 2: a group without a row tile; uniform per group, no barrier below)
    // acc is in units of expert 0's weight (the wrap after the last block)
    float gl[4], mx[4];
#pragma unroll
    for (int cb = 0; cb < 4; ++cb) {
      gl[cb] = sG[col0 + 16 * cb] * unscale;
      mx[cb] = 0.f;
    }
    // gA = 2 out + gA0 (rows >= M read 0 outside the resource), column maxima over the tile
    const int64_t i0 = 128 * (int64_t)t;
    const __amdgpu_buffer_rsrc_t r0 =
        __builtin_amdgcn_make_buffer_rsrc((void*)gA0, (short)0, (int)(uint32_t)(M * ld0 * 4), 0x00020000);
    uint32_t ld32 = (uint32_t)ld0;
    // (opaque per pass: otherwise the 128 per-lane epilogue offsets are hoisted out of the
    // pass loop and spilled across the main loop)
    asm volatile("" : "+s"(ld32));
    const uint32_t soff = (uint32_t)((i0 * ld0 + 256 * (int64_t)tn) * 4);
#pragma unroll
    for (int cb = 0; cb < 4; ++cb) {
      const int nl = col0 + 16 * cb;
      const bool ok = 256 * (int64_t)tn + nl < N;
#pragma unroll
      for (int ib = 0; ib < 8; ++ib)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const uint32_t rl = (uint32_t)(16 * ib + 4 * q + e);
          const float a0 =
              __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r0, (rl * ld32 + (uint32_t)nl) * 4u, soff, 0));
          const float v = ok ? fmaf(2.f, acc[ib][cb][e] * gl[cb], a0) : 0.f;
          acc[ib][cb][e] = v;
          mx[cb] = fmaxf(mx[cb], fabsf(v));
        }
      mx[cb] = fmaxf(mx[cb], lane_xor16(mx[cb]));
      mx[cb] = fmaxf(mx[cb], lane_xor32(mx[cb]));
      const int64_t n = 256 * (int64_t)tn + nl;
      if (q == 0 && ok) gexp[t * ldc + n] = mx[cb] > 0.f ? (float)img_exp(mx[cb]) : kCexpZero;
    }
    // the split-f16 image at 2^e per column (two factors: e can pass 127): fragment
    // (32-column block 8 tn + 2 w + c, k-step 8 t + ib) from the 16x16 blocks (ib, 2c)
    // and (ib, 2c + 1) through one lane-half exchange (K4's epilogue)
    const bool lo_half = lane < 32;
    const int pos = lo_half ? li + 32 * q : 16 + li + 32 * (q - 2);
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      const int ex = img_exp(lo_half ? mx[2 * c] : mx[2 * c + 1]), ex1 = ex / 2;
      const float sc1 = ldexpf(1.f, ex1), scale = ldexpf(1.f, ex - ex1);
#pragma unroll
      for (int ib = 0; ib < 8; ++ib) {
        float v[8];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          v[r] = acc[ib][2 * c][r];
          v[4 + r] = acc[ib][2 * c + 1][r];
          lane_half_swap(v[r], v[4 + r]);
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] *= sc1;
        store_split_f16(gAfr + ((((int64_t)8 * tn + 2 * w + c) * nmk + 8 * t + ib) * 3) * 64 + pos, v, scale);
      }
    }
  }
}

// max over k, j of ||tril(q_sqrt[k])[:, j]||_2 -> *out (float bits, atomicMax; zeroed
// beforehand).  Workgroup = (32 columns, expert k): thread (ty, tx) sums rows
// ty, ty + 8, ... of column 32 blockIdx.x + tx (row-contiguous loads), LDS sums
// the 8 partials, one atomic per workgroup.
__global__ __launch_bounds__(256) void colnorm_max_kernel(const float* __restrict__ q, int64_t ldq, int64_t sq,
                                                          int64_t M, unsigned int* __restrict__ out) {
  __shared__ float part[8][33];
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
  const int64_t j = (int64_t)blockIdx.x * 32 + tx;
  const float* Q = q + (int64_t)blockIdx.y * sq;
  float v = 0.f;
  if (j < M) {
#pragma unroll 8
    for (int64_t i = ty; i < M; i += 8) {
      const float x = i >= j ? Q[i * ldq + j] : 0.f;
      v = fmaf(x, x, v);
    }
  }
  part[ty][tx] = v;
  __syncthreads();
  if (threadIdx.x < 32) {
    float c = 0.f;
#pragma unroll
    for (int r = 0; r < 8; ++r) c += part[r][threadIdx.x];
    c = sqrtf(c);
#pragma unroll
    for (int off = 16; off > 0; off >>= 1) c = fmaxf(c, __shfl_xor(c, off, 32));
    if (threadIdx.x == 0) atomicMax(out, __float_as_uint(c));
  }
}

// B-d: gKuf = L^-T gA = Linv^T gA as f32 [M][ld]; T image = Linv (lower in
// (k, i)), B image = gA; items and main loop as K5 (one "expert").
__global__ __launch_bounds__(256, 2) void trsm_bwd_kernel(const bf16x8* __restrict__ gAfr,
                                                         const bf16x8* __restrict__ LIfr, uint32_t gafr_bytes,
                                                         uint32_t lifr_bytes, int nmk, int nmb, int nTn,
                                                         int64_t M, int64_t N, float* __restrict__ gKuf,
                                                         int64_t ldk) {
  __shared__ bf16x8 sL[2][4 * 3 * 64];
  int t, tn;
  col_major_item(blockIdx.x, nmk / 8, nTn, t, tn);
  t = nmk / 8 - 1 - t;  // lower T from the diagonal on: row tile 0 is the heaviest
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  floatx16 acc[4][2];
  x6_mainloop<1, 2, 3, false, false, true>(acc, sL, img_rsrc(LIfr, lifr_bytes), (uint32_t)((4 * t) * nmk) * 3u * kFragBytes,
                    img_rsrc(gAfr, gafr_bytes), (uint32_t)((8 * tn + 2 * w) * nmk) * 3u * kFragBytes, 8 * t, nmk, nmk);
  store_acc_f32(acc, gKuf, ldk, 128 * (int64_t)t, (int64_t)tn * kX6BN, M, N, nullptr);
}

// B-d on split-f16 images (MGP_TRSM_BWD16): three f16 products per block instead of
// six bf16 ones.  Linv's image at 2^img_exp(*li_bound); gA's image per (128-row tile
// t', column n) at 2^cexp[t'][n] (grad_a_c_store).  Each lane owns one column of each
// of its two sub-tiles: at the start it takes E = min over the tiles t' >= t it
// contracts of cexp[t'][n] (the largest tile), and every B fragment of tile t' is
// multiplied by 2^(E - cexp[t'][n]) <= 1 in f16 right before its MFMAs, so all
// tiles meet in the accumulator at the common scale 2^E (exact powers of two: the
// product is that of the exactly-scaled image; only parts below 2^-24 of the
// column's largest tile are lost to f16 underflow).  Output unscaled by 2^-(E + eL).
constexpr int kTrsmBwd16MaxT = 32;  // row tiles (M <= 4096); larger M: trsm_bwd_kernel
#ifndef MGP_TRSM_BWD16
#define MGP_TRSM_BWD16 1
#endif
constexpr bool kTrsmBwd16 = MGP_TRSM_BWD16;
#ifndef MGP_GLM_F16
#define MGP_GLM_F16 1
#endif
constexpr bool kGlmF16 = MGP_GLM_F16;
__global__ __launch_bounds__(256, 2) void trsm_bwd16_kernel(const bf16x8* __restrict__ gAfr,
                                                           const bf16x8* __restrict__ LIfr, uint32_t gafr_bytes,
                                                           uint32_t lifr_bytes, int nmk, int nmb, int nTn,
                                                           int64_t M, int64_t N, float* __restrict__ gKuf,
                                                           int64_t ldk, const float* __restrict__ cexp, int64_t ldc,
                                                           const float* __restrict__ li_bound,
                                                           float* __restrict__ gmax) {
  __shared__ bf16x8 sL[2][4 * 3 * 64];
  __shared__ float sF[kTrsmBwd16MaxT][kX6BN];  // per (tile t' - t, column): 2^(E - cexp)
  int t, tn;
  const int nT = nmk / 8;
  col_major_item(blockIdx.x, nT, nTn, t, tn);
  t = nT - 1 - t;  // lower T from the diagonal on: row tile 0 is the heaviest
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  {  // thread = one column of the item
    const int64_t n = (int64_t)tn * kX6BN + threadIdx.x;
    float E = kCexpZero;
    if (n < N)
      for (int tp = t; tp < nT; ++tp) E = fminf(E, cexp[tp * ldc + n]);
    for (int tp = t; tp < nT; ++tp) sF[tp - t][threadIdx.x] = n < N ? exp2f(E - cexp[tp * ldc + n]) : 0.f;
  }
  float E2[2];
#pragma unroll
  for (int c = 0; c < 2; ++c) {  // this lane's columns (the accumulators' and the B fragments')
    const int64_t n = (int64_t)tn * kX6BN + 64 * w + 32 * c + (lane & 31);
    float E = kCexpZero;
    if (n < N)
      for (int tp = t; tp < nT; ++tp) E = fminf(E, cexp[tp * ldc + n]);
    E2[c] = E;
  }
  int tcur = -1;
  _Float16 f[2] = {(_Float16)1.f, (_Float16)1.f};
  auto bh = [&](bf16x8 (&b)[2][3], int mk) {
    const int tp = mk >> 3;
    if (tp != tcur) {  // uniform: every 8 k-steps
      tcur = tp;
#pragma unroll
      for (int c = 0; c < 2; ++c) f[c] = (_Float16)sF[tp - t][64 * w + 32 * c + (lane & 31)];
    }
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
      for (int p = 0; p < 2; ++p)
        b[c][p] = __builtin_bit_cast(bf16x8, __builtin_bit_cast(halfx8, b[c][p]) * f[c]);
  };
  floatx16 acc[4][2];
  x6_mainloop<1, 2, 2, true, false, true>(acc, sL, img_rsrc(LIfr, lifr_bytes), (uint32_t)((4 * t) * nmk) * 3u * kFragBytes,
                    img_rsrc(gAfr, gafr_bytes), (uint32_t)((8 * tn + 2 * w) * nmk) * 3u * kFragBytes, 8 * t, nmk, nmk,
                    true, bh);
  const int eL = img_exp(*li_bound);
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    // 2^-(E + eL) as two factors (E reaches ~160 for a column of tiny values)
    const float x = E2[c] + (float)eL, x1 = floorf(0.5f * x);
    const float u1 = E2[c] >= kCexpZero ? 0.f : exp2f(-x1), u2 = exp2f(x1 - x);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][c][e] = acc[i][c][e] * u1 * u2;
  }
  if (gmax) {  // max |gKuf[m][.]| over this wave's 64 columns per row -> gmax[4 tn + w][m]
    float* dst = gmax + (int64_t)(4 * tn + w) * M;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const float m = half_max_f32(fmaxf(fabsf(acc[i][0][e]), fabsf(acc[i][1][e])));
        const int64_t row = 128 * (int64_t)t + 32 * i + acc_row(e, lane);
        if ((lane & 31) == 0 && row < M) dst[row] = m;
      }
  }
  store_acc_f32(acc, gKuf, ldk, 128 * (int64_t)t, (int64_t)tn * kX6BN, M, N, nullptr);
}

// out[m] = max over p < np of part[p][m] (blockIdx.y = 0: A's slab partials into
// out[0 .. M), 1: g_Kuf's wave partials into out[M .. 2M)).  Workgroup: 16 rows x 16
// partial groups (a thread takes partials g, g + 64, ... eight loads in flight), LDS
// (16 rows x 16 groups: 21 us per launch at c3; 64 groups: the loads' latency shared).
__global__ __launch_bounds__(1024) void rowmax_fold_kernel(const float* __restrict__ pa, int npa,
                                                           const float* __restrict__ pg, int npg, int64_t M,
                                                           float* __restrict__ out) {
  __shared__ float sm[64][17];
  const int r = threadIdx.x & 15, g = threadIdx.x >> 4;
  const int64_t m = (int64_t)blockIdx.x * 16 + r;
  const float* p = blockIdx.y ? pg : pa;
  const int np = blockIdx.y ? npg : npa;
  float v = 0.f;
  if (m < M) {
#pragma unroll 8
    for (int q = g; q < np; q += 64) v = fmaxf(v, p[(int64_t)q * M + m]);
  }
  sm[g][r] = v;
  __syncthreads();
  if (threadIdx.x < 16 && m < M) {
    float x = sm[0][r];
#pragma unroll
    for (int k = 1; k < 64; ++k) x = fmaxf(x, sm[k][r]);
    out[blockIdx.y * M + m] = x;
  }
}

// ------------------------------------------------------------------ K4 (x6)
// A = LinvT^T Kuf from the images Tfr (LinvT, upper) and Kfr (Kuf): item =
// (row tile t of 128 rows, heavy = large t first; column tile tn of 256), the
// 16 k-steps... 8 t + 8 k-steps of the lower triangle.  Epilogue: the A image
// (registers 8 s .. 8 s + 7 of each 32x32 tile are one B fragment of K5) and
// the stats of the two 64-row stats tiles 2 t, 2 t + 1 (same layout as the
// f32 K4: stats[st][0][n] = sum A^2, stats[st][1 + kk][n] = sum A q_mu[., kk]).
// a_var != nullptr: A's image is split-f16, scaled by 2^img_exp(sqrt(*a_var))
// (|A[m][n]| <= ||A[:, n]|| <= sqrt(k(x_n, x_n)) = sqrt(variance): the Nystrom
// bound; the image trailer a_bound receives sqrt(*a_var) for the consumer).
// F16IN: Tfr and Kfr are split-f16 images (scales 2^img_exp(*t_bound),
// 2^img_exp(*k_bound)): three f16 products per block instead of six bf16 ones;
// the accumulators are unscaled (exact power of two) before the epilogue.
// X8OUT (with F16OUT): the A image also gets its e4m3 cross-term plane (K5 f16x8);
// its f16 lo plane only when the f32 A is written too (training: the backward
// reads planes 0-1), so a forward-only image moves 4 B per element, not 6.
template <int KMAX, bool F16OUT = false, bool F16IN = false, bool X8OUT = false>
__device__ __forceinline__ void trsm_stats_x6_item(
    bf16x8 (*sL)[4 * 3 * 64], float* __restrict__ sQ, int t, int tn, const bf16x8* __restrict__ Tfr,
    uint32_t tfr_bytes, const bf16x8* __restrict__ Kfr, uint32_t kfr_bytes, int nmk, int64_t M, int64_t N,
    const float* __restrict__ q_mu, int64_t ldq, int K, bf16x8* __restrict__ Afr, float* __restrict__ stats,
    int64_t lds_, float* __restrict__ Af32, int64_t lda, const float* __restrict__ a_var,
    const float* __restrict__ t_bound = nullptr, const float* __restrict__ k_bound = nullptr) {
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t i0 = 128 * (int64_t)t;
  float a_scale = 1.f;
  if constexpr (F16OUT) a_scale = ldexpf(1.f, img_exp(sqrtf(*a_var)));
  // q_mu rows of this row tile -> LDS [128][KMAX] before the main loop (whose
  // barriers publish it), so the epilogue never waits on a global load.  F16OUT:
  // also max |q_mu| of the tile (sQ[128 KMAX], as float bits; the caller zeroes
  // it), the power-of-two scale of the split q_mu operand of the stats MFMAs
  if (stats) {
    float qmax = 0.f;
    for (int idx = threadIdx.x; idx < 128 * KMAX; idx += 256) {
      const int r = idx / KMAX, kk = idx % KMAX;
      const float q = (i0 + r < M && kk < K) ? q_mu[(i0 + r) * ldq + kk] : 0.f;
      sQ[idx] = q;
      qmax = fmaxf(qmax, fabsf(q));
    }
    if constexpr (F16OUT) {
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) qmax = fmaxf(qmax, __shfl_xor(qmax, off, 64));
      if ((threadIdx.x & 63) == 0) atomicMax(reinterpret_cast<unsigned int*>(sQ + 128 * KMAX), __float_as_uint(qmax));
    }
  }
  floatx16 acc[4][2];
  x6_mainloop<2, 2, F16IN ? 2 : 3, F16IN>(acc, sL, img_rsrc(Tfr, tfr_bytes), (uint32_t)(4 * t * nmk) * 3u * kFragBytes,
                                          img_rsrc(Kfr, kfr_bytes),
                                          (uint32_t)((8 * tn + 2 * w) * nmk) * 3u * kFragBytes, 0, 8 * t + 8, nmk);
  if constexpr (F16IN) {
    const float unscale = ldexpf(1.f, -(img_exp(*t_bound) + img_exp(*k_bound)));
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int c = 0; c < 2; ++c)
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[i][c][e] *= unscale;
  }
  if (Af32) store_acc_f32(acc, Af32, lda, i0, (int64_t)tn * kX6BN, M, N, nullptr);
  // ---- epilogue by 32-row sub-tile i: the A image fragments of acc[i] and its
  // contribution to the stats of 64-row stats tile i / 2 (stats[st][0][n] = sum A^2,
  // stats[st][1 + kk][n] = sum A q_mu[., kk]); acc[i] dies after its sub-tile, which
  // keeps the live set to the remaining accumulators + 2 (1 + KMAX) sums (no spills)
  if constexpr (F16OUT) {
    // ---- split-f16: the A image, and the stats q_mu^T A on the matrix cores --
    // per 16-row k-step, the image fragments of acc[i][c] (B operand, k = rows)
    // times the split q_mu fragment (A operand: rows kk < K, k = the same 16
    // rows, from sQ) into sq[c] (32 x 32, rows kk); sum A^2 stays VALU.  Stats
    // tile st = 2 t + i / 2 (64 rows) as the VALU path.
    const int qe = img_exp(__uint_as_float(reinterpret_cast<const unsigned int*>(sQ)[128 * KMAX]));
    const float q_scale = ldexpf(1.f, qe), s_unscale = ldexpf(1.f, -(qe + img_exp(sqrtf(*a_var))));
    const int r = lane & 31, h = lane >> 5;
    floatx16 sq[2];
    float a2[2];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      if ((i & 1) == 0) {
#pragma unroll
        for (int c = 0; c < 2; ++c) {
          a2[c] = 0.f;
#pragma unroll
          for (int e = 0; e < 16; ++e) sq[c][e] = 0.f;
        }
      }
      const int64_t mk = 8 * (int64_t)t + 2 * i;
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        bf16x8 qf[3];
        if (stats) {
          halfx8 qh, ql;
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const float x = (r < K ? sQ[(32 * i + 16 * s2 + kperm(h, j)) * KMAX + (r < KMAX ? r : 0)] : 0.f) * q_scale;
            const _Float16 xh = (_Float16)x;
            qh[j] = xh;
            ql[j] = (_Float16)(x - (float)xh);
          }
          qf[0] = __builtin_bit_cast(bf16x8, qh);
          qf[1] = __builtin_bit_cast(bf16x8, ql);
        }
#pragma unroll
        for (int c = 0; c < 2; ++c) {
          const int64_t nb = 8 * (int64_t)tn + 2 * w + c;
          float v[8];
#pragma unroll
          for (int j = 0; j < 8; ++j) v[j] = acc[i][c][8 * s2 + j];
          store_split_f16<X8OUT>(Afr + ((nb * nmk + mk + s2) * 3) * 64 + lane, v, a_scale, Af32 != nullptr);
          if (stats) {
            halfx8 vh, vl;
#pragma unroll
            for (int j = 0; j < 8; ++j) {
              const float x = v[j] * a_scale;
              const _Float16 xh = (_Float16)x;
              vh[j] = xh;
              vl[j] = (_Float16)(x - (float)xh);
              a2[c] = fmaf(v[j], v[j], a2[c]);
            }
            const bf16x8 bf[3] = {__builtin_bit_cast(bf16x8, vh), __builtin_bit_cast(bf16x8, vl), bf16x8{}};
            sq[c] = mfma_fmt<2, true>(qf, bf, sq[c]);
          }
        }
      }
      if (stats && (i & 1)) {
        const int64_t st = 2 * (int64_t)t + (i >> 1);
#pragma unroll
        for (int c = 0; c < 2; ++c) {
          const int64_t n = (int64_t)tn * kX6BN + 64 * w + 32 * c + (lane & 31);
          const float s_a2 = a2[c] + __shfl_xor(a2[c], 32, 64);
          if (n < N && 64 * st < M) {
            float* dst = stats + st * (K + 1) * lds_ + n;
            if (lane < 32) dst[0] = s_a2;
#pragma unroll
            for (int e = 0; e < 16; ++e) {
              const int kk = acc_row(e, lane);
              if (kk < K) dst[(int64_t)(1 + kk) * lds_] = sq[c][e] * s_unscale;
            }
          }
        }
      }
    }
    return;
  }
  float a2[2], qm[2][KMAX];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      const int64_t nb = 8 * (int64_t)tn + 2 * w + c;
      const int64_t mk = 8 * (int64_t)t + 2 * i;
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        float v[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = acc[i][c][8 * s2 + j];
        store_split(Afr + ((nb * nmk + mk + s2) * 3) * 64 + lane, v);
      }
    }
    if (!stats) continue;
    if ((i & 1) == 0) {
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        a2[c] = 0.f;
#pragma unroll
        for (int kk = 0; kk < KMAX; ++kk) qm[c][kk] = 0.f;
      }
    }
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const int lr = 32 * i + acc_row(e, lane);
      const float v0 = acc[i][0][e], v1 = acc[i][1][e];
      a2[0] = fmaf(v0, v0, a2[0]);
      a2[1] = fmaf(v1, v1, a2[1]);
#pragma unroll
      for (int kk = 0; kk < KMAX; ++kk) {
        const float q = sQ[lr * KMAX + kk];
        qm[0][kk] = fmaf(v0, q, qm[0][kk]);
        qm[1][kk] = fmaf(v1, q, qm[1][kk]);
      }
    }
    if (i & 1) {
      const int64_t st = 2 * (int64_t)t + (i >> 1);
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        const int64_t n = (int64_t)tn * kX6BN + 64 * w + 32 * c + (lane & 31);
        const float s_a2 = a2[c] + __shfl_xor(a2[c], 32, 64);
        float s_qm[KMAX];
#pragma unroll
        for (int kk = 0; kk < KMAX; ++kk) s_qm[kk] = qm[c][kk] + __shfl_xor(qm[c][kk], 32, 64);
        if (lane < 32 && n < N && 64 * st < M) {
          float* dst = stats + st * (K + 1) * lds_ + n;
          dst[0] = s_a2;
#pragma unroll
          for (int kk = 0; kk < KMAX; ++kk)
            if (kk < K) dst[(int64_t)(1 + kk) * lds_] = s_qm[kk];
        }
      }
    }
  }
}

// One workgroup per (pair of row tiles t, nT - 1 - t; column tile tn): the
// pair holds 8 t + 8 + 8 (nT - t) = 8 nT + 16 k-steps whatever t, so every
// workgroup has the same work; both items read the same Kuf column slab.  Odd
// nT: the middle row tile is an item alone.  (c3: 385 us vs 439 us for one item
// per workgroup, whose register count stays below 256 without spills.)
template <int KMAX, bool F16OUT = false, bool F16IN = false, bool X8OUT = false>
__global__ __launch_bounds__(256, 2) void trsm_stats_x6_kernel(
    const bf16x8* __restrict__ Tfr, uint32_t tfr_bytes, const bf16x8* __restrict__ Kfr, uint32_t kfr_bytes,
    int nmk, int nTn, int64_t M, int64_t N, const float* __restrict__ q_mu, int64_t ldq, int K,
    bf16x8* __restrict__ Afr, float* __restrict__ stats, int64_t lds_, float* __restrict__ Af32, int64_t lda,
    const float* __restrict__ a_var, float* __restrict__ a_bound, const float* __restrict__ t_bound = nullptr,
    const float* __restrict__ k_bound = nullptr) {
  __shared__ bf16x8 sL[2][4 * 3 * 64];
  __shared__ float sQ[128 * KMAX + 1];  // + the tile's max |q_mu| (F16OUT)
  const int nT = nmk / 8, nP = (nT + 1) / 2;
  int p, tn;
  if constexpr (F16OUT)
    if (blockIdx.x == 0 && threadIdx.x == 0) *a_bound = sqrtf(*a_var);
  col_major_item(blockIdx.x, nP, nTn, p, tn);
  if (threadIdx.x == 0) sQ[128 * KMAX] = 0.f;
  __syncthreads();
  trsm_stats_x6_item<KMAX, F16OUT, F16IN, X8OUT>(sL, sQ, nT - 1 - p, tn, Tfr, tfr_bytes, Kfr, kfr_bytes, nmk, M, N, q_mu,
                                          ldq, K, Afr, stats, lds_, Af32, lda, a_var, t_bound, k_bound);
  if (nT - 1 - p == p) return;
  __syncthreads();  // the epilogue's sQ reads before the next item's sQ stores
  if (threadIdx.x == 0) sQ[128 * KMAX] = 0.f;
  __syncthreads();
  trsm_stats_x6_item<KMAX, F16OUT, F16IN, X8OUT>(sL, sQ, p, tn, Tfr, tfr_bytes, Kfr, kfr_bytes, nmk, M, N, q_mu, ldq, K,
                                          Afr, stats, lds_, Af32, lda, a_var, t_bound, k_bound);
}

// ------------------------------------------------------------------ K4 (split-f16) on 16x16x32 MFMAs
// trsm_stats_x6_item<KMAX, true, true> on x6_mainloop16 (as expert_cond16_kernel is K5 on
// it): the same items, images, outputs and bounds.  Epilogue per 16-row block ib (k-step
// 8 t + ib of A's image): the image fragment of each 32-column block from two lanes of the
// 16x16 accumulator layout (one exchange across the lane halves, as K5's C_k images);
// sum A^2 straight from the accumulators; the q_mu^T A stats of each 64-row stats tile on
// 16x16x32 f16 MFMAs whose B operand is the accumulators themselves: lane (i, q) slot j
// holds row 4q + j (j < 4) of block ib and row 4q + j - 4 of block ib + 1 -- any k order
// shared by both operands is the same sum, so the split q_mu operand (from LDS) is built
// in that order and no exchange is needed.  Rows kk of the 16 x 16 stats block are q_mu's
// columns (KMAX <= 16).
__device__ __forceinline__ void store_acc16_f32(const floatx4v (&acc)[8][4], float* __restrict__ out, int64_t ld,
                                                int64_t i0, int64_t n0, int64_t M, int64_t N) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, li = lane & 15, q = lane >> 4;
  const __amdgpu_buffer_rsrc_t r =
      __builtin_amdgcn_make_buffer_rsrc((void*)out, (short)0, (int)(uint32_t)(M * ld * 4), 0x00020000);
  const uint32_t soff = (uint32_t)((i0 * ld + n0) * 4);
  const uint32_t ld32 = (uint32_t)ld;
#pragma unroll
  for (int cb = 0; cb < 4; ++cb) {
    const int nl = 64 * w + 16 * cb + li;
    if (n0 + nl < N) {
#pragma unroll
      for (int ib = 0; ib < 8; ++ib)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const uint32_t rl = (uint32_t)(16 * ib + 4 * q + e);
          // (through a float: __builtin_bit_cast of the vector element lvalue itself
          // reads element 0 with this compiler)
          const float x = acc[ib][cb][e];
          __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, x), r, (rl * ld32 + (uint32_t)nl) * 4u,
                                                soff, 0);
        }
    }
  }
}

template <int KMAX>
__device__ __forceinline__ void trsm_stats16_item(
    bf16x8 (*sL)[4 * 2 * 3 * 64], float* __restrict__ sQ, int t, int tn, const bf16x8* __restrict__ Tfr,
    uint32_t tfr_bytes, const bf16x8* __restrict__ Kfr, uint32_t kfr_bytes, int nmk, int64_t M, int64_t N,
    const float* __restrict__ q_mu, int64_t ldq, int K, bf16x8* __restrict__ Afr, float* __restrict__ stats,
    int64_t lds_, float* __restrict__ Af32, int64_t lda, const float* __restrict__ a_var,
    const float* __restrict__ t_bound, const float* __restrict__ k_bound, int sidx = -1, int sbase = 0) {
  static_assert(KMAX <= 16, "the stats block has 16 rows");
  const int lane = threadIdx.x & 63, li = lane & 15, q = lane >> 4;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t i0 = 128 * (int64_t)t;
  const float a_scale = ldexpf(1.f, img_exp(sqrtf(*a_var)));
  // q_mu rows of the tile -> LDS [128][KMAX] and max |q_mu| (published by the main loop's barriers)
  if (stats) {
    float qmax = 0.f;
    for (int idx = threadIdx.x; idx < 128 * KMAX; idx += 256) {
      const int r = idx / KMAX, kk = idx % KMAX;
      const float qv = (i0 + r < M && kk < K) ? q_mu[(i0 + r) * ldq + kk] : 0.f;
      sQ[idx] = qv;
      qmax = fmaxf(qmax, fabsf(qv));
    }
    qmax = wave_max_f32(qmax);
    if (lane == 0) atomicMax(reinterpret_cast<unsigned int*>(sQ + 128 * KMAX), __float_as_uint(qmax));
  }
  floatx4v acc[8][4];
  x6_mainloop16<2, 2, true>(acc, sL, img_rsrc(Tfr, tfr_bytes), (uint32_t)(4 * t * nmk) * 3u * kFragBytes,
                            img_rsrc(Kfr, kfr_bytes), (uint32_t)((8 * tn + 2 * w) * nmk) * 3u * kFragBytes, 0,
                            4 * t + 4, nmk);
  K4STAMP(sidx, sbase);
  {
    const float unscale = ldexpf(1.f, -(img_exp(*t_bound) + img_exp(*k_bound)));
#pragma unroll
    for (int ib = 0; ib < 8; ++ib)
#pragma unroll
      for (int cb = 0; cb < 4; ++cb)
#pragma unroll
        for (int e = 0; e < 4; ++e) acc[ib][cb][e] *= unscale;
  }
  if (Af32) store_acc16_f32(acc, Af32, lda, i0, (int64_t)tn * kX6BN, M, N);
  // A's image: fragment (column block 8 tn + 2 w + c, k-step 8 t + ib), lane position pos
  const bool lo_half = lane < 32;
  const int pos = lo_half ? li + 32 * q : 16 + li + 32 * (q - 2);
  if (!stats) {  // no stats: the image alone
#pragma unroll
    for (int ib = 0; ib < 8; ++ib)
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        float v[8];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          v[r] = acc[ib][2 * c][r];
          v[4 + r] = acc[ib][2 * c + 1][r];
          lane_half_swap(v[r], v[4 + r]);
        }
        store_split_f16(Afr + ((((int64_t)8 * tn + 2 * w + c) * nmk + 8 * t + ib) * 3) * 64 + pos, v, a_scale);
      }
    return;
  }
  // With the stats: every accumulator value is split once (x = a 2^e -> f16 hi, f16 lo,
  // packed two per dword) and both the image fragments and the stats products' B
  // operand are assembled from the packed halves (the image's lane-half exchange moves
  // packed halves); row-block pairs (ib0, ib0 + 1) = 64-row stats tile ib0 / 4.
  const int qe = img_exp(__uint_as_float(reinterpret_cast<const unsigned int*>(sQ)[128 * KMAX]));
  const float q_scale = ldexpf(1.f, qe), s_unscale = ldexpf(1.f, -(qe + img_exp(sqrtf(*a_var))));
  floatx4v sq[4];
  float a2[4];
#pragma unroll
  for (int pr4 = 0; pr4 < 4; ++pr4) {  // row blocks ib0 = 2 pr4, ib0 + 1
    const int ib0 = 2 * pr4, st2 = pr4 >> 1;
    if ((pr4 & 1) == 0) {
#pragma unroll
      for (int cb = 0; cb < 4; ++cb) {
        sq[cb] = floatx4v{0.f, 0.f, 0.f, 0.f};
        a2[cb] = 0.f;
      }
    }
    uint32_t hp[2][4][2], lp[2][4][2];  // [row block of the pair][column block][dword]
#pragma unroll
    for (int d = 0; d < 2; ++d)
#pragma unroll
      for (int cb = 0; cb < 4; ++cb)
#pragma unroll
        for (int h2 = 0; h2 < 2; ++h2) {
          const float a0 = acc[ib0 + d][cb][2 * h2], a1 = acc[ib0 + d][cb][2 * h2 + 1];
          a2[cb] = fmaf(a1, a1, fmaf(a0, a0, a2[cb]));
          const float x0 = a0 * a_scale, x1 = a1 * a_scale;
          const _Float16 h0 = (_Float16)x0, h1 = (_Float16)x1;
          const halfx2 hh = {h0, h1}, ll = {(_Float16)(x0 - (float)h0), (_Float16)(x1 - (float)h1)};
          hp[d][cb][h2] = __builtin_bit_cast(uint32_t, hh);
          lp[d][cb][h2] = __builtin_bit_cast(uint32_t, ll);
        }
    // the image fragments of row blocks ib0, ib0 + 1
#pragma unroll
    for (int d = 0; d < 2; ++d)
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        // lanes 0-31: (own block 2c, lane + 32's 2c); 32-63: (lane - 32's 2c + 1, own 2c + 1)
        uint32_t h0[2], h1[2], l0[2], l1[2];
#pragma unroll
        for (int h2 = 0; h2 < 2; ++h2) {
          h0[h2] = hp[d][2 * c][h2];
          h1[h2] = hp[d][2 * c + 1][h2];
          l0[h2] = lp[d][2 * c][h2];
          l1[h2] = lp[d][2 * c + 1][h2];
          lane_half_swap(h0[h2], h1[h2]);
          lane_half_swap(l0[h2], l1[h2]);
        }
        const u32x4v fh = u32x4v{h0[0], h0[1], h1[0], h1[1]};
        const u32x4v fl = u32x4v{l0[0], l0[1], l1[0], l1[1]};
        bf16x8* dst = Afr + ((((int64_t)8 * tn + 2 * w + c) * nmk + 8 * t + ib0 + d) * 3) * 64 + pos;
#if MGP_K4_STORE_NT   // streaming stores: fewer dirty L2 lines for the kernel boundary
        __builtin_nontemporal_store(__builtin_bit_cast(bf16x8, fh), dst);
        __builtin_nontemporal_store(__builtin_bit_cast(bf16x8, fl), dst + 64);
#else
        dst[0] = __builtin_bit_cast(bf16x8, fh);
        dst[64] = __builtin_bit_cast(bf16x8, fl);
#endif
      }
    // q_mu^T A of this row-block pair: B operand slot j = row 4q + j of block ib0 (j < 4),
    // row 4q + j - 4 of block ib0 + 1
    bf16x8 qf[3];
    {
      halfx8 qh, ql;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int row = 16 * ib0 + (j < 4 ? 4 * q + j : 16 + 4 * q + j - 4);
        const float x = (li < K ? sQ[row * KMAX + (li < KMAX ? li : 0)] : 0.f) * q_scale;
        const _Float16 xh = (_Float16)x;
        qh[j] = xh;
        ql[j] = (_Float16)(x - (float)xh);
      }
      qf[0] = __builtin_bit_cast(bf16x8, qh);
      qf[1] = __builtin_bit_cast(bf16x8, ql);
    }
#pragma unroll
    for (int cb = 0; cb < 4; ++cb) {
      const bf16x8 bf[3] = {__builtin_bit_cast(bf16x8, u32x4v{hp[0][cb][0], hp[0][cb][1], hp[1][cb][0], hp[1][cb][1]}),
                            __builtin_bit_cast(bf16x8, u32x4v{lp[0][cb][0], lp[0][cb][1], lp[1][cb][0], lp[1][cb][1]}),
                            bf16x8{}};
      sq[cb] = mfma16_fmt<2, true>(qf, bf, sq[cb]);
    }
    if ((pr4 & 1) == 1) {  // 64-row stats tile 2 t + st2 done
      const int64_t st = 2 * (int64_t)t + st2;
      if (64 * st < M) {
#pragma unroll
        for (int cb = 0; cb < 4; ++cb) {
          const int64_t n = (int64_t)tn * kX6BN + 64 * w + 16 * cb + li;
          float s_a2 = a2[cb] + lane_xor16(a2[cb]);
          s_a2 += lane_xor32(s_a2);
          if (n < N) {
            float* dst = stats + st * (K + 1) * lds_ + n;
            if (lane < 16) dst[0] = s_a2;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              const int kk = 4 * q + e;
              if (kk < K) dst[(int64_t)(1 + kk) * lds_] = sq[cb][e] * s_unscale;
            }
          }
        }
      }
    }
  }
}

// Row-tile pairs as trsm_stats_x6_kernel (equal work per workgroup).
template <int KMAX>
__global__ __launch_bounds__(256, 2) void trsm_stats16_kernel(
    const bf16x8* __restrict__ Tfr, uint32_t tfr_bytes, const bf16x8* __restrict__ Kfr, uint32_t kfr_bytes,
    int nmk, int nTn, int64_t M, int64_t N, const float* __restrict__ q_mu, int64_t ldq, int K,
    bf16x8* __restrict__ Afr, float* __restrict__ stats, int64_t lds_, float* __restrict__ Af32, int64_t lda,
    const float* __restrict__ a_var, float* __restrict__ a_bound, const float* __restrict__ t_bound,
    const float* __restrict__ k_bound) {
  __shared__ bf16x8 sL[2][4 * 2 * 3 * 64];
  __shared__ float sQ[128 * KMAX + 1];
  const int nT = nmk / 8, nP = (nT + 1) / 2;
  int p, tn;
  if (blockIdx.x == 0 && threadIdx.x == 0) *a_bound = sqrtf(*a_var);
  col_major_item(blockIdx.x, nP, nTn, p, tn);
  const int it = blockIdx.x;  // debug stamps only
  K4STAMP(it, 0);
  if (threadIdx.x == 0) sQ[128 * KMAX] = 0.f;
  __syncthreads();
  trsm_stats16_item<KMAX>(sL, sQ, nT - 1 - p, tn, Tfr, tfr_bytes, Kfr, kfr_bytes, nmk, M, N, q_mu, ldq, K, Afr, stats,
                          lds_, Af32, lda, a_var, t_bound, k_bound, it, 1);
  K4STAMP(it, 2);
  if (nT - 1 - p == p) return;
  __syncthreads();
  if (threadIdx.x == 0) sQ[128 * KMAX] = 0.f;
  __syncthreads();
  trsm_stats16_item<KMAX>(sL, sQ, p, tn, Tfr, tfr_bytes, Kfr, kfr_bytes, nmk, M, N, q_mu, ldq, K, Afr, stats, lds_,
                          Af32, lda, a_var, t_bound, k_bound, it, 3);
  K4STAMP(it, 4);
}

// One layer's operands of the batched K4 (both SMGP layers share M, N and K).
struct K4Layer {
  const bf16x8* Tfr;
  const bf16x8* Kfr;
  const float* q_mu;
  bf16x8* Afr;
  float* stats;
  float* Af32;
  const float* a_var;
  float* a_bound;
  const float* t_bound;
  const float* k_bound;
  int64_t ldq, lds, lda;
};

// trsm_stats16_kernel over two layers in one launch: workgroups [0, per) run layer 0's
// items, [per, 2 per) layer 1's, each exactly as the one-layer kernel does (same items,
// same arithmetic: bit-identical images and statistics).  One launch instead of two
// drops a dispatch round boundary and a kernel tail between the layers.
template <int KMAX>
__global__ __launch_bounds__(256, 2) void trsm_stats16_pair_kernel(K4Layer l0, K4Layer l1, int per,
                                                                  uint32_t tfr_bytes, uint32_t kfr_bytes, int nmk,
                                                                  int nTn, int64_t M, int64_t N, int K) {
  __shared__ bf16x8 sL[2][4 * 2 * 3 * 64];
  __shared__ float sQ[128 * KMAX + 1];
  const bool second = (int)blockIdx.x >= per;
  const K4Layer& l = second ? l1 : l0;
  const int bid = (int)blockIdx.x - (second ? per : 0);
  const int nT = nmk / 8, nP = (nT + 1) / 2;
  int p, tn;
  if (bid == 0 && threadIdx.x == 0) *l.a_bound = sqrtf(*l.a_var);
  col_major_item(bid, nP, nTn, p, tn);
  if (threadIdx.x == 0) sQ[128 * KMAX] = 0.f;
  __syncthreads();
  trsm_stats16_item<KMAX>(sL, sQ, nT - 1 - p, tn, l.Tfr, tfr_bytes, l.Kfr, kfr_bytes, nmk, M, N, l.q_mu, l.ldq, K,
                          l.Afr, l.stats, l.lds, l.Af32, l.lda, l.a_var, l.t_bound, l.k_bound);
  if (nT - 1 - p == p) return;
  __syncthreads();
  if (threadIdx.x == 0) sQ[128 * KMAX] = 0.f;
  __syncthreads();
  trsm_stats16_item<KMAX>(sL, sQ, p, tn, l.Tfr, tfr_bytes, l.Kfr, kfr_bytes, nmk, M, N, l.q_mu, l.ldq, K, l.Afr,
                          l.stats, l.lds, l.Af32, l.lda, l.a_var, l.t_bound, l.k_bound);
}

}  // namespace mgp

using namespace mgp;

static int64_t x6_mp(int64_t M) { return (M + kX6BM - 1) / kX6BM * kX6BM; }
static int64_t x6_np(int64_t N) { return (N + kX6BN - 1) / kX6BN * kX6BN; }

// Image = fragment planes + a 256-byte trailer whose first float is the
// split-f16 scale bound (unused by split-bf16 images).
constexpr size_t kTrailer = 256;
static size_t lower_planes(int64_t M, int32_t K) {
  const int64_t Mp = x6_mp(M);
  return (size_t)K * (size_t)(Mp / 32) * (size_t)(Mp / 16) * 3 * kFragBytes;
}
static size_t cols_planes(int64_t M, int64_t N) {
  return (size_t)(x6_np(N) / 32) * (size_t)(x6_mp(M) / 16) * 3 * kFragBytes;
}
static float* trailer(void* img, size_t planes) { return (float*)((char*)img + planes); }

extern "C" size_t mgp_x6_lower_bytes(int64_t M, int32_t K) {
  if (M <= 0 || K <= 0) return 0;
  return lower_planes(M, K) + kTrailer;
}

extern "C" size_t mgp_x6_cols_bytes(int64_t M, int64_t N) {
  if (M <= 0 || N <= 0) return 0;
  return cols_planes(M, N) + kTrailer;
}

extern "C" int mgp_split_lower_x6(const float* q_sqrt, int64_t ldqs, int64_t strideq, int64_t M, int32_t K,
                                  void* Lfr, size_t lfr_bytes, mgp_stream_t stream) {
  if (!q_sqrt) return -1;
  if (ldqs < M) return -2;
  if (K > 1 && strideq < ldqs * M) return -3;
  if (M < 0) return -4;
  if (K < 0) return -5;
  if (!Lfr) return -6;
  if (M == 0 || K == 0) return MGP_OK;
  if (lfr_bytes < mgp_x6_lower_bytes(M, K)) return MGP_ERR_WORKSPACE;
  if (!aligned16(Lfr)) return MGP_ERR_ALIGN;
  const int64_t Mp = x6_mp(M);
  const int nmb = (int)(Mp / 32), nmk = (int)(Mp / 16);
  const int64_t nfrag = (int64_t)K * nmb * nmk;
  hipLaunchKernelGGL(split_tri_kernel<true>, dim3((unsigned)((nfrag + 3) / 4)), dim3(256), 0,
                     (hipStream_t)stream, q_sqrt, ldqs, strideq, M, nmb, nmk, nfrag, (bf16x8*)Lfr);
  return launch_status();
}

extern "C" int mgp_split_upper_x6(const float* LinvT, int64_t ldl, int64_t M, void* Tfr, size_t tfr_bytes,
                                  mgp_stream_t stream) {
  if (!LinvT) return -1;
  if (ldl < M) return -2;
  if (M < 0) return -3;
  if (!Tfr) return -4;
  if (M == 0) return MGP_OK;
  if (tfr_bytes < mgp_x6_lower_bytes(M, 1)) return MGP_ERR_WORKSPACE;
  if (!aligned16(Tfr)) return MGP_ERR_ALIGN;
  const int64_t Mp = x6_mp(M);
  const int nmb = (int)(Mp / 32), nmk = (int)(Mp / 16);
  const int64_t nfrag = (int64_t)nmb * nmk;
  hipLaunchKernelGGL(split_tri_kernel<false>, dim3((unsigned)((nfrag + 3) / 4)), dim3(256), 0,
                     (hipStream_t)stream, LinvT, ldl, (int64_t)0, M, nmb, nmk, nfrag, (bf16x8*)Tfr);
  return launch_status();
}

extern "C" int mgp_split_cols_x6(const float* A, int64_t lda, int64_t M, int64_t N, void* Afr,
                                 size_t afr_bytes, mgp_stream_t stream) {
  if (!A) return -1;
  if (lda < N) return -2;
  if (M < 0) return -3;
  if (N < 0) return -4;
  if (!Afr) return -5;
  if (M == 0 || N == 0) return MGP_OK;
  if (afr_bytes < mgp_x6_cols_bytes(M, N)) return MGP_ERR_WORKSPACE;
  if (!aligned16(Afr)) return MGP_ERR_ALIGN;
  const int nmk = (int)(x6_mp(M) / 16);
  const int64_t nfrag = (x6_np(N) / 32) * nmk;
  hipLaunchKernelGGL(split_cols_kernel, dim3((unsigned)((nfrag + 3) / 4)), dim3(256), 0, (hipStream_t)stream,
                     A, lda, M, N, nmk, nfrag, (bf16x8*)Afr);
  return launch_status();
}

extern "C" size_t mgp_expert_x6_workspace_bytes(int64_t M, int64_t N, int32_t K) {
  if (M <= 0 || N <= 0 || K <= 0) return 16;
  return (size_t)K * (size_t)(x6_mp(M) / kX6BM) * (size_t)((N + 3) / 4 * 4) * sizeof(float);
}

// Argument checks report the index in mgp_expert_conditional_x6's signature.
static int expert_cond_planes(const void* Afr, size_t afr_bytes, const void* Lfr, size_t lfr_bytes,
                              const float* stats, int64_t lds, const float* variance, int64_t M, int64_t N,
                              int32_t K, int planes, float* fmean, float* fvar, int64_t ldf, void* workspace,
                              size_t workspace_bytes, mgp_stream_t stream, bool f16 = false,
                              bool x8 = false, void* Cfr = nullptr, size_t cfr_bytes = 0,
                              const float* colmax = nullptr) {
  if (!Afr) return -1;
  if (afr_bytes < mgp_x6_cols_bytes(M, N)) return -2;
  if (!Lfr) return -3;
  if (lfr_bytes < mgp_x6_lower_bytes(M, K)) return -4;
  if (!stats) return -5;
  if (lds < N) return -6;
  if (!variance) return -7;
  if (M < 0) return -8;
  if (N < 0) return -9;
  if (K < 1) return -10;
  if (!fmean) return -11;
  if (!fvar) return -12;
  if (ldf < N) return -13;
  if (!aligned16(Afr) || !aligned16(Lfr)) return MGP_ERR_ALIGN;
  if (afr_bytes >= ((size_t)1 << 32) || lfr_bytes >= ((size_t)1 << 32)) return MGP_ERR_UNSUPPORTED;
  if (M == 0 || N == 0) return MGP_OK;
  if (!workspace || workspace_bytes < mgp_expert_x6_workspace_bytes(M, N, K)) return MGP_ERR_WORKSPACE;
  hipStream_t s = (hipStream_t)stream;
  const int64_t Mp = x6_mp(M);
  const int nmk = (int)(Mp / 16), nmb = (int)(Mp / 32), nTp = (int)(Mp / kX6BM);
  const int nTn = (int)(x6_np(N) / kX6BN);
  const int64_t ldp = (N + 3) / 4 * 4;
  float* part = (float*)workspace;
  const dim3 grid((unsigned)(K * nTp * nTn));
  const float* a_bound = trailer(const_cast<void*>(Afr), cols_planes(M, N));
  const float* l_bound = trailer(const_cast<void*>(Lfr), lower_planes(M, K));
#define MGP_K5_CASE(NP, F16, X8)                                                                        \
  if (planes == NP && f16 == F16 && x8 == X8)                                                           \
    hipLaunchKernelGGL((expert_cond_x6_kernel<NP, F16, X8>), grid, dim3(256), 0, s, (const bf16x8*)Afr, \
                       (const bf16x8*)Lfr, (uint32_t)mgp_x6_cols_bytes(M, N),                           \
                       (uint32_t)mgp_x6_lower_bytes(M, K), nmk, nmb, nTn, K, N, part, ldp, a_bound,     \
                       l_bound);
  if (Cfr) {  // training: + the C_k images (mgp_expert_conditional_f16c)
    if (!f16 || x8 || planes != 2) return MGP_ERR_UNSUPPORTED;
    if (!colmax) return -18;
    const size_t cexp = cols_planes(M, N);
    if (cfr_bytes < (size_t)K * cexp) return -17;
    if (!aligned16(Cfr)) return MGP_ERR_ALIGN;
    hipLaunchKernelGGL((expert_cond16_kernel<true>), grid, dim3(256), 0, s, (const bf16x8*)Afr, (const bf16x8*)Lfr,
                       (uint32_t)mgp_x6_cols_bytes(M, N), (uint32_t)mgp_x6_lower_bytes(M, K), nmk, nmb, nTn, K, N,
                       part, ldp, a_bound, l_bound, (bf16x8*)Cfr, (int64_t)(cexp / 16), colmax);
  } else if (planes == 2 && f16 && !x8) {  // the split-f16 forward K5 (16x16x32 MFMA)
    hipLaunchKernelGGL((expert_cond16_kernel<false>), grid, dim3(256), 0, s, (const bf16x8*)Afr, (const bf16x8*)Lfr,
                       (uint32_t)mgp_x6_cols_bytes(M, N), (uint32_t)mgp_x6_lower_bytes(M, K), nmk, nmb, nTn, K, N,
                       part, ldp, a_bound, l_bound);
  } else {
  MGP_K5_CASE(3, false, false)
  MGP_K5_CASE(2, false, false)
  MGP_K5_CASE(1, false, false)
  MGP_K5_CASE(2, true, true)
  }
#undef MGP_K5_CASE
  int st = launch_status();
  if (st) return st;
  return mgp_launch_cond_finalize(stats, lds, mgp_stats_tiles(M), part, ldp, nTp, variance, N, K, fmean, fvar,
                                  ldf, s);
}

extern "C" int mgp_expert_conditional_x6(const void* Afr, size_t afr_bytes, const void* Lfr, size_t lfr_bytes,
                                         const float* stats, int64_t lds, const float* variance, int64_t M,
                                         int64_t N, int32_t K, float* fmean, float* fvar, int64_t ldf,
                                         void* workspace, size_t workspace_bytes, mgp_stream_t stream) {
  return expert_cond_planes(Afr, afr_bytes, Lfr, lfr_bytes, stats, lds, variance, M, N, K, 3, fmean, fvar, ldf,
                            workspace, workspace_bytes, stream);
}

extern "C" int mgp_expert_conditional_planes(const void* Afr, size_t afr_bytes, const void* Lfr, size_t lfr_bytes,
                                             const float* stats, int64_t lds, const float* variance, int64_t M,
                                             int64_t N, int32_t K, int32_t planes, float* fmean, float* fvar,
                                             int64_t ldf, void* workspace, size_t workspace_bytes,
                                             mgp_stream_t stream) {
  if (planes < 1 || planes > 3) return -11;
  const int st = expert_cond_planes(Afr, afr_bytes, Lfr, lfr_bytes, stats, lds, variance, M, N, K, planes, fmean,
                                    fvar, ldf, workspace, workspace_bytes, stream);
  return (st <= -11 && st >= -13) ? st - 1 : st;  // fmean, fvar, ldf follow `planes` here
}

template <int KMAX>
static int launch_trsm_x6(const void* Tfr, size_t tb, const void* Kfr, size_t kb, int64_t M, int64_t N,
                          const float* q_mu, int64_t ldq, int K, void* Afr, float* stats, int64_t lds,
                          float* A, int64_t lda, hipStream_t s, const float* a_var = nullptr,
                          bool f16in = false, bool x8 = false) {
  const int64_t Mp = x6_mp(M);
  const int nmk = (int)(Mp / 16), nT = (int)(Mp / kX6BM), nTn = (int)(x6_np(N) / kX6BN);
  const dim3 grid((unsigned)((nT + 1) / 2 * nTn));
  float* a_bound = trailer(Afr, cols_planes(M, N));
  if (f16in) {
    const float* t_bound = trailer(const_cast<void*>(Tfr), lower_planes(M, 1));
    const float* k_bound = trailer(const_cast<void*>(Kfr), cols_planes(M, N));
    if (x8)
      hipLaunchKernelGGL((trsm_stats_x6_kernel<KMAX, true, true, true>), grid, dim3(256), 0, s, (const bf16x8*)Tfr,
                         (uint32_t)tb, (const bf16x8*)Kfr, (uint32_t)kb, nmk, nTn, M, N, q_mu, ldq, K,
                         (bf16x8*)Afr, stats, lds, A, lda, a_var, a_bound, t_bound, k_bound);
    else
      hipLaunchKernelGGL((trsm_stats16_kernel<KMAX>), grid, dim3(256), 0, s, (const bf16x8*)Tfr, (uint32_t)tb,
                         (const bf16x8*)Kfr, (uint32_t)kb, nmk, nTn, M, N, q_mu, ldq, K, (bf16x8*)Afr, stats, lds, A,
                         lda, a_var, a_bound, t_bound, k_bound);
  } else if (a_var)
    hipLaunchKernelGGL((trsm_stats_x6_kernel<KMAX, true>), grid, dim3(256), 0, s, (const bf16x8*)Tfr,
                       (uint32_t)tb, (const bf16x8*)Kfr, (uint32_t)kb, nmk, nTn, M, N, q_mu, ldq, K,
                       (bf16x8*)Afr, stats, lds, A, lda, a_var, a_bound);
  else
    hipLaunchKernelGGL((trsm_stats_x6_kernel<KMAX, false>), grid, dim3(256), 0, s, (const bf16x8*)Tfr,
                       (uint32_t)tb, (const bf16x8*)Kfr, (uint32_t)kb, nmk, nTn, M, N, q_mu, ldq, K,
                       (bf16x8*)Afr, stats, lds, A, lda, a_var, a_bound);
  return launch_status();
}

extern "C" int mgp_trsm_stats_x6(const void* Tfr, size_t tfr_bytes, const void* Kfr, size_t kfr_bytes,
                                 int64_t M, int64_t N, const float* q_mu, int64_t ldq, int32_t K,
                                 void* Afr, size_t afr_bytes, float* stats, int64_t lds, float* A,
                                 int64_t lda, mgp_stream_t stream) {
  if (!Tfr) return -1;
  if (tfr_bytes < mgp_x6_lower_bytes(M, 1)) return -2;
  if (!Kfr) return -3;
  if (kfr_bytes < mgp_x6_cols_bytes(M, N)) return -4;
  if (M < 0) return -5;
  if (N < 0) return -6;
  if (!q_mu) return -7;
  if (ldq < K) return -8;
  if (K < 1) return -9;
  if (K > 16) return MGP_ERR_UNSUPPORTED;
  if (!Afr) return -10;
  if (afr_bytes < mgp_x6_cols_bytes(M, N)) return -11;
  if (stats && lds < N) return -13;
  if (A && lda < N) return -15;
  if (!aligned16(Tfr) || !aligned16(Kfr) || !aligned16(Afr)) return MGP_ERR_ALIGN;
  if (mgp_x6_cols_bytes(M, N) >= ((size_t)1 << 32) || mgp_x6_lower_bytes(M, 1) >= ((size_t)1 << 32))
    return MGP_ERR_UNSUPPORTED;
  if (M == 0 || N == 0) return MGP_OK;
  hipStream_t s = (hipStream_t)stream;
  const size_t tb = mgp_x6_lower_bytes(M, 1), kb = mgp_x6_cols_bytes(M, N);
  if (K <= 4) return launch_trsm_x6<4>(Tfr, tb, Kfr, kb, M, N, q_mu, ldq, K, Afr, stats, lds, A, lda, s);
  if (K <= 8) return launch_trsm_x6<8>(Tfr, tb, Kfr, kb, M, N, q_mu, ldq, K, Afr, stats, lds, A, lda, s);
  return launch_trsm_x6<16>(Tfr, tb, Kfr, kb, M, N, q_mu, ldq, K, Afr, stats, lds, A, lda, s);
}

// ------------------------------------------------------------------ split-f16 ("f16x3") K5 path
static int trsm_stats_f16_out(const void* Tfr, size_t tfr_bytes, const void* Kfr, size_t kfr_bytes, int64_t M,
                              int64_t N, const float* q_mu, int64_t ldq, int32_t K, const float* variance, void* Afr,
                              size_t afr_bytes, float* stats, int64_t lds, mgp_stream_t stream, bool f16in,
                              float* A = nullptr, int64_t lda = 0, bool x8 = false) {
  if (!Tfr) return -1;
  if (tfr_bytes < mgp_x6_lower_bytes(M, 1)) return -2;
  if (!Kfr) return -3;
  if (kfr_bytes < mgp_x6_cols_bytes(M, N)) return -4;
  if (M < 0) return -5;
  if (N < 0) return -6;
  if (!q_mu) return -7;
  if (ldq < K) return -8;
  if (K < 1) return -9;
  if (K > 16) return MGP_ERR_UNSUPPORTED;
  if (!variance) return -10;
  if (!Afr) return -11;
  if (afr_bytes < mgp_x6_cols_bytes(M, N)) return -12;
  if (stats && lds < N) return -14;  // stats may be NULL (A image only)
  
  if (!aligned16(Tfr) || !aligned16(Kfr) || !aligned16(Afr)) return MGP_ERR_ALIGN;
  if (mgp_x6_cols_bytes(M, N) >= ((size_t)1 << 32) || mgp_x6_lower_bytes(M, 1) >= ((size_t)1 << 32))
    return MGP_ERR_UNSUPPORTED;
  if (M == 0 || N == 0) return MGP_OK;
  hipStream_t s = (hipStream_t)stream;
  const size_t tb = mgp_x6_lower_bytes(M, 1), kb = mgp_x6_cols_bytes(M, N);
  if (K <= 4)
    return launch_trsm_x6<4>(Tfr, tb, Kfr, kb, M, N, q_mu, ldq, K, Afr, stats, lds, A, lda, s, variance, f16in, x8);
  if (K <= 8)
    return launch_trsm_x6<8>(Tfr, tb, Kfr, kb, M, N, q_mu, ldq, K, Afr, stats, lds, A, lda, s, variance, f16in, x8);
  return launch_trsm_x6<16>(Tfr, tb, Kfr, kb, M, N, q_mu, ldq, K, Afr, stats, lds, A, lda, s, variance, f16in, x8);
}

// x6 images in (Tfr, Kfr), split-f16 A image out (K5's operand).
extern "C" int mgp_trsm_stats_x6_f16(const void* Tfr, size_t tfr_bytes, const void* Kfr, size_t kfr_bytes,
                                     int64_t M, int64_t N, const float* q_mu, int64_t ldq, int32_t K,
                                     const float* variance, void* Afr, size_t afr_bytes, float* stats,
                                     int64_t lds, mgp_stream_t stream) {
  return trsm_stats_f16_out(Tfr, tfr_bytes, Kfr, kfr_bytes, M, N, q_mu, ldq, K, variance, Afr, afr_bytes, stats, lds,
                            stream, false);
}

// split-f16 images in (mgp_split_upper_f16, mgp_rbf_kuf_f16) and out: three f16
// products per block instead of six bf16 ones.
extern "C" int mgp_trsm_stats_f16(const void* Tfr, size_t tfr_bytes, const void* Kfr, size_t kfr_bytes, int64_t M,
                                  int64_t N, const float* q_mu, int64_t ldq, int32_t K, const float* variance,
                                  void* Afr, size_t afr_bytes, float* stats, int64_t lds, float* A, int64_t lda,
                                  mgp_stream_t stream) {
  if (A && lda < N) return -16;
  return trsm_stats_f16_out(Tfr, tfr_bytes, Kfr, kfr_bytes, M, N, q_mu, ldq, K, variance, Afr, afr_bytes, stats, lds,
                            stream, true, A, lda);
}

// mgp_trsm_stats_f16 for `batch` (1 or 2) layers of equal M, N, K in one launch (the two
// SMGP layers' K4); the per-layer operands are host arrays of device pointers (A[b] may be
// NULL; A itself may be NULL: no f32 A for any layer).  Results are bit-identical to one
// mgp_trsm_stats_f16 call per layer.  Errors: the single call's codes for the first bad
// layer; -17 for a batch outside [1, 2].
extern "C" int mgp_trsm_stats_f16_batch(int32_t batch, const void* const* Tfr, size_t tfr_bytes,
                                        const void* const* Kfr, size_t kfr_bytes, int64_t M, int64_t N,
                                        const float* const* q_mu, int64_t ldq, int32_t K,
                                        const float* const* variance, void* const* Afr, size_t afr_bytes,
                                        float* const* stats, int64_t lds, float* const* A, int64_t lda,
                                        mgp_stream_t stream) {
  if (batch < 1 || batch > 2) return -17;
  if (!Tfr || !Kfr || !q_mu || !variance || !Afr || !stats) return -1;
  if (A && lda < N) return -16;
  for (int b = 0; b < batch; ++b) {
    if (!Tfr[b]) return -1;
    if (tfr_bytes < mgp_x6_lower_bytes(M, 1)) return -2;
    if (!Kfr[b]) return -3;
    if (kfr_bytes < mgp_x6_cols_bytes(M, N)) return -4;
    if (M < 0) return -5;
    if (N < 0) return -6;
    if (!q_mu[b]) return -7;
    if (ldq < K) return -8;
    if (K < 1) return -9;
    if (K > 16) return MGP_ERR_UNSUPPORTED;
    if (!variance[b]) return -10;
    if (!Afr[b]) return -11;
    if (afr_bytes < mgp_x6_cols_bytes(M, N)) return -12;
    if (!stats[b]) return -13;
    if (lds < N) return -14;
    if (!aligned16(Tfr[b]) || !aligned16(Kfr[b]) || !aligned16(Afr[b])) return MGP_ERR_ALIGN;
  }
  if (mgp_x6_cols_bytes(M, N) >= ((size_t)1 << 32) || mgp_x6_lower_bytes(M, 1) >= ((size_t)1 << 32))
    return MGP_ERR_UNSUPPORTED;
  if (M == 0 || N == 0) return MGP_OK;
  const size_t tb = mgp_x6_lower_bytes(M, 1), kb = mgp_x6_cols_bytes(M, N);
  const int64_t Mp = x6_mp(M);
  const int nmk = (int)(Mp / 16), nT = (int)(Mp / kX6BM), nTn = (int)(x6_np(N) / kX6BN);
  const int per = (nT + 1) / 2 * nTn;
  K4Layer l[2];
  for (int b = 0; b < 2; ++b) {
    const int s = b < batch ? b : 0;
    l[b] = K4Layer{(const bf16x8*)Tfr[s], (const bf16x8*)Kfr[s], q_mu[s], (bf16x8*)Afr[s], stats[s],
                   A ? A[s] : nullptr, variance[s], trailer(Afr[s], cols_planes(M, N)),
                   trailer(const_cast<void*>(Tfr[s]), lower_planes(M, 1)),
                   trailer(const_cast<void*>(Kfr[s]), cols_planes(M, N)), ldq, lds, lda};
  }
  const dim3 grid((unsigned)(per * batch));
  hipStream_t s = (hipStream_t)stream;
  if (K <= 4)
    hipLaunchKernelGGL(trsm_stats16_pair_kernel<4>, grid, dim3(256), 0, s, l[0], l[1], per, (uint32_t)tb,
                       (uint32_t)kb, nmk, nTn, M, N, (int)K);
  else if (K <= 8)
    hipLaunchKernelGGL(trsm_stats16_pair_kernel<8>, grid, dim3(256), 0, s, l[0], l[1], per, (uint32_t)tb,
                       (uint32_t)kb, nmk, nTn, M, N, (int)K);
  else
    hipLaunchKernelGGL(trsm_stats16_pair_kernel<16>, grid, dim3(256), 0, s, l[0], l[1], per, (uint32_t)tb,
                       (uint32_t)kb, nmk, nTn, M, N, (int)K);
  return launch_status();
}

// mgp_trsm_stats_f16 that also writes the A image's e4m3 cross-term plane (the
// operand of mgp_expert_conditional_f16x8).  With A == NULL the f16 lo plane is
// not written (only the f16x8 K5 reads that image).
extern "C" int mgp_trsm_stats_f16x8(const void* Tfr, size_t tfr_bytes, const void* Kfr, size_t kfr_bytes, int64_t M,
                                    int64_t N, const float* q_mu, int64_t ldq, int32_t K, const float* variance,
                                    void* Afr, size_t afr_bytes, float* stats, int64_t lds, float* A, int64_t lda,
                                    mgp_stream_t stream) {
  if (A && lda < N) return -16;
  return trsm_stats_f16_out(Tfr, tfr_bytes, Kfr, kfr_bytes, M, N, q_mu, ldq, K, variance, Afr, afr_bytes, stats, lds,
                            stream, true, A, lda, true);
}

// absmax of the source into the trailer, then the scaled split.
extern "C" int mgp_split_lower_f16(const float* q_sqrt, int64_t ldqs, int64_t strideq, int64_t M, int32_t K,
                                   void* Lfr, size_t lfr_bytes, mgp_stream_t stream) {
  if (!q_sqrt) return -1;
  if (ldqs < M) return -2;
  if (K > 1 && strideq < ldqs * M) return -3;
  if (M < 0) return -4;
  if (K < 0) return -5;
  if (!Lfr) return -6;
  if (M == 0 || K == 0) return MGP_OK;
  if (lfr_bytes < mgp_x6_lower_bytes(M, K)) return MGP_ERR_WORKSPACE;
  if (!aligned16(Lfr)) return MGP_ERR_ALIGN;
  hipStream_t s = (hipStream_t)stream;
  float* bound = trailer(Lfr, lower_planes(M, K));
  int st = hip_status(hipMemsetAsync(bound, 0, sizeof(float), s));
  if (st) return st;
  const int64_t rows = (int64_t)K * M;
  launch_absmax<1>(q_sqrt, ldqs, strideq, M, M, rows, bound, s);
  st = launch_status();
  if (st) return st;
  const int64_t Mp = x6_mp(M);
  const int nmb = (int)(Mp / 32), nmk = (int)(Mp / 16);
  const int64_t nfrag = (int64_t)K * nmb * nmk;
  hipLaunchKernelGGL(split_tri_kernel<true>, dim3((unsigned)((nfrag + 3) / 4)), dim3(256), 0, s, q_sqrt, ldqs,
                     strideq, M, nmb, nmk, nfrag, (bf16x8*)Lfr, (const float*)bound);
  return launch_status();
}

// Per layer: the KL partial sums [nblk][3] doubles, then the block maxima [nblk] floats.
static int64_t qsqrt_nblk(int64_t M, int32_t K) { return (int64_t)K * ((M + kKlRows - 1) / kKlRows) + 1; }

extern "C" size_t mgp_qsqrt_workspace_bytes(int64_t M, int32_t K) {
  if (M <= 0 || K <= 0) return 0;
  const int64_t n = qsqrt_nblk(M, K);
  return (size_t)((n * 3 * 8 + n * 4 + 15) / 16 * 16);
}

extern "C" int mgp_qsqrt_images_kl_f16_batch(int32_t batch, const float* const* q_mu, int64_t ldq,
                                             const float* const* q_sqrt, int64_t ldqs, int64_t strideq, int64_t M,
                                             int32_t K, void* const* Lfr, size_t lfr_bytes, double* const* kl_out,
                                             void* workspace, size_t workspace_bytes, mgp_stream_t stream) {
  if (batch < 1 || batch > 2) return -1;
  if (!q_mu) return -2;
  if (ldq < K) return -3;
  if (!q_sqrt) return -4;
  if (ldqs < M) return -5;
  if (K > 1 && strideq < ldqs * M) return -6;
  if (M < 1) return -7;
  if (K < 1) return -8;
  if (!Lfr) return -9;
  if (lfr_bytes < mgp_x6_lower_bytes(M, K)) return -10;
  if (!kl_out) return -11;
  if ((ldqs & 3) || (strideq & 3)) return MGP_ERR_ALIGN;   // the KL sums' float4 rows
  const size_t wb = mgp_qsqrt_workspace_bytes(M, K);
  if (!workspace || workspace_bytes < wb * (size_t)batch) return MGP_ERR_WORKSPACE;
  if (!aligned16(workspace)) return MGP_ERR_ALIGN;
  const int64_t nblk = qsqrt_nblk(M, K);
  QLayer l[2];
  for (int b = 0; b < 2; ++b) {
    const int s = b < batch ? b : 0;
    if (!q_mu[s]) return -2;
    if (!q_sqrt[s]) return -4;
    if (!Lfr[s]) return -9;
    if (!kl_out[s]) return -11;
    if (!aligned16(q_sqrt[s]) || !aligned16(Lfr[s])) return MGP_ERR_ALIGN;
    char* w = (char*)workspace + wb * (size_t)s;
    l[b] = QLayer{q_mu[s], q_sqrt[s], (bf16x8*)Lfr[s], trailer(Lfr[s], lower_planes(M, K)), kl_out[s],
                  (double*)w, (float*)(w + nblk * 3 * 8)};
  }
  hipStream_t st = (hipStream_t)stream;
  const int nrb = (int)((M + kKlRows - 1) / kKlRows);
  const int64_t kgrid = kQsGrid > 0 && nblk > kQsGrid ? kQsGrid : nblk;
  hipLaunchKernelGGL(kl_absmax2_kernel, dim3((unsigned)kgrid, (unsigned)batch), dim3(256), 0, st, l[0], l[1], ldq,
                     ldqs, strideq, M, K, nrb, (int)nblk);
  int rc = launch_status();
  if (rc) return rc;
  hipLaunchKernelGGL(kl_final2_kernel, dim3((unsigned)batch), dim3(1024), 0, st, l[0], l[1], (int)nblk,
                     (double)M * (double)K);
  rc = launch_status();
  if (rc) return rc;
  const int64_t Mp = x6_mp(M);
  const int nmb = (int)(Mp / 32), nmk = (int)(Mp / 16);
  const int64_t nfrag = (int64_t)K * nmb * nmk;
  const int64_t sgrid = kQsGrid > 0 && (nfrag + 3) / 4 > kQsGrid ? kQsGrid : (nfrag + 3) / 4;
  hipLaunchKernelGGL(split_lower2_kernel, dim3((unsigned)sgrid, (unsigned)batch), dim3(256), 0, st, l[0],
                     l[1], ldqs, strideq, M, nmb, nmk, nfrag);
  return launch_status();
}

// L^-T (upper triangle) as a split-f16 T image for mgp_trsm_stats_f16: absmax
// of the triangle into the trailer, then the scaled split.
extern "C" int mgp_split_upper_f16(const float* LinvT, int64_t ldl, int64_t M, void* Tfr, size_t tfr_bytes,
                                   mgp_stream_t stream) {
  if (!LinvT) return -1;
  if (ldl < M) return -2;
  if (M < 0) return -3;
  if (!Tfr) return -4;
  if (M == 0) return MGP_OK;
  if (tfr_bytes < mgp_x6_lower_bytes(M, 1)) return MGP_ERR_WORKSPACE;
  if (!aligned16(Tfr)) return MGP_ERR_ALIGN;
  hipStream_t s = (hipStream_t)stream;
  float* bound = trailer(Tfr, lower_planes(M, 1));
  int st = hip_status(hipMemsetAsync(bound, 0, sizeof(float), s));
  if (st) return st;
  launch_absmax<2>(LinvT, ldl, (int64_t)0, M, M, M, bound, s);
  st = launch_status();
  if (st) return st;
  const int64_t Mp = x6_mp(M);
  const int nmb = (int)(Mp / 32), nmk = (int)(Mp / 16);
  const int64_t nfrag = (int64_t)nmb * nmk;
  hipLaunchKernelGGL(split_tri_kernel<false>, dim3((unsigned)((nfrag + 3) / 4)), dim3(256), 0, s, LinvT, ldl,
                     (int64_t)0, M, nmb, nmk, nfrag, (bf16x8*)Tfr, (const float*)bound);
  return launch_status();
}

// mgp_split_upper_f16 whose trailer already holds max |LinvT| (written by
// mgp_kuu_potrf_trtri_ex into mgp_x6_bound_ptr(Tfr)): the split alone.
extern "C" int mgp_split_upper_f16_bounded(const float* LinvT, int64_t ldl, int64_t M, void* Tfr, size_t tfr_bytes,
                                           mgp_stream_t stream) {
  if (!LinvT) return -1;
  if (ldl < M) return -2;
  if (M < 0) return -3;
  if (!Tfr) return -4;
  if (M == 0) return MGP_OK;
  if (tfr_bytes < mgp_x6_lower_bytes(M, 1)) return MGP_ERR_WORKSPACE;
  if (!aligned16(Tfr)) return MGP_ERR_ALIGN;
  const int64_t Mp = x6_mp(M);
  const int nmb = (int)(Mp / 32), nmk = (int)(Mp / 16);
  const int64_t nfrag = (int64_t)nmb * nmk;
  const float* bound = trailer(Tfr, lower_planes(M, 1));
  hipLaunchKernelGGL(split_tri_kernel<false>, dim3((unsigned)((nfrag + 3) / 4)), dim3(256), 0, (hipStream_t)stream,
                     LinvT, ldl, (int64_t)0, M, nmb, nmk, nfrag, (bf16x8*)Tfr, bound);
  return launch_status();
}

// mgp_split_upper_f16_bounded for `batch` (1 or 2) matrices at LinvT + b strideL into the
// images Tfr[b] (host array of device pointers) in one launch; bit-identical.
extern "C" int mgp_split_upper_f16_bounded_batch(int32_t batch, const float* LinvT, int64_t ldl, int64_t strideL,
                                                 int64_t M, void* const* Tfr, size_t tfr_bytes,
                                                 mgp_stream_t stream) {
  if (batch < 1 || batch > 2) return -9;   // its own code (-1 .. -8 name the arguments)
  if (!LinvT) return -2;
  if (ldl < M) return -3;
  if (batch > 1 && strideL < ldl * M) return -4;
  if (M < 0) return -5;
  if (!Tfr) return -6;
  for (int b = 0; b < batch; ++b) {
    if (!Tfr[b]) return -6;
    if (!aligned16(Tfr[b])) return MGP_ERR_ALIGN;
  }
  if (M == 0) return MGP_OK;
  if (tfr_bytes < mgp_x6_lower_bytes(M, 1)) return MGP_ERR_WORKSPACE;
  const int64_t Mp = x6_mp(M);
  const int nmb = (int)(Mp / 32), nmk = (int)(Mp / 16);
  const int64_t nfrag = (int64_t)nmb * nmk;
  void* t1 = Tfr[batch - 1];
  hipLaunchKernelGGL(split_upper2_kernel, dim3((unsigned)((nfrag + 3) / 4), (unsigned)batch), dim3(256), 0,
                     (hipStream_t)stream, LinvT, ldl, strideL, M, nmb, nmk, nfrag, (bf16x8*)Tfr[0],
                     (const float*)trailer(Tfr[0], lower_planes(M, 1)), (bf16x8*)t1,
                     (const float*)trailer(t1, lower_planes(M, 1)));
  return launch_status();
}

// Device address of the split-f16 scale bound in an image's trailer (lower /
// upper images: K = matrices in the batch; column images: K = 0, N columns).
extern "C" float* mgp_x6_bound_ptr(void* img, int64_t M, int64_t N, int32_t K) {
  if (!img || M <= 0) return nullptr;
  return trailer(img, K > 0 ? lower_planes(M, K) : cols_planes(M, N));
}

extern "C" int mgp_split_cols_f16(const float* A, int64_t lda, int64_t M, int64_t N, void* Afr,
                                  size_t afr_bytes, mgp_stream_t stream) {
  if (!A) return -1;
  if (lda < N) return -2;
  if (M < 0) return -3;
  if (N < 0) return -4;
  if (!Afr) return -5;
  if (M == 0 || N == 0) return MGP_OK;
  if (afr_bytes < mgp_x6_cols_bytes(M, N)) return MGP_ERR_WORKSPACE;
  if (!aligned16(Afr)) return MGP_ERR_ALIGN;
  hipStream_t s = (hipStream_t)stream;
  float* bound = trailer(Afr, cols_planes(M, N));
  int st = hip_status(hipMemsetAsync(bound, 0, sizeof(float), s));
  if (st) return st;
  launch_absmax<0>(A, lda, (int64_t)0, M, N, M, bound, s);
  st = launch_status();
  if (st) return st;
  const int nmk = (int)(x6_mp(M) / 16);
  const int64_t nfrag = (x6_np(N) / 32) * nmk;
  hipLaunchKernelGGL(split_cols_kernel, dim3((unsigned)((nfrag + 3) / 4)), dim3(256), 0, s, A, lda, M, N, nmk,
                     nfrag, (bf16x8*)Afr, (const float*)bound);
  return launch_status();
}

extern "C" int mgp_expert_conditional_f16(const void* Afr, size_t afr_bytes, const void* Lfr, size_t lfr_bytes,
                                          const float* stats, int64_t lds, const float* variance, int64_t M,
                                          int64_t N, int32_t K, float* fmean, float* fvar, int64_t ldf,
                                          void* workspace, size_t workspace_bytes, mgp_stream_t stream) {
  return expert_cond_planes(Afr, afr_bytes, Lfr, lfr_bytes, stats, lds, variance, M, N, K, 2, fmean, fvar, ldf,
                            workspace, workspace_bytes, stream, true);
}

// Training: mgp_expert_conditional_f16 that also writes C_k = L_k^T A per expert as a
// split-f16 B-layout image (Cfr, mgp_c_images_bytes; colmax from mgp_colnorm_max
// of q_sqrt), consumed by mgp_conditional_backward_f16c.
extern "C" size_t mgp_c_images_bytes(int64_t M, int64_t N, int32_t K) {
  if (M <= 0 || N <= 0 || K <= 0) return 16;
  return (size_t)K * cols_planes(M, N);
}

extern "C" int mgp_colnorm_max(const float* q_sqrt, int64_t ldq, int64_t strideq, int64_t M, int32_t K,
                               float* out, mgp_stream_t stream) {
  if (!q_sqrt) return -1;
  if (ldq < M) return -2;
  if (M < 0) return -4;
  if (K < 1) return -5;
  if (!out) return -6;
  hipStream_t s = (hipStream_t)stream;
  int st = hip_status(hipMemsetAsync(out, 0, sizeof(float), s));
  if (st || M == 0) return st;
  hipLaunchKernelGGL(colnorm_max_kernel, dim3((unsigned)((M + 31) / 32), (unsigned)K), dim3(256), 0, s, q_sqrt, ldq,
                     strideq, M, (unsigned int*)out);
  return launch_status();
}

extern "C" int mgp_expert_conditional_f16c(const void* Afr, size_t afr_bytes, const void* Lfr, size_t lfr_bytes,
                                           const float* stats, int64_t lds, const float* variance, int64_t M,
                                           int64_t N, int32_t K, float* fmean, float* fvar, int64_t ldf,
                                           void* workspace, size_t workspace_bytes, void* Cfr, size_t cfr_bytes,
                                           const float* colmax, mgp_stream_t stream) {
  if (!Cfr) return -16;
  return expert_cond_planes(Afr, afr_bytes, Lfr, lfr_bytes, stats, lds, variance, M, N, K, 2, fmean, fvar, ldf,
                            workspace, workspace_bytes, stream, true, false, Cfr, cfr_bytes, colmax);
}

// mgp_expert_conditional_f16 (Cfr == NULL) or mgp_expert_conditional_f16c (Cfr, colmax:
// host arrays of device pointers) for `batch` (1 or 2) layers of equal M, N, K: one K5
// launch over both layers, then each layer's finalize.  Per-layer operands are host arrays
// of device pointers, one workspace per layer.  Bit-identical to one call per layer.
// Errors: the single call's codes for the first bad layer; -20 for a batch outside [1, 2].
extern "C" int mgp_expert_conditional_f16_batch(int32_t batch, const void* const* Afr, size_t afr_bytes,
                                                const void* const* Lfr, size_t lfr_bytes, const float* const* stats,
                                                int64_t lds, const float* const* variance, int64_t M, int64_t N,
                                                int32_t K, float* const* fmean, float* const* fvar, int64_t ldf,
                                                void* const* workspace, size_t workspace_bytes,
                                                void* const* Cfr, size_t cfr_bytes, const float* const* colmax,
                                                mgp_stream_t stream) {
  if (batch < 1 || batch > 2) return -20;
  if (!Afr || !Lfr || !stats || !variance || !fmean || !fvar || !workspace) return -1;
  const size_t cexp = cols_planes(M, N);
  for (int b = 0; b < batch; ++b) {
    if (!Afr[b]) return -1;
    if (afr_bytes < mgp_x6_cols_bytes(M, N)) return -2;
    if (!Lfr[b]) return -3;
    if (lfr_bytes < mgp_x6_lower_bytes(M, K)) return -4;
    if (!stats[b]) return -5;
    if (lds < N) return -6;
    if (!variance[b]) return -7;
    if (M < 0) return -8;
    if (N < 0) return -9;
    if (K < 1) return -10;
    if (!fmean[b]) return -11;
    if (!fvar[b]) return -12;
    if (ldf < N) return -13;
    if (!aligned16(Afr[b]) || !aligned16(Lfr[b])) return MGP_ERR_ALIGN;
    if (M > 0 && N > 0 && (!workspace[b] || workspace_bytes < mgp_expert_x6_workspace_bytes(M, N, K)))
      return MGP_ERR_WORKSPACE;
    if (Cfr) {
      if (!Cfr[b]) return -16;
      if (cfr_bytes < (size_t)K * cexp) return -17;
      if (!colmax || !colmax[b]) return -18;
      if (!aligned16(Cfr[b])) return MGP_ERR_ALIGN;
    }
  }
  if (afr_bytes >= ((size_t)1 << 32) || lfr_bytes >= ((size_t)1 << 32)) return MGP_ERR_UNSUPPORTED;
  if (M == 0 || N == 0) return MGP_OK;
  hipStream_t s = (hipStream_t)stream;
  const int64_t Mp = x6_mp(M);
  const int nmk = (int)(Mp / 16), nmb = (int)(Mp / 32), nTp = (int)(Mp / kX6BM);
  const int nTn = (int)(x6_np(N) / kX6BN);
  const int64_t ldp = (N + 3) / 4 * 4;
  const int per = K * nTp * nTn;
  K5Layer l[2];
  for (int b = 0; b < 2; ++b) {
    const int q = b < batch ? b : 0;
    l[b] = K5Layer{(const bf16x8*)Afr[q], (const bf16x8*)Lfr[q], (float*)workspace[q],
                   trailer(const_cast<void*>(Afr[q]), cols_planes(M, N)),
                   trailer(const_cast<void*>(Lfr[q]), lower_planes(M, K)), Cfr ? (bf16x8*)Cfr[q] : nullptr,
                   Cfr ? colmax[q] : nullptr};
  }
  const dim3 grid((unsigned)(per * batch));
  const uint32_t ab = (uint32_t)mgp_x6_cols_bytes(M, N), lb = (uint32_t)mgp_x6_lower_bytes(M, K);
  if (Cfr)
    hipLaunchKernelGGL(expert_cond16_pair_kernel<true>, grid, dim3(256), 0, s, l[0], l[1], per, ab, lb, nmk, nmb, nTn,
                       (int)K, N, ldp, (int64_t)(cexp / 16));
  else
    hipLaunchKernelGGL(expert_cond16_pair_kernel<false>, grid, dim3(256), 0, s, l[0], l[1], per, ab, lb, nmk, nmb,
                       nTn, (int)K, N, ldp, (int64_t)0);
  int st = launch_status();
  if (st) return st;
  if (batch == 2)   // both layers' finalize in one launch too
    return mgp_launch_cond_finalize2(CondFinLayer{stats[0], (const float*)workspace[0], variance[0], fmean[0], fvar[0]},
                                     CondFinLayer{stats[1], (const float*)workspace[1], variance[1], fmean[1], fvar[1]},
                                     lds, mgp_stats_tiles(M), ldp, nTp, N, K, ldf, s);
  return mgp_launch_cond_finalize(stats[0], lds, mgp_stats_tiles(M), (const float*)workspace[0], ldp, nTp,
                                  variance[0], N, K, fmean[0], fvar[0], ldf, s);
}

// Split-f16 images with the X8 plane (mgp_split_lower_f16, mgp_split_cols_f16,
// mgp_trsm_stats_f16x8): hi products on f16, cross terms on e4m3 (mfma_f8x).
extern "C" int mgp_expert_conditional_f16x8(const void* Afr, size_t afr_bytes, const void* Lfr, size_t lfr_bytes,
                                            const float* stats, int64_t lds, const float* variance, int64_t M,
                                            int64_t N, int32_t K, float* fmean, float* fvar, int64_t ldf,
                                            void* workspace, size_t workspace_bytes, mgp_stream_t stream) {
  return expert_cond_planes(Afr, afr_bytes, Lfr, lfr_bytes, stats, lds, variance, M, N, K, 2, fmean, fvar, ldf,
                            workspace, workspace_bytes, stream, true, true);
}

// ------------------------------------------------------------------ conditional backward (x6)
extern "C" size_t mgp_gram_workspace_bytes(int64_t MI, int64_t MJ, int64_t N, int32_t tri);
extern "C" size_t mgp_rows_f16_bytes(int64_t M, int64_t N);
extern "C" int64_t mgp_rows_f16_ksteps(int64_t N);
extern "C" int mgp_split_rows_f16(const float* X, int64_t ldx, int64_t M, int64_t N, const float* bound, void* img,
                                  size_t img_bytes, mgp_stream_t stream);
extern "C" int mgp_gram_f16_rows(const void* ximg, size_t ximg_bytes, int64_t MI, const float* Y, int64_t ldy,
                                 int64_t MJ, const float* W, int64_t sw, int64_t N, int32_t batch, float alpha,
                                 int32_t mode, float* out, int64_t ldo, int64_t so, const float* x_bound,
                                 const float* y_bound, const float* w_bound, void* workspace, size_t workspace_bytes,
                                 mgp_stream_t stream);
extern "C" size_t mgp_gram_x6_workspace_bytes(int64_t MI, int64_t MJ, int64_t N, int32_t batch, int32_t mode);

extern "C" int mgp_gram_x6(const float* X, int64_t ldx, int64_t sx, int64_t MI, const float* Y, int64_t ldy,
                           int64_t sy, int64_t MJ, const float* W, int64_t sw, int64_t N, int32_t batch, float alpha,
                           int32_t mode, float* out, int64_t ldo, int64_t so, void* workspace,
                           size_t workspace_bytes, mgp_stream_t stream);
extern "C" int mgp_gram_f16(const float* X, int64_t ldx, int64_t sx, int64_t MI, const float* Y, int64_t ldy,
                            int64_t sy, int64_t MJ, const float* W, int64_t sw, int64_t N, int32_t batch, float alpha,
                            int32_t mode, float* out, int64_t ldo, int64_t so, const float* x_bound,
                            const float* y_bound, const float* w_bound, void* workspace, size_t workspace_bytes,
                            mgp_stream_t stream);
extern "C" int mgp_gram(const float* X, int64_t ldx, int64_t MI, const float* Y, int64_t ldy, int64_t MJ,
                        int64_t N, float alpha, int32_t tri, float* out, int64_t ldo, void* workspace,
                        size_t workspace_bytes, mgp_stream_t stream);

int gram_f16_rowscaled(const float* X, int64_t ldx, int64_t MI, const float* Y, int64_t ldy, int64_t MJ, int64_t N,
                       float alpha, int32_t mode, float* out, int64_t ldo, const float* xb, const float* yb,
                       void* workspace, size_t workspace_bytes, mgp_stream_t stream);  // gram.hip

constexpr int kRowSumChunks = 32;  // column chunks of row_sums_kernel

namespace {
struct CondBwdWs {  // workspace carve-up (256-B aligned pieces)
  size_t sfr, ga0, rimg, qpart, gafr, lifr, P, LT, part, bnd, cexp, rmax, rpart, gram, total;
};
size_t al256(size_t x) { return (x + 255) / 256 * 256; }
CondBwdWs cond_bwd_layout(int64_t M, int64_t N, int32_t K) {
  CondBwdWs w;
  const int64_t ldn = (N + 3) / 4 * 4;
  size_t o = 0;
  const int64_t ldm = (M + 3) / 4 * 4;
  w.sfr = o;  o += al256(mgp_x6_lower_bytes(M, K));
  // gA0 (read last by step 3), then A's row image for the P_k gram (step 5)
  w.ga0 = o;  o += al256(std::max((size_t)M * ldn * 4, mgp_rows_f16_bytes(M, N)));
  // A's row image written beside gA0 by grad_a_prep_kernel (split-f16), its g_q_mu partials
  w.rimg = o; o += al256(mgp_rows_f16_bytes(M, N));
  w.qpart = o; o += al256((size_t)((mgp_rows_f16_ksteps(N) + 7) / 8) * M * K * 4);
  w.gafr = o; o += al256(mgp_x6_cols_bytes(M, N));
  w.lifr = o; o += al256(mgp_x6_lower_bytes(M, 1));
  w.P = o;    o += al256((size_t)K * M * ldm * 4);
  w.LT = o;   o += al256((size_t)K * M * ldm * 4);
  w.part = o; o += al256((size_t)K * kRowSumChunks * 8);  // row_sums partials
  w.bnd = o;  o += 256;  // split-f16 bounds: max |Gv|, max |LinvT| (MGP_TRSM_BWD16)
  w.cexp = o; o += al256((size_t)((M + 127) / 128) * ldn * 4);  // gA image scales per (row tile, column)
  w.rmax = o; o += al256((size_t)2 * M * 4);  // row maxima of A and g_Kuf (the f16 g_Lm gram)
  // their partials: per slab of 128 n (grad_a_prep), per 64 columns (trsm_bwd16)
  w.rpart = o; o += al256((size_t)(mgp_rows_f16_ksteps(N) / 8 + 1 + (N + 63) / 64 + 4) * M * 4);
  w.gram = o;
  size_t g = mgp_gram_x6_workspace_bytes(M, M, N, K, 2);
  g = g > mgp_gram_x6_workspace_bytes(M, M, M, K, 2) ? g : mgp_gram_x6_workspace_bytes(M, M, M, K, 2);
  const size_t sizes[3] = {mgp_gram_x6_workspace_bytes(M, M, M, K, 1), mgp_gram_x6_workspace_bytes(M, M, N, 1, 1),
                           mgp_gram_workspace_bytes(M, K, N, 0)};
  for (size_t v : sizes) g = v > g ? v : g;
  o += al256(g);
  w.total = o;
  return w;
}
}  // namespace

// part[k][c] = sum of x[k][n] over column chunk c (grid: rows x kRowSumChunks), then
// out = sum of all parts (fixed order).
__global__ __launch_bounds__(256) void row_sums_kernel(const float* __restrict__ x, int64_t cols, int64_t ld,
                                                       double* __restrict__ part) {
  __shared__ double scratch[16];
  const float* row = x + (int64_t)blockIdx.x * ld;
  const int64_t per = (cols + kRowSumChunks - 1) / kRowSumChunks;
  const int64_t nb = (int64_t)blockIdx.y * per, ne = nb + per < cols ? nb + per : cols;
  double v = 0.0;
  for (int64_t n = nb + threadIdx.x; n < ne; n += 256) v += (double)row[n];
  v = mgp::block_sum<double>(v, scratch);
  if (threadIdx.x == 0) part[blockIdx.x * kRowSumChunks + blockIdx.y] = v;
}

// out = sum of part[0 .. rows) in index order (one wave stages the partials in LDS,
// lane 0 adds them: the single-thread loop over global memory took 16 us)
constexpr int kSumPartsMax = 16 * kRowSumChunks;
__global__ __launch_bounds__(64) void sum_parts_kernel(const double* __restrict__ part, int rows,
                                                       double* __restrict__ out) {
  __shared__ double sp[kSumPartsMax];
  for (int i = threadIdx.x; i < rows; i += 64) sp[i] = part[i];
  __syncthreads();
  if (threadIdx.x == 0) {
    double v = 0.0;
#pragma unroll 8
    for (int k = 0; k < rows; ++k) v += sp[k];
    *out = v;
  }
}

// T[k][i][j] = L_k[i][j] for j <= i, else 0 (the lower triangle of q_sqrt).
__global__ __launch_bounds__(256) void tril_copy_kernel(const float* __restrict__ q, int64_t ldq, int64_t sq,
                                                        int64_t M, float* __restrict__ T, int64_t ldt, int64_t st) {
  const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (idx >= M * M) return;
  const int k = blockIdx.y;
  const int64_t i = idx / M, j = idx % M;
  T[k * st + i * ldt + j] = j <= i ? q[k * sq + i * ldq + j] : 0.f;
}

// LT[k][j][l] = L_k[l][j] for l >= j, else 0 (the transposed lower triangle of q_sqrt).
__global__ __launch_bounds__(256) void tril_transpose_kernel(const float* __restrict__ q, int64_t ldq, int64_t sq,
                                                             int64_t M, float* __restrict__ LT, int64_t ldt,
                                                             int64_t st) {
  __shared__ float tile[32][33];
  const int k = blockIdx.z;
  const int64_t r0 = (int64_t)blockIdx.y * 32, c0 = (int64_t)blockIdx.x * 32;  // source rows l, columns j
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
  for (int y = ty; y < 32; y += 8) {
    const int64_t l = r0 + y, j = c0 + tx;
    tile[y][tx] = (l < M && j < M && l >= j) ? q[k * sq + l * ldq + j] : 0.f;
  }
  __syncthreads();
  for (int y = ty; y < 32; y += 8) {
    const int64_t j = c0 + y, l = r0 + tx;
    if (j < M && l < M) LT[k * st + j * ldt + l] = tile[tx][y];
  }
}

extern "C" size_t mgp_conditional_backward_workspace_bytes(int64_t M, int64_t N, int32_t K) {
  if (M <= 0 || N <= 0 || K <= 0) return 256;
  return cond_bwd_layout(M, N, K).total;
}

static int conditional_backward(
    const void* Afr, size_t afr_bytes, const float* A, int64_t lda,
    const float* q_sqrt, int64_t ldqs, int64_t strideq, const float* q_mu, int64_t ldq, const float* LinvT,
    int64_t ldl, const float* Gmu, const float* Gv, int64_t ldg, int64_t M, int64_t N, int32_t K,
    float* g_q_mu, int64_t ldgq, float* g_q_sqrt, int64_t ldgs, int64_t strideg, float* g_Kuf, int64_t ldk,
    float* g_Lm, int64_t ldgl, double* g_var, void* workspace, size_t workspace_bytes, mgp_stream_t stream,
    bool f16, bool x8 = false, const void* Cfr = nullptr, size_t cfr_bytes = 0, const float* colmax = nullptr,
    const float* l_bound = nullptr, const void* qprep = nullptr, const float* t_bound = nullptr) {
  if (!Afr) return -1;
  if (afr_bytes < mgp_x6_cols_bytes(M, N)) return -2;
  if (!A) return -3;
  if (lda < N) return -4;
  if (!q_sqrt) return -7;
  if (ldqs < M) return -8;
  if (!q_mu) return -10;
  if (ldq < K) return -11;
  if (!LinvT) return -12;
  if (ldl < M) return -13;
  if (!Gmu) return -14;
  if (!Gv) return -15;
  if (ldg < N) return -16;
  if (M <= 0) return -17;
  if (N <= 0) return -18;
  if (K < 1) return -19;
  if (K > 16) return MGP_ERR_UNSUPPORTED;
  if (!g_q_mu) return -20;
  if (!g_q_sqrt) return -22;
  if (!g_Kuf) return -25;
  if (!g_Lm) return -27;
  if (!g_var) return -29;
  if (!workspace || workspace_bytes < mgp_conditional_backward_workspace_bytes(M, N, K)) return MGP_ERR_WORKSPACE;
  if (!aligned16(workspace) || !aligned16(Afr)) return MGP_ERR_ALIGN;
  const size_t img = mgp_x6_cols_bytes(M, N);
  if (img >= ((size_t)1 << 32) || (size_t)M * ((N + 3) / 4 * 4) * 4 >= ((size_t)1 << 32)) return MGP_ERR_UNSUPPORTED;
  // the S_k / L_k image is addressed through one 32-bit buffer resource by the gA kernels
  if (lower_planes(M, K) >= ((size_t)1 << 32)) return MGP_ERR_UNSUPPORTED;
  hipStream_t s = (hipStream_t)stream;
  const CondBwdWs L = cond_bwd_layout(M, N, K);
  char* ws = (char*)workspace;
  const int64_t ldn = (N + 3) / 4 * 4;
  float* P = (float*)(ws + L.P);
  float* LT = qprep ? (float*)((char*)const_cast<void*>(qprep) + al256(mgp_x6_lower_bytes(M, K))) : (float*)(ws + L.LT);
  double* part = (double*)(ws + L.part);
  const int64_t ldm = (M + 3) / 4 * 4;
  // qprep (mgp_conditional_backward_prep_f16c, the C path only): L_k's image and the
  // transposed triangles already formed from q_sqrt, e.g. beside the forward's K3
  bf16x8* Sfr = qprep ? (bf16x8*)const_cast<void*>(qprep) : (bf16x8*)(ws + L.sfr);
  float* gA0 = (float*)(ws + L.ga0);
  bf16x8* gAfr = (bf16x8*)(ws + L.gafr);
  bf16x8* LIfr = (bf16x8*)(ws + L.lifr);
  void* gws = ws + L.gram;
  const size_t gwsb = L.total - L.gram;
  const int64_t Mp = x6_mp(M);
  const int nmk = (int)(Mp / 16), nmb = (int)(Mp / 32), nT = (int)(Mp / kX6BM);
  const int nTn = (int)(x6_np(N) / kX6BN);
  int st;
  const bool cpath = f16 && !x8 && Cfr;  // B-b from the forward's C_k images
  // B-d on split-f16 images (trsm_bwd16_kernel): the C path, M <= 4096
  const bool bwd16 = kTrsmBwd16 && cpath && nT <= kTrsmBwd16MaxT;
  // max |LinvT| given (t_bound: the forward's L^-T image bound from K3) or formed here
  float* li_bound = t_bound ? const_cast<float*>(t_bound) : (float*)(ws + L.bnd) + 1;
  float* cexp = (float*)(ws + L.cexp);
  if (cpath) {
    if (!colmax || !l_bound) return -32;
    if (cfr_bytes < mgp_c_images_bytes(M, N, K)) return -31;
    if ((int64_t)K * ldg * 4 >= ((int64_t)1 << 32)) return MGP_ERR_UNSUPPORTED;  // grad_a_c's Gv resource
    if (!aligned16(Cfr)) return MGP_ERR_ALIGN;
    // L_k's image (rows m, k-steps over m' <= m) into the S image's space; Linv's image
    const int64_t nfrag = (int64_t)K * nmb * nmk, nf1 = (int64_t)nmb * nmk;
    if (!qprep)
      hipLaunchKernelGGL((split_tri_kernel<false, true>), dim3((unsigned)((nfrag + 3) / 4)), dim3(256), 0, s, q_sqrt,
                         ldqs, strideq, M, nmb, nmk, nfrag, Sfr, l_bound);
    if (bwd16 && !t_bound) {  // Linv's split-f16 image at max |LinvT| (its upper triangle)
      if ((st = hip_status(hipMemsetAsync(li_bound, 0, sizeof(float), s)))) return st;
      launch_absmax<2>(LinvT, ldl, (int64_t)0, M, M, M, li_bound, s);
    }
    hipLaunchKernelGGL((split_tri_kernel<true, true>), dim3((unsigned)((nf1 + 3) / 4)), dim3(256), 0, s, LinvT, ldl,
                       (int64_t)0, M, nmb, nmk, nf1, LIfr, bwd16 ? (const float*)li_bound : nullptr);
    if ((st = launch_status())) return st;
  } else {
  // 1. S_k = L_k L_k^T (x6 gram over M of tril(q_sqrt), into the LT buffer) and its
  //    full split images; the image of Linv (T operand of B-d)
  hipLaunchKernelGGL(tril_copy_kernel, dim3((unsigned)((M * M + 255) / 256), (unsigned)K), dim3(256), 0, s, q_sqrt,
                     ldqs, strideq, M, P, ldm, M * ldm);
  if ((st = launch_status())) return st;
  st = mgp_gram_x6(P, ldm, M * ldm, M, P, ldm, M * ldm, M, nullptr, 0, M, K, 1.f, 2, LT, ldm, M * ldm, gws, gwsb,
                   stream);
  if (st) return st;
  {
    const int64_t nfrag = (int64_t)K * nmb * nmk;
    float* s_bound = trailer(Sfr, lower_planes(M, K));
    if (f16) {  // max |S_k| over the experts into the image trailer, then the scaled split
      if ((st = hip_status(hipMemsetAsync(s_bound, 0, sizeof(float), s)))) return st;
      launch_absmax<0>(LT, ldm, M * ldm, M, M, (int64_t)K * M, s_bound, s);
    }
    hipLaunchKernelGGL((split_tri_kernel<true, false, true>), dim3((unsigned)((nfrag + 3) / 4)), dim3(256), 0, s, LT,
                       ldm, M * ldm, M, nmb, nmk, nfrag, Sfr, f16 ? (const float*)s_bound : nullptr);
    const int64_t nf1 = (int64_t)nmb * nmk;
    hipLaunchKernelGGL((split_tri_kernel<true, true>), dim3((unsigned)((nf1 + 3) / 4)), dim3(256), 0, s, LinvT, ldl,
                       (int64_t)0, M, nmb, nmk, nf1, LIfr);
    if ((st = launch_status())) return st;
  }
  }
  // 2. gA0 = q_mu G_mu - 2 A sum_k Gv_k; split-f16: with A's row image (step 5) and
  //    g_q_mu's partials (step 6) in the same pass over A
  const float* a_bound = trailer(const_cast<void*>(Afr), cols_planes(M, N));
  bf16x8* rimg = (bf16x8*)(ws + L.rimg);
  float* qpart = (float*)(ws + L.qpart);
  const int nns = (int)mgp_rows_f16_ksteps(N);
  const int slabs = (nns + 7) / 8;
  const bool prep = f16 && lda % 4 == 0 && aligned16(A);  // else grad_a_base, split_rows_f16, gram_narrow
  // g_Lm on f16 products with exact per-row scales (MGP_GLM_F16): the row maxima of A
  // (grad_a_prep) and of g_Kuf (trsm_bwd16) by atomics
  const bool glm16 = kGlmF16 && bwd16 && prep;
  float* rmaxA = (float*)(ws + L.rmax);
  float* rmaxG = rmaxA + M;
  float* rpartA = glm16 ? (float*)(ws + L.rpart) : nullptr;
  float* rpartG = glm16 ? rpartA + (int64_t)slabs * M : nullptr;
  if (prep) {
    const int rbs = kPrepRB;
    const dim3 grid((unsigned)slabs, (unsigned)((M + 32 * rbs - 1) / (32 * rbs)));
    const int qvec = (ldq % 4 == 0 && K % 4 == 0 && aligned16(q_mu)) ? 1 : 0;
    if (K <= 4)
      hipLaunchKernelGGL(grad_a_prep_kernel<4>, grid, dim3(256), 0, s, A, lda, q_mu, ldq, Gmu, Gv, ldg, M, N, K, nns,
                         a_bound, gA0, ldn, rimg, qpart, rbs, qvec, rpartA);
    else if (K <= 8)
      hipLaunchKernelGGL(grad_a_prep_kernel<8>, grid, dim3(256), 0, s, A, lda, q_mu, ldq, Gmu, Gv, ldg, M, N, K, nns,
                         a_bound, gA0, ldn, rimg, qpart, rbs, qvec, rpartA);
    else
      hipLaunchKernelGGL(grad_a_prep_kernel<16>, grid, dim3(256), 0, s, A, lda, q_mu, ldq, Gmu, Gv, ldg, M, N, K, nns,
                         a_bound, gA0, ldn, rimg, qpart, rbs, qvec, rpartA);
    if ((st = launch_status())) return st;
  } else {
    const int rows = 128;
    const dim3 grid((unsigned)((N + 255) / 256), (unsigned)((M + rows - 1) / rows));
    if (K <= 4)
      hipLaunchKernelGGL(grad_a_base_kernel<4>, grid, dim3(256), 0, s, A, lda, q_mu, ldq, Gmu, Gv, ldg, M, N, K, rows,
                         gA0, ldn);
    else if (K <= 8)
      hipLaunchKernelGGL(grad_a_base_kernel<8>, grid, dim3(256), 0, s, A, lda, q_mu, ldq, Gmu, Gv, ldg, M, N, K, rows,
                         gA0, ldn);
    else
      hipLaunchKernelGGL(grad_a_base_kernel<16>, grid, dim3(256), 0, s, A, lda, q_mu, ldq, Gmu, Gv, ldg, M, N, K,
                         rows, gA0, ldn);
    if ((st = launch_status())) return st;
  }
  // 3. gA (image) = 2 sum_k (S_k A) diag(Gv_k) + gA0  (C path: 2 sum_k L_k C_k diag(Gv_k) + gA0)
  if (cpath && kGac16 && bwd16 && K <= kGac16KMax)
    hipLaunchKernelGGL(grad_a_c16_kernel<kGac16G>, dim3((unsigned)((nT + 1) / 2 * nTn)), dim3(256 * kGac16G), 0, s,
                       (const bf16x8*)Sfr,
                       (uint32_t)lower_planes(M, K), (const bf16x8*)Cfr, (int64_t)(cols_planes(M, N) / 16),
                       (uint32_t)cols_planes(M, N), nmk, nTn, K, M, N, Gv, ldg, gA0, ldn, gAfr, l_bound,
                       (const float*)trailer(const_cast<void*>(Afr), cols_planes(M, N)), colmax, cexp, ldn);
  else if (cpath)
    hipLaunchKernelGGL((grad_a_c_kernel<kGacPD, kGacNC>), dim3((unsigned)((nT + 1) / 2 * (2 / kGacNC) * nTn)), dim3(256), 0, s,
                       (const bf16x8*)Sfr, (uint32_t)lower_planes(M, K), (const bf16x8*)Cfr,
                       (int64_t)(cols_planes(M, N) / 16), (uint32_t)cols_planes(M, N), nmk, (2 / kGacNC) * nTn, K, M, N, Gv, ldg, gA0, ldn, gAfr, l_bound,
                       (const float*)trailer(const_cast<void*>(Afr), cols_planes(M, N)), colmax,
                       bwd16 ? cexp : nullptr, ldn);
  else if (f16 && x8)
    hipLaunchKernelGGL((grad_a_s_kernel<true, true>), dim3((unsigned)(nT * 2 * nTn)), dim3(256), 0, s,
                       (const bf16x8*)Sfr, (uint32_t)mgp_x6_lower_bytes(M, 1), (const bf16x8*)Afr, (uint32_t)afr_bytes,
                       nmk, 2 * nTn, K, M, N, Gv, ldg, gA0, ldn, gAfr, (const float*)trailer(Sfr, lower_planes(M, K)),
                       (const float*)trailer(const_cast<void*>(Afr), cols_planes(M, N)));
  else if (f16)
    hipLaunchKernelGGL(grad_a_s_f16_kernel, dim3((unsigned)(nT * 2 * nTn)), dim3(256), 0, s, (const bf16x8*)Sfr,
                       (uint32_t)lower_planes(M, K), (const bf16x8*)Afr, (uint32_t)afr_bytes, nmk, 2 * nTn, K, M, N,
                       Gv, ldg, gA0, ldn, gAfr, (const float*)trailer(Sfr, lower_planes(M, K)),
                       (const float*)trailer(const_cast<void*>(Afr), cols_planes(M, N)));
  else
    hipLaunchKernelGGL(grad_a_s_kernel<false>, dim3((unsigned)(nT * 2 * nTn)), dim3(256), 0, s, (const bf16x8*)Sfr,
                       (uint32_t)mgp_x6_lower_bytes(M, 1), (const bf16x8*)Afr, (uint32_t)afr_bytes, nmk, 2 * nTn, K,
                       M, N, Gv, ldg, gA0, ldn, gAfr, nullptr, nullptr);
  if ((st = launch_status())) return st;
  // 4. gKuf = Linv^T gA
  if (bwd16)
    hipLaunchKernelGGL(trsm_bwd16_kernel, dim3((unsigned)(nT * nTn)), dim3(256), 0, s, (const bf16x8*)gAfr,
                       (const bf16x8*)LIfr, (uint32_t)img, (uint32_t)mgp_x6_lower_bytes(M, 1), nmk, nmb, nTn, M, N,
                       g_Kuf, ldk, (const float*)cexp, ldn, (const float*)li_bound, rpartG);
  else
  hipLaunchKernelGGL(trsm_bwd_kernel, dim3((unsigned)(nT * nTn)), dim3(256), 0, s, (const bf16x8*)gAfr,
                     (const bf16x8*)LIfr, (uint32_t)img, (uint32_t)mgp_x6_lower_bytes(M, 1), nmk, nmb, nTn, M, N, g_Kuf,
                     ldk);
  if ((st = launch_status())) return st;
  // 5. g_q_sqrt[k] = 2 tril(A diag(Gv_k) (L_k^T A)^T) = 2 tril(P_k L_k), P_k = A diag(Gv_k) A^T
  //    (x6 grams over N, then over M with the transposed triangle of L_k); f16: the
  //    grams over N on f16 products, bounds |A| <= sqrt(var) (Afr's trailer), max |Gv|
  float* bnd = (float*)(ws + L.bnd);
  if (f16) {
    if ((st = hip_status(hipMemsetAsync(bnd, 0, sizeof(float), s)))) return st;
    launch_absmax<0>(Gv, ldg, (int64_t)0, (int64_t)K, N, (int64_t)K, bnd, s);
    if ((st = launch_status())) return st;
    // A's row image (step 2) as the grams' unweighted side
    if (!prep && (st = mgp_split_rows_f16(A, lda, M, N, a_bound, rimg, mgp_rows_f16_bytes(M, N), stream))) return st;
    st = mgp_gram_f16_rows(rimg, mgp_rows_f16_bytes(M, N), M, A, lda, M, Gv, ldg, N, K, 1.f, 2, P, ldm, M * ldm,
                           a_bound, a_bound, bnd, gws, gwsb, stream);
  } else {
    st = mgp_gram_x6(A, lda, 0, M, A, lda, 0, M, Gv, ldg, N, K, 1.f, 2, P, ldm, M * ldm, gws, gwsb, stream);
  }
  if (st) return st;
  if (!(cpath && qprep)) {
    hipLaunchKernelGGL(tril_transpose_kernel, dim3((unsigned)((M + 31) / 32), (unsigned)((M + 31) / 32), (unsigned)K),
                       dim3(256), 0, s, q_sqrt, ldqs, strideq, M, LT, ldm, M * ldm);
    if ((st = launch_status())) return st;
  }
  st = mgp_gram_x6(P, ldm, M * ldm, M, LT, ldm, M * ldm, M, nullptr, 0, M, K, 2.f, 1, g_q_sqrt, ldgs, strideg, gws,
                   gwsb, stream);
  if (st) return st;
  // 6. g_Lm = -tril(g_Kuf A^T), g_q_mu = A G_mu^T, g_var = sum G_v.  g_Lm stays x6 in
  //    both modes: it feeds the near-cancelling Z / lengthscale / variance gradients
  //    through the Cholesky backward (split-f16 operands measured 3.6e-4 normwise on a
  //    lengthscale gradient where float32 autograd is 2.2e-4)
  //    (the C path with MGP_GLM_F16: f16 products, every row of g_Kuf and of A split at
  //    its own exact scale -- the global-bound split was what lost the accuracy)
  if (glm16) {
    hipLaunchKernelGGL(rowmax_fold_kernel, dim3((unsigned)((M + 15) / 16), 2), dim3(1024), 0, s, rpartA, slabs,
                       rpartG, 4 * nTn, M, rmaxA);
    if ((st = launch_status())) return st;
  }
  if (glm16)
    st = gram_f16_rowscaled(g_Kuf, ldk, M, A, lda, M, N, -1.f, 1, g_Lm, ldgl, (const float*)rmaxG,
                            (const float*)rmaxA, gws, gwsb, stream);
  else
    st = mgp_gram_x6(g_Kuf, ldk, 0, M, A, lda, 0, M, nullptr, 0, N, 1, -1.f, 1, g_Lm, ldgl, M * ldgl, gws, gwsb,
                     stream);
  if (st) return st;
  if (prep) {  // g_q_mu from step 2's partials
    hipLaunchKernelGGL(prep_fold_kernel, dim3((unsigned)((M * K + 15) / 16)), dim3(256), 0, s, qpart, slabs, M, K,
                       g_q_mu, ldgq);
  } else {
    st = mgp_gram(A, lda, M, Gmu, ldg, K, N, 1.f, 0, g_q_mu, ldgq, gws, gwsb, stream);
    if (st) return st;
  }
  hipLaunchKernelGGL(row_sums_kernel, dim3((unsigned)K, kRowSumChunks), dim3(256), 0, s, Gv, N, ldg, part);
  hipLaunchKernelGGL(sum_parts_kernel, dim3(1), dim3(64), 0, s, part, (int)K * kRowSumChunks, g_var);
  return launch_status();
}

extern "C" int mgp_conditional_backward_x6(
    const void* Afr, size_t afr_bytes, const float* A, int64_t lda,
    const float* q_sqrt, int64_t ldqs, int64_t strideq, const float* q_mu, int64_t ldq, const float* LinvT,
    int64_t ldl, const float* Gmu, const float* Gv, int64_t ldg, int64_t M, int64_t N, int32_t K,
    float* g_q_mu, int64_t ldgq, float* g_q_sqrt, int64_t ldgs, int64_t strideg, float* g_Kuf, int64_t ldk,
    float* g_Lm, int64_t ldgl, double* g_var, void* workspace, size_t workspace_bytes, mgp_stream_t stream) {
  return conditional_backward(Afr, afr_bytes, A, lda, q_sqrt, ldqs, strideq, q_mu, ldq, LinvT, ldl, Gmu, Gv, ldg, M,
                              N, K, g_q_mu, ldgq, g_q_sqrt, ldgs, strideg, g_Kuf, ldk, g_Lm, ldgl, g_var, workspace,
                              workspace_bytes, stream, false);
}

// Afr is A's split-f16 image (mgp_trsm_stats_f16); S_k = L_k L_k^T is split the same
// way, so the S_k A product (B-b) runs on three f16 products per block.
extern "C" int mgp_conditional_backward_f16(
    const void* Afr, size_t afr_bytes, const float* A, int64_t lda,
    const float* q_sqrt, int64_t ldqs, int64_t strideq, const float* q_mu, int64_t ldq, const float* LinvT,
    int64_t ldl, const float* Gmu, const float* Gv, int64_t ldg, int64_t M, int64_t N, int32_t K,
    float* g_q_mu, int64_t ldgq, float* g_q_sqrt, int64_t ldgs, int64_t strideg, float* g_Kuf, int64_t ldk,
    float* g_Lm, int64_t ldgl, double* g_var, void* workspace, size_t workspace_bytes, mgp_stream_t stream) {
  return conditional_backward(Afr, afr_bytes, A, lda, q_sqrt, ldqs, strideq, q_mu, ldq, LinvT, ldl, Gmu, Gv, ldg, M,
                              N, K, g_q_mu, ldgq, g_q_sqrt, ldgs, strideg, g_Kuf, ldk, g_Lm, ldgl, g_var, workspace,
                              workspace_bytes, stream, true);
}

// mgp_conditional_backward_f16 with the forward's C_k images (mgp_expert_conditional_f16c
// with the same Afr, q_sqrt and colmax; l_bound = the bound of its Lfr image):
// B-b as 2 sum_k L_k C_k diag(Gv_k), no S_k = L_k L_k^T.
extern "C" int mgp_conditional_backward_f16c(
    const void* Afr, size_t afr_bytes, const float* A, int64_t lda,
    const float* q_sqrt, int64_t ldqs, int64_t strideq, const float* q_mu, int64_t ldq, const float* LinvT,
    int64_t ldl, const float* Gmu, const float* Gv, int64_t ldg, int64_t M, int64_t N, int32_t K,
    float* g_q_mu, int64_t ldgq, float* g_q_sqrt, int64_t ldgs, int64_t strideg, float* g_Kuf, int64_t ldk,
    float* g_Lm, int64_t ldgl, double* g_var, void* workspace, size_t workspace_bytes, const void* Cfr,
    size_t cfr_bytes, const float* colmax, const float* l_bound, mgp_stream_t stream) {
  if (!Cfr) return -30;
  return conditional_backward(Afr, afr_bytes, A, lda, q_sqrt, ldqs, strideq, q_mu, ldq, LinvT, ldl, Gmu, Gv, ldg, M,
                              N, K, g_q_mu, ldgq, g_q_sqrt, ldgs, strideg, g_Kuf, ldk, g_Lm, ldgl, g_var, workspace,
                              workspace_bytes, stream, true, false, Cfr, cfr_bytes, colmax, l_bound);
}

// The q_sqrt-only part of mgp_conditional_backward_f16c -- L_k's image (the B-b operand,
// scale l_bound: the bound of the forward's Lfr image) and the transposed triangles
// L_k^T (B-d's operand) -- into prep, so that it can run off the backward's critical
// path (the Python host: on the side stream beside the forward's K3).
extern "C" size_t mgp_conditional_backward_prep_bytes(int64_t M, int32_t K) {
  if (M <= 0 || K <= 0) return 256;
  const int64_t ldm = (M + 3) / 4 * 4;
  return al256(mgp_x6_lower_bytes(M, K)) + al256((size_t)K * M * ldm * 4);
}

extern "C" int mgp_conditional_backward_prep_f16c(const float* q_sqrt, int64_t ldqs, int64_t strideq, int64_t M,
                                                  int32_t K, const float* l_bound, void* prep, size_t prep_bytes,
                                                  mgp_stream_t stream) {
  if (!q_sqrt) return -1;
  if (ldqs < M) return -2;
  if (K > 1 && strideq < ldqs * M) return -3;
  if (M <= 0) return -4;
  if (K < 1) return -5;
  if (K > 16) return MGP_ERR_UNSUPPORTED;
  if (!l_bound) return -6;
  if (!prep) return -7;
  if (prep_bytes < mgp_conditional_backward_prep_bytes(M, K)) return MGP_ERR_WORKSPACE;
  if (!aligned16(prep)) return MGP_ERR_ALIGN;
  if (lower_planes(M, K) >= ((size_t)1 << 32)) return MGP_ERR_UNSUPPORTED;
  hipStream_t s = (hipStream_t)stream;
  const int64_t Mp = x6_mp(M), ldm = (M + 3) / 4 * 4;
  const int nmk = (int)(Mp / 16), nmb = (int)(Mp / 32);
  const int64_t nfrag = (int64_t)K * nmb * nmk;
  float* LT = (float*)((char*)prep + al256(mgp_x6_lower_bytes(M, K)));
  // (full grids: the capped grid-stride form of the ELBO's q_sqrt launches measured slower here,
  // training step 14.02-14.11 vs 13.98-14.01 ms, profiles/r06w_side_grid_ab.log)
  hipLaunchKernelGGL((split_tri_kernel<false, true>), dim3((unsigned)((nfrag + 3) / 4)), dim3(256), 0, s, q_sqrt,
                     ldqs, strideq, M, nmb, nmk, nfrag, (bf16x8*)prep, l_bound);
  hipLaunchKernelGGL(tril_transpose_kernel, dim3((unsigned)((M + 31) / 32), (unsigned)((M + 31) / 32), (unsigned)K),
                     dim3(256), 0, s, q_sqrt, ldqs, strideq, M, LT, ldm, M * ldm);
  return launch_status();
}

// mgp_conditional_backward_f16c on a prep of the same q_sqrt and l_bound
// (mgp_conditional_backward_prep_f16c): two launches fewer, the same results.
extern "C" int mgp_conditional_backward_f16c_prepped(
    const void* Afr, size_t afr_bytes, const float* A, int64_t lda,
    const float* q_sqrt, int64_t ldqs, int64_t strideq, const float* q_mu, int64_t ldq, const float* LinvT,
    int64_t ldl, const float* Gmu, const float* Gv, int64_t ldg, int64_t M, int64_t N, int32_t K,
    float* g_q_mu, int64_t ldgq, float* g_q_sqrt, int64_t ldgs, int64_t strideg, float* g_Kuf, int64_t ldk,
    float* g_Lm, int64_t ldgl, double* g_var, void* workspace, size_t workspace_bytes, const void* Cfr,
    size_t cfr_bytes, const float* colmax, const float* l_bound, const void* prep, size_t prep_bytes,
    const float* t_bound, mgp_stream_t stream) {
  if (!Cfr) return -30;
  if (!prep) return -33;
  if (prep_bytes < mgp_conditional_backward_prep_bytes(M, K)) return -34;
  if (!aligned16(prep)) return MGP_ERR_ALIGN;
  return conditional_backward(Afr, afr_bytes, A, lda, q_sqrt, ldqs, strideq, q_mu, ldq, LinvT, ldl, Gmu, Gv, ldg, M,
                              N, K, g_q_mu, ldgq, g_q_sqrt, ldgs, strideg, g_Kuf, ldk, g_Lm, ldgl, g_var, workspace,
                              workspace_bytes, stream, true, false, Cfr, cfr_bytes, colmax, l_bound, prep, t_bound);
}

// Afr from mgp_trsm_stats_f16x8 with the f32 A (all three planes): S_k A on f16 hi
// products + e4m3 cross terms (grad_a_s_kernel<true, true>).
extern "C" int mgp_conditional_backward_f16x8(
    const void* Afr, size_t afr_bytes, const float* A, int64_t lda,
    const float* q_sqrt, int64_t ldqs, int64_t strideq, const float* q_mu, int64_t ldq, const float* LinvT,
    int64_t ldl, const float* Gmu, const float* Gv, int64_t ldg, int64_t M, int64_t N, int32_t K,
    float* g_q_mu, int64_t ldgq, float* g_q_sqrt, int64_t ldgs, int64_t strideg, float* g_Kuf, int64_t ldk,
    float* g_Lm, int64_t ldgl, double* g_var, void* workspace, size_t workspace_bytes, mgp_stream_t stream) {
  return conditional_backward(Afr, afr_bytes, A, lda, q_sqrt, ldqs, strideq, q_mu, ldq, LinvT, ldl, Gmu, Gv, ldg, M,
                              N, K, g_q_mu, ldgq, g_q_sqrt, ldgs, strideg, g_Kuf, ldk, g_Lm, ldgl, g_var, workspace,
                              workspace_bytes, stream, true, true);
}

#ifdef MGP_DBG_STAMPS
extern "C" int mgp_dbg_k4_stamps(unsigned long long* host) {
  return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(mgp::g_k4_stamps), sizeof(mgp::g_k4_stamps));
}
#endif
