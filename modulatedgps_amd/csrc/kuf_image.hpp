// K1's block body (Kuf = K(Z, X) written as a split-bf16 / split-f16 fragment image),
// shared by its own launch (rbf.hip: rbf_kuf_x6_kernel) and by the extra workgroups
// the K3 step launches carry (chol.hip: chol_step_pair's Kuf side job).
//
// Reference: MixtureGPs/models.py:139 (self.kernel.K(Z, Xnew)); GPflow 2.7
// SquaredExponential.K_r2(r2) = var * exp(-0.5 r2), r2 = square_distance(X / l, Z / l).
//
// r2 = |z'|^2 + |x'|^2 - 2 z'.x' (scaled inputs, the expanded form GPflow's
// square_distance uses) is ONE [32 x (D + 2)] x [(D + 2) x 32] product on
// v_mfma_f32_32x32x2_f32 (exact f32 products): rows of Z carry (z', |z'|^2, 1),
// columns of X carry (-2 x', 1, |x'|^2).  The accumulator of that MFMA holds
// row (r & 3) + 8 (r >> 2) + 4 h of column l & 31 in register r -- exactly the
// order of an image fragment: registers 0..7 / 8..15 of a 32x32 tile are the
// lane's 8 elements of k-steps 2 mb / 2 mb + 1.  So each lane finishes its 16
// values with one exp2 and one multiply each (variance and, split-f16, the
// image's power-of-two scale folded into one per-lane multiplier that is 0 on
// padded columns), splits them and stores 16-B fragments.
// Block = 4 waves (a 256-thread group) x 32 columns x 128 rows (4 row tiles per
// wave); block `bid` is row block bid % row_blocks of column group bid / row_blocks
// (consecutive blocks walk down a column group: adjacent image windows).
// Rows >= M and columns >= N of the padded image are written as zeros.
// F16: split-f16 image (Kuf <= variance, so the image scale is 2^img_exp(variance)
// and block 0 writes the variance into the trailer `bound`).
#pragma once

#include <type_traits>

#include "mgp_common.hpp"

namespace mgp {

struct KufImageArgs {
  const float* X; int64_t ldx;
  const float* Z; int64_t ldz;
  int64_t N, M; int D;
  const float* variance; const float* ls; int n_ls;
  int nmk, row_blocks;
  bf16x8* Kfr; float* bound;
};

// LDS floats a group needs: zs [128][DP] + cs [2 KS]
template <int DMAX>
constexpr int kuf_block_lds_floats() {
  return 128 * (2 * ((DMAX + 1) / 2 + 1) + 1) + 2 * ((DMAX + 1) / 2);
}

// Stores of the image fragments (16 B per lane): POL 0 plain, 1 non-temporal (streaming:
// fewer dirty L2 lines left for the kernel boundary to write back -- the K3 step
// launches' side job, where every boundary is on the Cholesky chain's critical path).
template <int POL>
__device__ __forceinline__ void img_store(bf16x8* p, bf16x8 v) {
  if constexpr (POL == 0) *p = v;
  else __builtin_nontemporal_store(v, p);
}

template <bool F16, int POL>
__device__ __forceinline__ void store_fragment(bf16x8* __restrict__ dst, const float (&v)[8]) {
  if constexpr (POL == 0) {
    if constexpr (F16) store_split_f16(dst, v, 1.f);
    else store_split(dst, v);
  } else if constexpr (F16) {   // store_split_f16 (no e4m3 plane) with POL stores
    halfx8 h, l;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const _Float16 hi = (_Float16)v[j];
      h[j] = hi;
      l[j] = (_Float16)(v[j] - (float)hi);
    }
    img_store<POL>(dst, __builtin_bit_cast(bf16x8, h));
    img_store<POL>(dst + 64, __builtin_bit_cast(bf16x8, l));
  } else {                      // store_split with POL stores
    bf16x8 h, m, l;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      __bf16 a, b, c;
      split3(v[j], a, b, c);
      h[j] = a; m[j] = b; l[j] = c;
    }
    img_store<POL>(dst, h);
    img_store<POL>(dst + 64, m);
    img_store<POL>(dst + 128, l);
  }
}

// One block by the 256 threads of a group (t = thread index within the group).  Every
// thread of the WORKGROUP must call it the same number of times: it takes three
// __syncthreads(); a group with nothing to do passes active = false (it joins the
// barriers, loads and stores nothing).  lds: kuf_block_lds_floats<DMAX>() floats of
// this group's own.
template <int DMAX, bool F16, int POL = 0>
__device__ __forceinline__ void kuf_image_block(const KufImageArgs& a, int64_t bid, int t, bool active,
                                                float* __restrict__ lds) {
  constexpr int KS = (DMAX + 1) / 2;     // MFMA k-steps over the dims (2 each) ...
  constexpr int KA = KS + 1;             // ... + one for the (|z'|^2, 1) x (1, |x'|^2) terms
  constexpr int DP = 2 * KA + 1;         // LDS row pitch (odd: spreads banks)
  float* zs = lds;
  float* cs = lds + 128 * DP;
  const int lane = t & 63, w = t >> 6, h = lane >> 5, c32 = lane & 31;
  const int64_t rb = bid % a.row_blocks, cg = bid / a.row_blocks;
  const int64_t nb = cg * 4 + w;
  const int64_t n = 32 * nb + c32;
  const int64_t m0 = 128 * rb;
  const float kHalfLog2e = 0.8493218002880191f;  // sqrt(0.5 * log2(e))
  if (active && t < 2 * KS) cs[t] = (t < a.D) ? kHalfLog2e / a.ls[a.n_ls == 1 ? 0 : t] : 0.f;
  __syncthreads();
  float xk[KA], xx = 0.f;
  if (active) {
    for (int i = t; i < 128 * 2 * KS; i += 256) {
      const int r = i / (2 * KS), d = i % (2 * KS);
      const int64_t m = m0 + r;
      zs[r * DP + d] = (m < a.M && d < a.D) ? a.Z[m * a.ldz + d] * cs[d] : 0.f;
    }
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      const int d = 2 * s + h;
      const float xd = (n < a.N && d < a.D) ? a.X[n * a.ldx + d] * cs[d] : 0.f;
      xx = fmaf(xd, xd, xx);
      xk[s] = -2.f * xd;
    }
  }
  xx += __shfl_xor(xx, 32, 64);  // the two lane halves hold the even / odd dims
  xk[KS] = h ? xx : 1.f;         // k = 2 KS: |z'|^2 * 1, k = 2 KS + 1: 1 * |x'|^2
  __syncthreads();
  if (active && t < 128) {
    float s2 = 0.f;
#pragma unroll
    for (int d = 0; d < 2 * KS; ++d) s2 = fmaf(zs[t * DP + d], zs[t * DP + d], s2);
    zs[t * DP + 2 * KS] = s2;
    zs[t * DP + 2 * KS + 1] = 1.f;
  }
  __syncthreads();
  if (!active) return;
  const float var = a.variance[0];
  // the image scale (a power of two, split-f16) and the variance fold into one
  // per-lane multiplier; padded columns (n >= N) get 0 (their r2 is finite)
  float mult = var;
  if constexpr (F16) {
    mult = var * ldexpf(1.f, img_exp(var));
    if (bid == 0 && t == 0) *a.bound = var;
  }
  if (n >= a.N) mult = 0.f;
  auto tiles = [&](auto ragged) {
    constexpr bool RAGGED = decltype(ragged)::value;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      floatx16 acc;
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[e] = 0.f;
#pragma unroll
      for (int s = 0; s < KA; ++s) acc = mfma32x32x2(zs[(32 * i + c32) * DP + 2 * s + h], xk[s], acc);
      const int64_t mb = (m0 >> 5) + i;
#pragma unroll
      for (int half = 0; half < 2; ++half) {
        float v[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          // acc = r2 >= 0 up to rounding; raw v_exp_f32 (results below 2^-126 flush)
          v[j] = __builtin_amdgcn_exp2f(-acc[8 * half + j]) * mult;
          if constexpr (RAGGED)
            if (m0 + 32 * i + acc_row(8 * half + j, lane) >= a.M) v[j] = 0.f;
          // the split below must see v as the rounded f32 value: without this the
          // compiler contracts the multiply into the hi / lo conversions
          // (v_fma_mix{lo,hi}_f16 on the unrounded product beside v_cvt_pk_f16_f32 of
          // the rounded one), which left the lo plane inconsistent with hi whenever
          // mult is not a power of two (kernel variance 0.1: Kuf image off by half an
          // f16 ulp of hi, 3e-4 of the maximum, tests/diag_f16_images.py)
          asm volatile("" : "+v"(v[j]));
        }
        store_fragment<F16, POL>(a.Kfr + ((nb * a.nmk + 2 * mb + half) * 3) * 64 + lane, v);
      }
    }
  };
  if (m0 + 128 <= a.M)   // uniform: only the last row block is ragged
    tiles(std::false_type{});
  else
    tiles(std::true_type{});
}

// The image geometry of a Kuf image (rbf.hip's launch, chol.hip's side job): row
// blocks of 128 rows, column groups of 128 columns over the padded Np = 256 ceil(N / 256).
inline int kuf_row_blocks(int64_t M) { return (int)((M + 127) / 128); }
inline int64_t kuf_blocks(int64_t M, int64_t N) { return ((N + 255) / 256 * 256 / 128) * kuf_row_blocks(M); }

}  // namespace mgp
