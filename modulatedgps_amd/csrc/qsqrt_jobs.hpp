// The work on tril(q_sqrt) that depends only on a layer's variational parameters, shared
// by its per-layer launches and by the two-layer launches of mgp_qsqrt_images_kl_f16_batch:
//   - the whitened-KL partial sums (K7: kl_partials_kernel, elbo.hip), here also the
//     maximum |L_k[i][c]| over the lower triangle they read (the split-f16 image's scale
//     bound, absmax_kernel<1>'s result);
//   - one fragment of the split-f16 image of L_k = tril(q_sqrt[k]) (split_tri_kernel,
//     split3.hip).
// Reference: models.py:79 (prior_kl -> gauss_kl(q_mu, q_sqrt) whitened) and the q_sqrt
// operand of base_conditional (models.py:141-143).
#pragma once

#include "mgp_common.hpp"

namespace mgp {

constexpr int kKlRows = 16;   // rows of one L_k per KL block

struct KlPartial {
  float tr, ld, mh, amax;
};

// Thread t of nthr of KL block blk: blk < K * nRowBlocks: kKlRows rows of one L_k, sum of x^2
// over its lower triangle (tr), sum of log(x_ii^2) (ld), max |x| (amax); blk == K * nRowBlocks:
// sum of q_mu^2 (mh).  Each thread owns 4 consecutive columns of every row of the block
// (float4 loads of all the rows issued before any use).
__device__ __forceinline__ KlPartial kl_partials_thread(const float* __restrict__ q_mu, int64_t ldq,
                                                        const float* __restrict__ q_sqrt, int64_t ldqs,
                                                        int64_t strideq, int64_t M, int K, int nRowBlocks, int blk,
                                                        int t, int nthr) {
  KlPartial r = {0.f, 0.f, 0.f, 0.f};
  if (blk < K * nRowBlocks) {
    const int k = blk / nRowBlocks;
    const int64_t r0 = (int64_t)(blk % nRowBlocks) * kKlRows;
    const float* L = q_sqrt + (int64_t)k * strideq;
    const int64_t rmax = min<int64_t>(r0 + kKlRows, M) - 1;  // last row of the block
    for (int64_t c0 = 4 * (int64_t)t; c0 <= rmax; c0 += 4 * (int64_t)nthr) {
      floatx4 v[kKlRows];
#pragma unroll
      for (int rr = 0; rr < kKlRows; ++rr) {
        const int64_t i = r0 + rr;
        v[rr] = (i <= rmax && c0 <= i) ? *reinterpret_cast<const floatx4*>(L + i * ldqs + c0)
                                       : floatx4{0.f, 0.f, 0.f, 0.f};
      }
#pragma unroll
      for (int rr = 0; rr < kKlRows; ++rr) {
        const int64_t i = r0 + rr;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float x = (c0 + e <= i) ? v[rr][e] : 0.f;
          r.tr = fmaf(x, x, r.tr);
          r.amax = fmaxf(r.amax, fabsf(x));
          if (c0 + e == i && i <= rmax) r.ld += logf(x * x);
        }
      }
    }
  } else {  // the last block: Mahalanobis term sum q_mu^2
    for (int64_t m = t; m < M; m += nthr)
      for (int k = 0; k < K; ++k) {
        const float v = q_mu[m * ldq + k];
        r.mh = fmaf(v, v, r.mh);
      }
  }
  return r;
}

// Thread t of nthr of the final KL sum over the nblk partial triples.
__device__ __forceinline__ void kl_final_thread(const double* __restrict__ p, int nblk, int t, int nthr, double& tr,
                                                double& ld, double& mh) {
  tr = ld = mh = 0.0;
  for (int i = t; i < nblk; i += nthr) {
    tr += p[3 * i];
    ld += p[3 * i + 1];
    mh += p[3 * i + 2];
  }
}

// Fragment f of the A-operand image of a batch of triangular matrices (split_tri_kernel):
// element (k-row m, row m') = S_b[m][m'] kept where m >= m' (LOWER) or m <= m'; one wave.
// bound != nullptr: split-f16 image scaled by 2^img_exp(*bound) (with its e4m3 plane).
template <bool LOWER, bool TRANS = false, bool FULL = false>
__device__ __forceinline__ void split_tri_frag(const float* __restrict__ src, int64_t ld, int64_t stride, int64_t M,
                                               int nmb, int nmk, int64_t f, int lane, bf16x8* __restrict__ img,
                                               const float* __restrict__ bound) {
  const int r = lane & 31, h = lane >> 5;
  const int mk = (int)(f % nmk);
  const int64_t kb = f / nmk;
  const int mb = (int)(kb % nmb);
  const int b = (int)(kb / nmb);
  const int64_t mc = 32 * (int64_t)mb + r;
  const float* S = src + (int64_t)b * stride;
  float v[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int64_t m = 16 * (int64_t)mk + kperm(h, j);
    const bool keep = FULL || (LOWER ? (m >= mc) : (m <= mc));
    v[j] = (m < M && mc < M && keep) ? S[TRANS ? mc * ld + m : m * ld + mc] : 0.f;
  }
  if (bound)
    store_split_f16<true>(img + f * 3 * 64 + lane, v, ldexpf(1.f, img_exp(*bound)));
  else
    store_split(img + f * 3 * 64 + lane, v);
}

}  // namespace mgp
