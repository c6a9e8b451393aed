// K6 / K7 and the small epilogues of the SMGP ELBO.
//
// K6  mgp_elbo_terms: the Monte-Carlo data term.  Reference:
//       SMGP.W_dist (models.py:55-61), reparameterize (utils.py:26-27),
//       RelaxedOneHotCategorical(1e-2).sample (models.py:60,73-74; TFP 0.18
//       ExpRelaxedOneHotCategorical._sample_n + Exp bijector),
//       GaussianModified._variational_expectations (likelihoods.py:39-41) via
//       BroadcastingLikelihood (broadcasting_lik.py:23-24,39-42),
//       E_log_p_Y (models.py:63-67) and the batch mean (models.py:76).
//     One thread per data point n: the K expert var-exps are S-invariant and
//     computed once; the S samples are a running (online) logsumexp, so
//     neither W [S,N,K] nor the logits are ever materialised.  Noise is drawn
//     in-register from Philox4x32-10 keyed by the GLOBAL index (shard
//     invariant) or read from explicit arrays (parity mode).
//     Reduction: wave shuffles -> one partial per workgroup -> one-block
//     double-precision final sum (deterministic, no atomics).
// K7  mgp_gauss_kl_white: GPflow gauss_kl(q_mu, q_sqrt) whitened (models.py:79),
//     a streaming reduction over the packed lower triangle of each L_k.
#include <math.h>

#include <algorithm>

#include "mgp_common.hpp"
#include "qsqrt_jobs.hpp"

namespace mgp {

constexpr int kElboThreads = 256;

// z ~ N(0,1), u ~ U(0,1) of sample s, point n: explicit arrays [S][N][K] or
// Philox4x32-10 keyed by (global n, s, k / 4, stream 0 = z / 1 = u).
template <int KMAX>
__device__ __forceinline__ void draw_noise(float (&z)[KMAX], float (&u)[KMAX], const float* __restrict__ noise_z,
                                           const float* __restrict__ noise_u, int64_t N, int K, int64_t n, int s,
                                           uint32_t ng, uint32_t key0, uint32_t key1) {
  if (noise_z != nullptr) {
    const float* pz = noise_z + ((int64_t)s * N + n) * K;
    const float* pu = noise_u + ((int64_t)s * N + n) * K;
#pragma unroll
    for (int k = 0; k < KMAX; ++k) {
      z[k] = (k < K) ? pz[k] : 0.f;
      u[k] = (k < K) ? pu[k] : 0.5f;
    }
  } else {
#pragma unroll
    for (int kb = 0; kb < (KMAX + 3) / 4; ++kb) {
      if (4 * kb >= K) break;
      const u32x4 wz = philox4x32_10(u32x4{ng, (uint32_t)s, (uint32_t)kb, 0u}, key0, key1);
      const u32x4 wu = philox4x32_10(u32x4{ng, (uint32_t)s, (uint32_t)kb, 1u}, key0, key1);
      float zz[4];
      box_muller4(wz, zz);
      const uint32_t uw[4] = {wu.x, wu.y, wu.z, wu.w};
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        if (4 * kb + e < KMAX) {
          z[4 * kb + e] = zz[e];
          u[4 * kb + e] = u01(uw[e]);
        }
      }
    }
  }
}

// ------------------------------------------------------------------ MultiClass / RobustMax
// GPflow 2.7.0 likelihoods.MultiClass(num_classes = K, invlink = RobustMax(K))
// (gpflow pinned at environment.yml:95, not vendored), the pred likelihood of the
// multiclass demos (demos/demo_tf2_modified_multiclass.py:43-45), reached through
// BroadcastingLikelihood's flatten path (broadcasting_lik.py:19-37,39-42) from
// E_log_p_Y (models.py:63-67,113-120):
//   p    = RobustMax.prob_is_largest(y, mu, var): 20-point Gauss-Hermite over the
//          selected latent, X_g = mu_y + x_g sqrt(2 var_y),
//          p = sum_g w_g / sqrt(pi) prod_{k != y} [(1 - 2e-6) Phi((X_g - mu_k) / sqrt(var_k)) + 1e-6]
//          (safe_sqrt: square roots of max(., 1e-10); a label outside [0, K) selects nothing)
//   ve   = p log(1 - eps) + (1 - p) log(eps / (K - 1))
// ve is one value per point; the reference multiplies it by W [S, N, K] and sums
// over K, so the sample mixture is l_s = ve sum_k W_sk.
__constant__ float kGHx[20] = {
    -5.387480890e+00f, -4.603682450e+00f, -3.944764040e+00f, -3.347854567e+00f, -2.788806058e+00f,
    -2.254974002e+00f, -1.738537712e+00f, -1.234076215e+00f, -7.374737285e-01f, -2.453407083e-01f,
    2.453407083e-01f,  7.374737285e-01f,  1.234076215e+00f,  1.738537712e+00f,  2.254974002e+00f,
    2.788806058e+00f,  3.347854567e+00f,  3.944764040e+00f,  4.603682450e+00f,  5.387480890e+00f};
__constant__ float kGHc[20] = {  // w_g / sqrt(pi)
    1.257800672e-13f, 2.482062362e-10f, 6.127490260e-08f, 4.402121090e-06f, 1.288262800e-04f,
    1.830103131e-03f, 1.399783745e-02f, 6.150637206e-02f, 1.617393340e-01f, 2.607930634e-01f,
    2.607930634e-01f, 1.617393340e-01f, 6.150637206e-02f, 1.399783745e-02f, 1.830103131e-03f,
    1.288262800e-04f, 4.402121090e-06f, 6.127490260e-08f, 2.482062362e-10f, 1.257800672e-13f};

// p and (GRAD) dp/dmu[k], dp/dvar[k] for label y over the first K latents.
template <int KMAX, bool GRAD>
__device__ __forceinline__ float robustmax_p(int y, const float (&mu)[KMAX], const float (&var)[KMAX], int K,
                                             float (&dmu)[KMAX], float (&dvar)[KMAX]) {
  constexpr float kSq = 1e-6f, kKeep = 1.f - 2e-6f, kRsqrt2 = 0.70710678118654752f;
  constexpr float kInvSqrt2Pi = 0.39894228040143268f;
  float mus = 0.f, vs = 0.f, rs[KMAX];
#pragma unroll
  for (int k = 0; k < KMAX; ++k) {
    if (k == y) { mus = mu[k]; vs = var[k]; }
    rs[k] = (k < K) ? 1.f / sqrtf(fmaxf(var[k], 1e-10f)) : 0.f;
    if constexpr (GRAD) { dmu[k] = 0.f; dvar[k] = 0.f; }
  }
  const float sx = sqrtf(fmaxf(2.f * vs, 1e-10f));
  float p = 0.f, gsel = 0.f, gselx = 0.f;
  for (int g = 0; g < 20; ++g) {
    const float X = fmaf(kGHx[g], sx, mus);
    float d[KMAX], C[KMAX], prod = 1.f;
#pragma unroll
    for (int k = 0; k < KMAX; ++k) {
      if (k < K && k != y) {
        d[k] = (X - mu[k]) * rs[k];
        C[k] = fmaf(kKeep, 0.5f * erfcf(-d[k] * kRsqrt2), kSq);
        prod *= C[k];
      }
    }
    p = fmaf(kGHc[g], prod, p);
    if constexpr (GRAD) {
      float acc = 0.f;
#pragma unroll
      for (int k = 0; k < KMAX; ++k) {
        if (k < K && k != y) {
          // c_g prod_{j != k} C_j (1 - 2e-6) phi(d_k) / sqrt(var_k)
          const float t = kGHc[g] * (prod / C[k]) * kKeep * kInvSqrt2Pi * __expf(-0.5f * d[k] * d[k]) * rs[k];
          dmu[k] -= t;
          if (var[k] > 1e-10f) dvar[k] -= 0.5f * t * d[k] * rs[k];
          acc += t;
        }
      }
      gsel += acc;
      gselx = fmaf(acc, kGHx[g], gselx);
    }
  }
  if constexpr (GRAD) {
#pragma unroll
    for (int k = 0; k < KMAX; ++k) {
      if (k == y) {
        dmu[k] = gsel;
        dvar[k] = (2.f * vs > 1e-10f) ? gselx / sx : 0.f;
      }
    }
  }
  return p;
}

// Load the K latents of point n (expert-major [K][ldf]).
template <int KMAX>
__device__ __forceinline__ void load_latents(const float* __restrict__ mu_f, const float* __restrict__ var_f,
                                             int64_t ldf, int64_t n, int K, float (&mu)[KMAX],
                                             float (&var)[KMAX]) {
#pragma unroll
  for (int k = 0; k < KMAX; ++k) {
    mu[k] = (k < K) ? mu_f[(int64_t)k * ldf + n] : 0.f;
    var[k] = (k < K) ? var_f[(int64_t)k * ldf + n] : 1.f;
  }
}

// MOD: SMGPModified.E_log_p_Y (models.py:112-123) -- a second Gaussian
// var-exp of the assignment layer (likelihood variances lik_var_a) weighted by
// the same W, with its own logsumexp over S: lse_S(sum_k W ve_a) + lse_S(sum_k W ve_f) - 2 log S.
// MC: the pred likelihood is MultiClass/RobustMax (mc_a = log(1 - eps),
// mc_b = log(eps / (K - 1)); lik_var unused): ve_k = the point's RobustMax var-exp.
// LANES consecutive lanes share a point: lane `sub` takes the samples s = sub (mod
// LANES) and the lanes' running (max, sum) pairs are merged by shuffles (a point per
// thread left 65536 threads -- one wave per SIMD -- for the latency-bound Philox /
// transcendental chain at c3).
template <int LANES>
__device__ __forceinline__ void lse_merge(float& run_max, float& run_sum) {
#pragma unroll
  for (int off = 1; off < LANES; off <<= 1) {
    const float om = __shfl_xor(run_max, off, 64), os = __shfl_xor(run_sum, off, 64);
    const float m = fmaxf(run_max, om);
    if (m != -INFINITY) run_sum = run_sum * __expf(run_max - m) + os * __expf(om - m);
    run_max = m;
  }
}

template <int KMAX, bool MOD, bool MC, int LANES>
__global__ __launch_bounds__(kElboThreads) void elbo_terms_kernel(
    const float* __restrict__ mu_f, const float* __restrict__ var_f, const float* __restrict__ mu_a,
    const float* __restrict__ var_a, int64_t ldf, const float* __restrict__ Y,
    const float* __restrict__ lik_var, const float* __restrict__ lik_var_a, int64_t N, int K, int S,
    float inv_tau, float jitter,
    const float* __restrict__ noise_z, const float* __restrict__ noise_u, uint32_t key0,
    uint32_t key1, int64_t n_offset, double* __restrict__ partials, float mc_a, float mc_b) {
  __shared__ double scratch[16];
  const int64_t gt = (int64_t)blockIdx.x * kElboThreads + threadIdx.x;
  const int64_t n = gt / LANES;
  const int sub = (int)(gt % LANES);
  float val = 0.f;
  float run_max = -INFINITY, run_sum = 0.f, run_max_a = -INFINITY, run_sum_a = 0.f;
  if (n < N) {
    const float kHalfLog2Pi = 0.91893853320467274f;
    float ve[KMAX], ma[KMAX], sa[KMAX], vea[MOD ? KMAX : 1];
    const float y = Y[n];
    float vemc = 0.f;
    if constexpr (MC) {
      float mu[KMAX], var[KMAX], dm[KMAX], dv[KMAX];
      load_latents<KMAX>(mu_f, var_f, ldf, n, K, mu, var);
      const float p = robustmax_p<KMAX, false>((int)y, mu, var, K, dm, dv);
      vemc = fmaf(p, mc_a - mc_b, mc_b);
    }
#pragma unroll
    for (int k = 0; k < KMAX; ++k) {
      if (k < K) {
        if constexpr (MC) {
          ve[k] = vemc;
        } else {
          const float s2 = lik_var[k];
          const float d = y - mu_f[(int64_t)k * ldf + n];
          ve[k] = -kHalfLog2Pi - 0.5f * logf(s2) - 0.5f * (d * d + var_f[(int64_t)k * ldf + n]) / s2;
        }
        ma[k] = mu_a[(int64_t)k * ldf + n];
        const float va = var_a[(int64_t)k * ldf + n];
        // max(va + jitter, 0): a float32 marginal variance can round below -jitter
        // where the reference's float64 one sits at ~0 (the sqrt would be NaN); on
        // (-jitter, 0] the value is the reference's sqrt(va + jitter) (utils.py:27)
        sa[k] = sqrtf(fmaxf(va + jitter, 0.f));
        if constexpr (MOD) {
          const float s2a = lik_var_a[k];
          const float da = y - ma[k];
          vea[k] = -kHalfLog2Pi - 0.5f * logf(s2a) - 0.5f * (da * da + va) / s2a;
        }
      } else {
        ve[k] = 0.f; ma[k] = 0.f; sa[k] = 0.f;
        if constexpr (MOD) vea[k] = 0.f;
      }
    }
    const uint32_t ng = (uint32_t)(n + n_offset);
    for (int s = sub; s < S; s += LANES) {
      float z[KMAX], u[KMAX];
      draw_noise<KMAX>(z, u, noise_z, noise_u, N, K, n, s, ng, key0, key1);
      float x[KMAX], xm = -INFINITY;
#pragma unroll
      for (int k = 0; k < KMAX; ++k) {
        if (k < K) {
          const float g = -logf(-logf(u[k]));
          x[k] = (g + fmaf(z[k], sa[k], ma[k])) * inv_tau;
          xm = fmaxf(xm, x[k]);
        }
      }
      float den = 0.f, num = 0.f, numa = 0.f;
#pragma unroll
      for (int k = 0; k < KMAX; ++k) {
        if (k < K) {
          const float e = __expf(x[k] - xm);
          den += e;
          num = fmaf(e, ve[k], num);
          if constexpr (MOD) numa = fmaf(e, vea[k], numa);
        }
      }
      const float l = num / den;
      if (l > run_max) {
        run_sum = run_sum * __expf(run_max - l) + 1.f;
        run_max = l;
      } else {
        run_sum += __expf(l - run_max);
      }
      if constexpr (MOD) {
        const float la = numa / den;
        if (la > run_max_a) {
          run_sum_a = run_sum_a * __expf(run_max_a - la) + 1.f;
          run_max_a = la;
        } else {
          run_sum_a += __expf(la - run_max_a);
        }
      }
    }
  }
  if constexpr (LANES > 1) {  // every lane of the wave takes part (points beyond N included)
    lse_merge<LANES>(run_max, run_sum);
    if constexpr (MOD) lse_merge<LANES>(run_max_a, run_sum_a);
  }
  if (n < N && sub == 0) {
    val = run_max + logf(run_sum) - logf((float)S);
    if constexpr (MOD) val += run_max_a + logf(run_sum_a) - logf((float)S);
  }
  const double bs = block_sum<double>((double)val, scratch);
  if (threadIdx.x == 0) partials[blockIdx.x] = bs;
}

// ------------------------------------------------------------------ K6 backward
// Gradient of the data term of one point, DT_n = lse_s(l_s) - log S with
// l_s = sum_k W_sk ve_k (MOD: + lse_s(la_s) - log S, la_s = sum_k W_sk ve^a_k),
// W_s = softmax_k(x_s), x_sk = (g_sk + mu_a,k + z_sk sqrt(v_a,k + jitter)) / tau:
//   dDT/dve_k   = om_k = sum_s pi_s W_sk,            pi_s = exp(l_s - lse)
//   dDT/dx_sk   = pi_s W_sk (ve_k - l_s)             (softmax Jacobian)
//   dDT/dmu_f   = om_k (y - mu_f,k) / s2_k,  dDT/dvar_f = -om_k / (2 s2_k)
//   dDT/dmu_a   = sum_s dDT/dx_sk / tau,     dDT/dvar_a = sum_s dDT/dx_sk z_sk / (2 tau sqrt(v_a,k + jitter))
//   dDT/ds2_k   = om_k (-1/(2 s2_k) + ((y - mu_f,k)^2 + var_f,k) / (2 s2_k^2))
// (MOD adds the same terms of the assignment var-exp to the mu_a / var_a / s2^a
// gradients).  Two passes over the samples with the noise redrawn (Philox is
// counter-based): the first finds lse, the second accumulates.  Outputs are
// multiplied by `scale` (1 / N_total for the ELBO's batch mean).
// MC: dDT/dve_mc = sum_k om_k, chained through robustmax_p's gradient; no
// likelihood-variance gradient (MultiClass has no trainable parameter).
// LANES lanes per point as the forward: the lanes split the samples of both passes,
// merge the log-sum-exp pairs after pass 1 and sum the per-sample accumulators after
// pass 2 (butterfly shuffles, so every lane ends with the totals); lane 0 writes.
template <int LANES>
__device__ __forceinline__ float lanes_sum(float v) {
#pragma unroll
  for (int off = 1; off < LANES; off <<= 1) v += __shfl_xor(v, off, 64);
  return v;
}

template <int KMAX, bool MOD, bool MC, int LANES>
__global__ __launch_bounds__(kElboThreads) void elbo_terms_bwd_kernel(
    const float* __restrict__ mu_f, const float* __restrict__ var_f, const float* __restrict__ mu_a,
    const float* __restrict__ var_a, int64_t ldf, const float* __restrict__ Y,
    const float* __restrict__ lik_var, const float* __restrict__ lik_var_a, int64_t N, int K, int S,
    float inv_tau, float jitter, const float* __restrict__ noise_z, const float* __restrict__ noise_u,
    uint32_t key0, uint32_t key1, int64_t n_offset, float scale, float* __restrict__ G, int64_t ldg,
    double* __restrict__ partials, float mc_a, float mc_b) {
  __shared__ double scratch[16];
  const int64_t gt = (int64_t)blockIdx.x * kElboThreads + threadIdx.x;
  const int64_t n = gt / LANES;
  const int sub = (int)(gt % LANES);
  float glv[KMAX], glva[MOD ? KMAX : 1];
#pragma unroll
  for (int k = 0; k < KMAX; ++k) glv[k] = 0.f;
  if constexpr (MOD) {
#pragma unroll
    for (int k = 0; k < KMAX; ++k) glva[k] = 0.f;
  }
  // (LANES > 1: a point beyond N is computed for the last valid one, so that all lanes
  // of the wave take part in the shuffles, and not written)
  if (LANES > 1 || n < N) {
    const int64_t n = (gt / LANES < N) ? gt / LANES : N - 1;
    const float kHalfLog2Pi = 0.91893853320467274f;
    const float y = Y[n];
    float ve[KMAX], ma[KMAX], sa[KMAX], vea[MOD ? KMAX : 1];
    float mcm[MC ? KMAX : 1], mcv[MC ? KMAX : 1], dpm[MC ? KMAX : 1], dpv[MC ? KMAX : 1], vemc = 0.f;
    if constexpr (MC) {
      load_latents<KMAX>(mu_f, var_f, ldf, n, K, mcm, mcv);
      const float p = robustmax_p<KMAX, true>((int)y, mcm, mcv, K, dpm, dpv);
      vemc = fmaf(p, mc_a - mc_b, mc_b);
    }
#pragma unroll
    for (int k = 0; k < KMAX; ++k) {
      if (k < K) {
        if constexpr (MC) {
          ve[k] = vemc;
        } else {
          const float s2 = lik_var[k];
          const float d = y - mu_f[(int64_t)k * ldf + n];
          ve[k] = -kHalfLog2Pi - 0.5f * logf(s2) - 0.5f * (d * d + var_f[(int64_t)k * ldf + n]) / s2;
        }
        ma[k] = mu_a[(int64_t)k * ldf + n];
        const float va = var_a[(int64_t)k * ldf + n];
        sa[k] = sqrtf(fmaxf(va + jitter, 0.f));  // as in the forward
        if constexpr (MOD) {
          const float s2a = lik_var_a[k];
          const float da = y - ma[k];
          vea[k] = -kHalfLog2Pi - 0.5f * logf(s2a) - 0.5f * (da * da + va) / s2a;
        }
      } else {
        ve[k] = 0.f; ma[k] = 0.f; sa[k] = 1.f;
        if constexpr (MOD) vea[k] = 0.f;
      }
    }
    const uint32_t ng = (uint32_t)(n + n_offset);
    // sample s: softmax weights W and the two mixtures l, la
    auto sample = [&](int s, float (&z)[KMAX], float (&W)[KMAX], float& l, float& la) {
      float u[KMAX];
      draw_noise<KMAX>(z, u, noise_z, noise_u, N, K, n, s, ng, key0, key1);
      float xm = -INFINITY;
#pragma unroll
      for (int k = 0; k < KMAX; ++k) {
        if (k < K) {
          const float g = -logf(-logf(u[k]));
          W[k] = (g + fmaf(z[k], sa[k], ma[k])) * inv_tau;
          xm = fmaxf(xm, W[k]);
        }
      }
      float den = 0.f;
#pragma unroll
      for (int k = 0; k < KMAX; ++k) {
        if (k < K) {
          W[k] = __expf(W[k] - xm);
          den += W[k];
        } else {
          W[k] = 0.f;
        }
      }
      const float rden = 1.f / den;
      l = 0.f;
      la = 0.f;
#pragma unroll
      for (int k = 0; k < KMAX; ++k) {
        W[k] *= rden;
        l = fmaf(W[k], ve[k], l);
        if constexpr (MOD) la = fmaf(W[k], vea[k], la);
      }
    };
    // pass 1: log-sum-exp over the samples
    float mx = -INFINITY, sm = 0.f, mxa = -INFINITY, sma = 0.f;
    for (int s = sub; s < S; s += LANES) {
      float z[KMAX], W[KMAX], l, la;
      sample(s, z, W, l, la);
      if (l > mx) { sm = sm * __expf(mx - l) + 1.f; mx = l; } else { sm += __expf(l - mx); }
      if constexpr (MOD) {
        if (la > mxa) { sma = sma * __expf(mxa - la) + 1.f; mxa = la; } else { sma += __expf(la - mxa); }
      }
    }
    if constexpr (LANES > 1) {
      lse_merge<LANES>(mx, sm);
      if constexpr (MOD) lse_merge<LANES>(mxa, sma);
    }
    const float lse = mx + logf(sm), lsea = MOD ? mxa + logf(sma) : 0.f;
    // pass 2: accumulate
    float om[KMAX], oma[MOD ? KMAX : 1], gx[KMAX], gxz[KMAX];
#pragma unroll
    for (int k = 0; k < KMAX; ++k) {
      om[k] = 0.f; gx[k] = 0.f; gxz[k] = 0.f;
      if constexpr (MOD) oma[k] = 0.f;
    }
    for (int s = sub; s < S; s += LANES) {
      float z[KMAX], W[KMAX], l, la;
      sample(s, z, W, l, la);
      const float pi = __expf(l - lse);
      const float pia = MOD ? __expf(la - lsea) : 0.f;
#pragma unroll
      for (int k = 0; k < KMAX; ++k) {
        const float pw = pi * W[k];
        om[k] += pw;
        float t = pw * (ve[k] - l);
        if constexpr (MOD) {
          const float pwa = pia * W[k];
          oma[k] += pwa;
          t = fmaf(pwa, vea[k] - la, t);
        }
        gx[k] += t;
        gxz[k] = fmaf(t, z[k], gxz[k]);
      }
    }
    if constexpr (LANES > 1) {
#pragma unroll
      for (int k = 0; k < KMAX; ++k) {
        om[k] = lanes_sum<LANES>(om[k]);
        gx[k] = lanes_sum<LANES>(gx[k]);
        gxz[k] = lanes_sum<LANES>(gxz[k]);
        if constexpr (MOD) oma[k] = lanes_sum<LANES>(oma[k]);
      }
    }
    const bool writer = sub == 0 && gt / LANES < N;
    float gve_mc = 0.f;
    if constexpr (MC) {
#pragma unroll
      for (int k = 0; k < KMAX; ++k) gve_mc += (k < K) ? om[k] : 0.f;
      gve_mc *= scale * (mc_a - mc_b);
    }
#pragma unroll
    for (int k = 0; k < KMAX; ++k) {
      if (k < K && writer) {
        float gma = gx[k] * inv_tau;
        float gva = (var_a[(int64_t)k * ldf + n] + jitter > 0.f) ? gxz[k] * inv_tau * 0.5f / sa[k] : 0.f;
        float gmf, gvf;
        if constexpr (MC) {
          gmf = gve_mc * dpm[k];
          gvf = gve_mc * dpv[k];
        } else {
          const float s2 = lik_var[k];
          const float mf = mu_f[(int64_t)k * ldf + n], vf = var_f[(int64_t)k * ldf + n];
          const float d = y - mf;
          glv[k] = scale * om[k] * (-0.5f / s2 + 0.5f * (d * d + vf) / (s2 * s2));
          gmf = scale * om[k] * d / s2;
          gvf = -0.5f * scale * om[k] / s2;
        }
        if constexpr (MOD) {
          const float s2a = lik_var_a[k];
          const float da = y - ma[k];
          const float va = var_a[(int64_t)k * ldf + n];
          gma = fmaf(oma[k], da / s2a, gma);
          gva -= 0.5f * oma[k] / s2a;
          glva[k] = scale * oma[k] * (-0.5f / s2a + 0.5f * (da * da + va) / (s2a * s2a));
        }
        G[(int64_t)(0 * K + k) * ldg + n] = gmf;
        G[(int64_t)(1 * K + k) * ldg + n] = gvf;
        G[(int64_t)(2 * K + k) * ldg + n] = scale * gma;
        G[(int64_t)(3 * K + k) * ldg + n] = scale * gva;
      }
    }
  }
  // block partials of the likelihood-variance gradients: [block][2 * KMAX]
#pragma unroll
  for (int k = 0; k < KMAX; ++k) {
    if (k >= K) break;
    const double v = block_sum<double>((double)glv[k], scratch);
    if (threadIdx.x == 0) partials[(int64_t)blockIdx.x * 2 * KMAX + k] = v;
    if constexpr (MOD) {
      const double va = block_sum<double>((double)glva[k], scratch);
      if (threadIdx.x == 0) partials[(int64_t)blockIdx.x * 2 * KMAX + KMAX + k] = va;
    }
  }
}

// out[c] = sum_b p[b * stride + c] for c < C (one workgroup per c).
__global__ __launch_bounds__(256) void column_sums_kernel(const double* __restrict__ p, int nb, int64_t stride,
                                                          double* __restrict__ out, int64_t out_stride) {
  __shared__ double scratch[16];
  const int c = blockIdx.x;
  double v = 0.0;
  for (int b = threadIdx.x; b < nb; b += blockDim.x) v += p[(int64_t)b * stride + c];
  v = block_sum<double>(v, scratch);
  if (threadIdx.x == 0) out[(int64_t)c * out_stride] = v;
}

__global__ __launch_bounds__(1024) void sum_partials_kernel(const double* __restrict__ p, int n,
                                                            double* __restrict__ out) {
  __shared__ double scratch[16];
  double v = 0.0;
  for (int i = threadIdx.x; i < n; i += blockDim.x) v += p[i];
  v = block_sum<double>(v, scratch);
  if (threadIdx.x == 0) *out = v;
}

// ------------------------------------------------------------------ K7
// Block = kKlRows rows of one L_k, or (the last block) the q_mu term; the body is shared with
// the two-layer launches of mgp_qsqrt_images_kl_f16_batch (qsqrt_jobs.hpp).
__global__ __launch_bounds__(256) void kl_partials_kernel(const float* __restrict__ q_mu, int64_t ldq,
                                                          const float* __restrict__ q_sqrt,
                                                          int64_t ldqs, int64_t strideq, int64_t M,
                                                          int K, int nRowBlocks,
                                                          double* __restrict__ partials) {
  __shared__ double scratch[16];
  const int blk = blockIdx.x;
  const KlPartial r = kl_partials_thread(q_mu, ldq, q_sqrt, ldqs, strideq, M, K, nRowBlocks, blk, threadIdx.x, 256);
  const double a = block_sum<double>((double)r.tr, scratch);
  const double b = block_sum<double>((double)r.ld, scratch);
  const double c = block_sum<double>((double)r.mh, scratch);
  if (threadIdx.x == 0) {
    partials[3 * blk + 0] = a;
    partials[3 * blk + 1] = b;
    partials[3 * blk + 2] = c;
  }
}

__global__ __launch_bounds__(1024) void kl_final_kernel(const double* __restrict__ p, int nblk,
                                                        double MK, double* __restrict__ out) {
  __shared__ double scratch[16];
  double tr, ld, mh;
  kl_final_thread(p, nblk, threadIdx.x, blockDim.x, tr, ld, mh);
  tr = block_sum<double>(tr, scratch);
  ld = block_sum<double>(ld, scratch);
  mh = block_sum<double>(mh, scratch);
  if (threadIdx.x == 0) *out = 0.5 * (mh - MK - ld + tr);
}

__global__ void elbo_combine_kernel(const double* data_sum, const double* kl_f, const double* kl_a,
                                    double n_batch, double num_data, float* out, double* out64) {
  const double e = *data_sum / n_batch - (*kl_f + *kl_a) / num_data;
  if (out) *out = (float)e;
  if (out64) *out64 = e;
}

__global__ __launch_bounds__(256) void predict_epilogue_kernel(
    const float* __restrict__ fmean, const float* __restrict__ fvar, const float* __restrict__ amean,
    int64_t ldf, const float* __restrict__ lik_var, int64_t N, int K, float* __restrict__ y_mean,
    float* __restrict__ y_var, float* __restrict__ assign) {
  const int64_t n = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (n >= N) return;
  for (int k = 0; k < K; ++k) {
    if (y_mean) y_mean[n * K + k] = fmean[(int64_t)k * ldf + n];
    if (y_var) y_var[n * K + k] = fvar[(int64_t)k * ldf + n] + lik_var[k];
  }
  if (assign) {
    float m = -INFINITY;
    for (int k = 0; k < K; ++k) m = fmaxf(m, amean[(int64_t)k * ldf + n]);
    float den = 0.f;
    for (int k = 0; k < K; ++k) den += __expf(amean[(int64_t)k * ldf + n] - m);
    for (int k = 0; k < K; ++k) assign[n * K + k] = __expf(amean[(int64_t)k * ldf + n] - m) / den;
  }
}

__global__ __launch_bounds__(256) void philox_noise_kernel(uint32_t key0, uint32_t key1,
                                                           int64_t n_offset, int64_t N, int K, int S,
                                                           float* __restrict__ z,
                                                           float* __restrict__ u) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= N * (int64_t)S) return;
  const int s = (int)(idx / N);
  const int64_t n = idx % N;
  const uint32_t ng = (uint32_t)(n + n_offset);
  for (int kb = 0; 4 * kb < K; ++kb) {
    const u32x4 wz = philox4x32_10(u32x4{ng, (uint32_t)s, (uint32_t)kb, 0u}, key0, key1);
    const u32x4 wu = philox4x32_10(u32x4{ng, (uint32_t)s, (uint32_t)kb, 1u}, key0, key1);
    float zz[4];
    box_muller4(wz, zz);
    const uint32_t uw[4] = {wu.x, wu.y, wu.z, wu.w};
    for (int e = 0; e < 4 && 4 * kb + e < K; ++e) {
      const int64_t o = ((int64_t)s * N + n) * K + 4 * kb + e;
      if (z) z[o] = zz[e];
      if (u) u[o] = u01(uw[e]);
    }
  }
}

// MultiClass._predict_mean_and_var (GPflow 2.7.0, via broadcasting_lik.py:44-46):
// ps[i] = p_i (1 - eps) + (1 - p_i) eps / (K - 1) with p_i = prob_is_largest(i, mu, var)
// for every class i; mean = ps, var = ps - ps^2.
template <int KMAX>
__device__ __forceinline__ void multiclass_ps(const float (&mu)[KMAX], const float (&var)[KMAX], int K,
                                              float keep, float other, float (&ps)[KMAX]) {
  float dm[KMAX], dv[KMAX];
#pragma unroll
  for (int i = 0; i < KMAX; ++i) {
    ps[i] = 0.f;
    if (i < K) {
      const float p = robustmax_p<KMAX, false>(i, mu, var, K, dm, dv);
      ps[i] = fmaf(p, keep - other, other);
    }
  }
}

template <int KMAX>
__global__ __launch_bounds__(256) void multiclass_predict_kernel(const float* __restrict__ fmean,
                                                                 const float* __restrict__ fvar, int64_t ldf,
                                                                 int64_t N, int K, float keep, float other,
                                                                 float* __restrict__ y_mean,
                                                                 float* __restrict__ y_var) {
  const int64_t n = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (n >= N) return;
  float mu[KMAX], var[KMAX], ps[KMAX];
  load_latents<KMAX>(fmean, fvar, ldf, n, K, mu, var);
  multiclass_ps<KMAX>(mu, var, K, keep, other, ps);
#pragma unroll
  for (int i = 0; i < KMAX; ++i) {
    if (i < K) {
      if (y_mean) y_mean[n * K + i] = ps[i];
      if (y_var) y_var[n * K + i] = ps[i] - ps[i] * ps[i];
    }
  }
}

// SMGP.predict_samples (models.py:91-103).  One thread per (s, n).
// MC: the likelihood's predictive mean / variance are MultiClass's (ps, ps - ps^2).
template <int KMAX, bool MC = false>
__global__ __launch_bounds__(256) void predict_samples_kernel(
    const float* __restrict__ mu_f, const float* __restrict__ var_f, const float* __restrict__ mu_a,
    const float* __restrict__ var_a, int64_t ldf, const float* __restrict__ lik_var, int64_t N, int K,
    int S, float inv_tau, float jitter, const float* __restrict__ zw_in, const float* __restrict__ uw_in,
    const float* __restrict__ zy_in, uint32_t key0, uint32_t key1, int64_t n_offset,
    float* __restrict__ sy, float* __restrict__ sf, float mc_keep = 0.f, float mc_other = 0.f) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= N * (int64_t)S) return;
  const int s = (int)(idx / N);
  const int64_t n = idx % N;
  const uint32_t ng = (uint32_t)(n + n_offset);
  float zw[KMAX], uw[KMAX], zy[KMAX];
  if (zw_in != nullptr) {
    const int64_t o = ((int64_t)s * N + n) * K;
#pragma unroll
    for (int k = 0; k < KMAX; ++k) {
      zw[k] = (k < K) ? zw_in[o + k] : 0.f;
      uw[k] = (k < K) ? uw_in[o + k] : 0.5f;
      zy[k] = (k < K) ? zy_in[o + k] : 0.f;
    }
  } else {
#pragma unroll
    for (int kb = 0; kb < (KMAX + 3) / 4; ++kb) {
      if (4 * kb >= K) break;
      const u32x4 a = philox4x32_10(u32x4{ng, (uint32_t)s, (uint32_t)kb, 0u}, key0, key1);
      const u32x4 b = philox4x32_10(u32x4{ng, (uint32_t)s, (uint32_t)kb, 1u}, key0, key1);
      const u32x4 c = philox4x32_10(u32x4{ng, (uint32_t)s, (uint32_t)kb, 2u}, key0, key1);
      float za[4], zc[4];
      box_muller4(a, za);
      box_muller4(c, zc);
      const uint32_t bw[4] = {b.x, b.y, b.z, b.w};
#pragma unroll
      for (int e = 0; e < 4; ++e)
        if (4 * kb + e < KMAX) {
          zw[4 * kb + e] = za[e];
          uw[4 * kb + e] = u01(bw[e]);
          zy[4 * kb + e] = zc[e];
        }
    }
  }
  float x[KMAX], xm = -INFINITY;
#pragma unroll
  for (int k = 0; k < KMAX; ++k)
    if (k < K) {
      const float logit = fmaf(zw[k], sqrtf(fmaxf(var_a[(int64_t)k * ldf + n] + jitter, 0.f)), mu_a[(int64_t)k * ldf + n]);
      x[k] = (-logf(-logf(uw[k])) + logit) * inv_tau;
      xm = fmaxf(xm, x[k]);
    }
  float ps[MC ? KMAX : 1];
  if constexpr (MC) {
    float mu[KMAX], var[KMAX];
    load_latents<KMAX>(mu_f, var_f, ldf, n, K, mu, var);
    multiclass_ps<KMAX>(mu, var, K, mc_keep, mc_other, ps);
  }
  float den = 0.f, ay = 0.f, af = 0.f;
#pragma unroll
  for (int k = 0; k < KMAX; ++k)
    if (k < K) {
      const float e = __expf(x[k] - xm);
      const float m = mu_f[(int64_t)k * ldf + n], v = var_f[(int64_t)k * ldf + n];
      den += e;
      if constexpr (MC)
        ay = fmaf(e, fmaf(zy[k], sqrtf(ps[k] - ps[k] * ps[k] + jitter), ps[k]), ay);
      else
        ay = fmaf(e, fmaf(zy[k], sqrtf(fmaxf(v + lik_var[k] + jitter, 0.f)), m), ay);
      af = fmaf(e, fmaf(zy[k], sqrtf(fmaxf(v + jitter, 0.f)), m), af);
    }
  if (sy) sy[(int64_t)s * N + n] = ay / den;
  if (sf) sf[(int64_t)s * N + n] = af / den;
}

__global__ __launch_bounds__(256) void philox_normal2_kernel(uint32_t key0, uint32_t key1,
                                                             int64_t n_offset, int64_t N, int K,
                                                             int S, float* __restrict__ z) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= N * (int64_t)S) return;
  const int s = (int)(idx / N);
  const int64_t n = idx % N;
  for (int kb = 0; 4 * kb < K; ++kb) {
    const u32x4 w = philox4x32_10(u32x4{(uint32_t)(n + n_offset), (uint32_t)s, (uint32_t)kb, 2u}, key0, key1);
    float zz[4];
    box_muller4(w, zz);
    for (int e = 0; e < 4 && 4 * kb + e < K; ++e) z[((int64_t)s * N + n) * K + 4 * kb + e] = zz[e];
  }
}

// ------------------------------------------------------------------ method-level API
// The pieces K6 fuses, as separate kernels for the reference's public methods.
// Latents are expert-major [K][ldf]; the sample s of point n sits in column
// s * stride_s + n (stride_s = 0: the S-invariant conditional of S tiled copies).
// Noise: explicit [S][N][K] arrays or the same Philox streams K6 draws (stream 0 =
// z, stream 1 = u, keyed by (global n, s, k / 4)), so W_dist(seed) -> sample ->
// E_log_p_Y reproduces _build_likelihood(seed).

// SMGP.W_dist's logits (models.py:56-59, utils.py:26-27):
// log_assign[s][n][k] = mu_a + z sqrt(var_a + jitter).  One thread per (s, n).
__global__ __launch_bounds__(256) void assign_logits_kernel(
    const float* __restrict__ mu_a, const float* __restrict__ var_a, int64_t ldf, int64_t stride_s, int64_t N,
    int K, int S, float jitter, const float* __restrict__ noise_z, uint32_t key0, uint32_t key1,
    int64_t n_offset, float* __restrict__ logits) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= N * (int64_t)S) return;
  const int s = (int)(idx / N);
  const int64_t n = idx % N, col = (int64_t)s * stride_s + n, o = idx * K;
  const uint32_t ng = (uint32_t)(n + n_offset);
  for (int kb = 0; 4 * kb < K; ++kb) {
    float zz[4];
    if (noise_z == nullptr) box_muller4(philox4x32_10(u32x4{ng, (uint32_t)s, (uint32_t)kb, 0u}, key0, key1), zz);
    for (int e = 0; e < 4 && 4 * kb + e < K; ++e) {
      const int k = 4 * kb + e;
      const float z = noise_z ? noise_z[o + k] : zz[e];
      logits[o + k] = fmaf(z, sqrtf(fmaxf(var_a[(int64_t)k * ldf + col] + jitter, 0.f)),
                           mu_a[(int64_t)k * ldf + col]);
    }
  }
}

// RelaxedOneHotCategorical(temperature, logits).sample() (TFP 0.18,
// models.py:60,73): W = exp(log_softmax((g + logits) / tau)), g = -log(-log u),
// over rows r = s * N + n of logits [S * N][K].  One thread per row.
template <int KMAX>
__global__ __launch_bounds__(256) void relaxed_onehot_kernel(const float* __restrict__ logits, int64_t N, int K,
                                                             int S, float inv_tau,
                                                             const float* __restrict__ noise_u, uint32_t key0,
                                                             uint32_t key1, int64_t n_offset,
                                                             float* __restrict__ W) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= N * (int64_t)S) return;
  const int s = (int)(idx / N);
  const int64_t n = idx % N, o = idx * K;
  const uint32_t ng = (uint32_t)(n + n_offset);
  float x[KMAX], xm = -INFINITY;
#pragma unroll
  for (int kb = 0; kb < (KMAX + 3) / 4; ++kb) {
    if (4 * kb >= K) break;
    u32x4 w{0u, 0u, 0u, 0u};
    if (noise_u == nullptr) w = philox4x32_10(u32x4{ng, (uint32_t)s, (uint32_t)kb, 1u}, key0, key1);
    const uint32_t uw[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int k = 4 * kb + e;
      if (k < KMAX && k < K) {
        const float u = noise_u ? noise_u[o + k] : u01(uw[e]);
        x[k] = (-logf(-logf(u)) + logits[o + k]) * inv_tau;
        xm = fmaxf(xm, x[k]);
      }
    }
  }
  float den = 0.f;
#pragma unroll
  for (int k = 0; k < KMAX; ++k)
    if (k < K) {
      x[k] = __expf(x[k] - xm);
      den += x[k];
    }
  const float r = 1.f / den;
#pragma unroll
  for (int k = 0; k < KMAX; ++k)
    if (k < K) W[o + k] = x[k] * r;
}

// SMGP.E_log_p_Y(Xt, Y, W) (models.py:63-67): logsumexp_s(sum_k W ve) - log S per
// point; MOD: SMGPModified.E_log_p_Y (models.py:112-123), the assignment
// likelihood's var-exp on the assign latents adds its own logsumexp; MC: the pred
// likelihood is MultiClass / RobustMax (ve is one value per (s, n), times sum_k W).
template <int KMAX, bool MOD, bool MC>
__global__ __launch_bounds__(256) void e_log_p_y_kernel(
    const float* __restrict__ mu_f, const float* __restrict__ var_f, const float* __restrict__ mu_a,
    const float* __restrict__ var_a, int64_t ldf, int64_t stride_s, const float* __restrict__ Y,
    const float* __restrict__ lik_var, const float* __restrict__ lik_var_a, const float* __restrict__ W,
    int64_t N, int K, int S, float mc_a, float mc_b, float* __restrict__ out) {
  const int64_t n = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (n >= N) return;
  constexpr float kHalfLog2Pi = 0.91893853320467274f;
  const float y = Y[n];
  float mx = -INFINITY, sm = 0.f, mxa = -INFINITY, sma = 0.f;
  for (int s = 0; s < S; ++s) {
    const int64_t col = (int64_t)s * stride_s + n;
    const float* w = W + ((int64_t)s * N + n) * K;
    float l = 0.f, la = 0.f;
    if constexpr (MC) {
      float mu[KMAX], var[KMAX], dm[KMAX], dv[KMAX], ws = 0.f;
      load_latents<KMAX>(mu_f, var_f, ldf, col, K, mu, var);
      const float p = robustmax_p<KMAX, false>((int)y, mu, var, K, dm, dv);
      for (int k = 0; k < K; ++k) ws += w[k];
      l = fmaf(p, mc_a - mc_b, mc_b) * ws;
    } else {
      for (int k = 0; k < K; ++k) {
        const float s2 = lik_var[k], d = y - mu_f[(int64_t)k * ldf + col];
        l = fmaf(w[k], -kHalfLog2Pi - 0.5f * logf(s2) - 0.5f * (d * d + var_f[(int64_t)k * ldf + col]) / s2, l);
      }
    }
    if constexpr (MOD) {
      for (int k = 0; k < K; ++k) {
        const float s2 = lik_var_a[k], d = y - mu_a[(int64_t)k * ldf + col];
        la = fmaf(w[k], -kHalfLog2Pi - 0.5f * logf(s2) - 0.5f * (d * d + var_a[(int64_t)k * ldf + col]) / s2, la);
      }
    }
    if (l > mx) { sm = sm * __expf(mx - l) + 1.f; mx = l; } else { sm += __expf(l - mx); }
    if constexpr (MOD) {
      if (la > mxa) { sma = sma * __expf(mxa - la) + 1.f; mxa = la; } else { sma += __expf(la - mxa); }
    }
  }
  float v = mx + logf(sm) - logf((float)S);
  if constexpr (MOD) v += mxa + logf(sma) - logf((float)S);
  out[n] = v;
}

}  // namespace mgp

using namespace mgp;

extern "C" int mgp_assign_logits(const float* mu_a, const float* var_a, int64_t ldf, int64_t stride_s, int64_t N,
                                 int32_t K, int32_t S, float jitter, const float* noise_z, uint64_t seed,
                                 int64_t n_offset, float* logits, mgp_stream_t stream) {
  if (!mu_a) return -1;
  if (!var_a) return -2;
  if (ldf < (S > 1 ? stride_s * (S - 1) + N : N)) return -3;
  if (stride_s < 0) return -4;
  if (N < 0) return -5;
  if (K < 1) return -6;
  if (S < 1) return -7;
  if (!(jitter >= 0.f)) return -8;
  if (n_offset < 0) return -11;
  if (!logits) return -12;
  if (N == 0) return MGP_OK;
  const int64_t total = N * (int64_t)S;
  hipLaunchKernelGGL(assign_logits_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, mu_a, var_a, ldf, stride_s, N, K, S, jitter, noise_z,
                     (uint32_t)(seed & 0xffffffffu), (uint32_t)(seed >> 32), n_offset, logits);
  return launch_status();
}

extern "C" int mgp_relaxed_onehot_sample(const float* logits, int64_t N, int32_t K, int32_t S, float tau,
                                         const float* noise_u, uint64_t seed, int64_t n_offset, float* W,
                                         mgp_stream_t stream) {
  if (!logits) return -1;
  if (N < 0) return -2;
  if (K < 1) return -3;
  if (K > 32) return MGP_ERR_UNSUPPORTED;
  if (S < 1) return -4;
  if (!(tau > 0.f)) return -5;
  if (n_offset < 0) return -8;
  if (!W) return -9;
  if (N == 0) return MGP_OK;
  const int64_t total = N * (int64_t)S;
  const dim3 grid((unsigned)((total + 255) / 256)), block(256);
  const uint32_t k0 = (uint32_t)(seed & 0xffffffffu), k1 = (uint32_t)(seed >> 32);
  hipStream_t s = (hipStream_t)stream;
#define MGP_RO_CASE(KM)                                                                                        \
  if (K <= KM) {                                                                                                \
    hipLaunchKernelGGL(relaxed_onehot_kernel<KM>, grid, block, 0, s, logits, N, K, S, 1.f / tau, noise_u, k0, k1, \
                       n_offset, W);                                                                            \
  } else
  MGP_RO_CASE(4) MGP_RO_CASE(8) MGP_RO_CASE(16) MGP_RO_CASE(32) {}
#undef MGP_RO_CASE
  return launch_status();
}

extern "C" int mgp_e_log_p_y(const float* mu_f, const float* var_f, const float* mu_a, const float* var_a,
                             int64_t ldf, int64_t stride_s, const float* Y, const float* lik_var,
                             const float* assign_lik_var, float multiclass_eps, const float* W, int64_t N,
                             int32_t K, int32_t S, float* out, mgp_stream_t stream) {
  const bool mc = lik_var == nullptr, mod = assign_lik_var != nullptr;
  if (!mu_f) return -1;
  if (!var_f) return -2;
  if (mod && !mu_a) return -3;
  if (mod && !var_a) return -4;
  if (ldf < (S > 1 ? stride_s * (S - 1) + N : N)) return -5;
  if (stride_s < 0) return -6;
  if (!Y) return -7;
  if (mc && !(multiclass_eps > 0.f && multiclass_eps < 1.f)) return -10;
  if (!W) return -11;
  if (N < 0) return -12;
  if (K < 1 || (mc && K < 2)) return -13;
  if (K > 32) return MGP_ERR_UNSUPPORTED;
  if (S < 1) return -14;
  if (!out) return -15;
  if (N == 0) return MGP_OK;
  float a = 0.f, b = 0.f;
  if (mc) {
    a = logf(1.f - multiclass_eps);
    b = logf(multiclass_eps / (float)(K - 1));
  }
  const dim3 grid((unsigned)((N + 255) / 256)), block(256);
  hipStream_t s = (hipStream_t)stream;
#define MGP_ELPY(KM, MOD, MC)                                                                                  \
  hipLaunchKernelGGL((e_log_p_y_kernel<KM, MOD, MC>), grid, block, 0, s, mu_f, var_f, mu_a, var_a, ldf,        \
                     stride_s, Y, lik_var, assign_lik_var, W, N, K, S, a, b, out)
#define MGP_ELPY_CASE(KM)                                                                                      \
  if (K <= KM) {                                                                                                \
    if (mc && mod) MGP_ELPY(KM, true, true);                                                                    \
    else if (mc) MGP_ELPY(KM, false, true);                                                                     \
    else if (mod) MGP_ELPY(KM, true, false);                                                                    \
    else MGP_ELPY(KM, false, false);                                                                            \
  } else
  MGP_ELPY_CASE(4) MGP_ELPY_CASE(8) MGP_ELPY_CASE(16) MGP_ELPY_CASE(32) {}
#undef MGP_ELPY_CASE
#undef MGP_ELPY
  return launch_status();
}

static int predict_samples_run(const float* mu_f, const float* var_f, const float* mu_a, const float* var_a,
                               int64_t ldf, const float* lik_var, int64_t N, int32_t K, int32_t S, float tau,
                               float jitter, const float* noise_zw, const float* noise_uw, const float* noise_zy, uint64_t seed,
                               int64_t n_offset, float* samples_y, float* samples_f, hipStream_t s, bool mc,
                               float keep, float other) {
  if (N == 0) return MGP_OK;
  const int64_t total = N * (int64_t)S;
  const dim3 grid((unsigned)((total + 255) / 256)), block(256);
  const uint32_t k0 = (uint32_t)(seed & 0xffffffffu), k1 = (uint32_t)(seed >> 32);
#define MGP_PS_CASE(KM)                                                                                      \
  if (K <= KM) {                                                                                              \
    if (mc)                                                                                                   \
      hipLaunchKernelGGL((predict_samples_kernel<KM, true>), grid, block, 0, s, mu_f, var_f, mu_a, var_a, ldf, \
                         lik_var, N, K, S, 1.f / tau, jitter, noise_zw, noise_uw, noise_zy, k0, k1, n_offset, samples_y, \
                         samples_f, keep, other);                                                              \
    else                                                                                                      \
      hipLaunchKernelGGL((predict_samples_kernel<KM, false>), grid, block, 0, s, mu_f, var_f, mu_a, var_a,     \
                         ldf, lik_var, N, K, S, 1.f / tau, jitter, noise_zw, noise_uw, noise_zy, k0, k1, n_offset,     \
                         samples_y, samples_f, 0.f, 0.f);                                                      \
  } else
  MGP_PS_CASE(4) MGP_PS_CASE(8) MGP_PS_CASE(16) MGP_PS_CASE(32) {}
#undef MGP_PS_CASE
  return launch_status();
}

extern "C" int mgp_predict_samples(const float* mu_f, const float* var_f, const float* mu_a,
                                   const float* var_a, int64_t ldf, const float* lik_var, int64_t N,
                                   int32_t K, int32_t S, float tau, float jitter, const float* noise_zw,
                                   const float* noise_uw, const float* noise_zy, uint64_t seed,
                                   int64_t n_offset, float* samples_y, float* samples_f,
                                   mgp_stream_t stream) {
  if (!mu_f) return -1;
  if (!var_f) return -2;
  if (!mu_a) return -3;
  if (!var_a) return -4;
  if (ldf < N) return -5;
  if (!lik_var) return -6;
  if (N < 0) return -7;
  if (K < 1) return -8;
  if (K > 32) return MGP_ERR_UNSUPPORTED;
  if (S < 1) return -9;
  if (!(tau > 0.f)) return -10;
  if (!(jitter >= 0.f)) return -16;
  const bool any = noise_zw || noise_uw || noise_zy, all = noise_zw && noise_uw && noise_zy;
  if (any && !all) return -11;
  if (n_offset < 0) return -15;
  return predict_samples_run(mu_f, var_f, mu_a, var_a, ldf, lik_var, N, K, S, tau, jitter, noise_zw, noise_uw, noise_zy,
                             seed, n_offset, samples_y, samples_f, (hipStream_t)stream, false, 0.f, 0.f);
}

extern "C" int mgp_predict_samples_multiclass(const float* mu_f, const float* var_f, const float* mu_a,
                                              const float* var_a, int64_t ldf, float epsilon, int64_t N,
                                              int32_t K, int32_t S, float tau, float jitter, const float* noise_zw,
                                              const float* noise_uw, const float* noise_zy, uint64_t seed,
                                              int64_t n_offset, float* samples_y, float* samples_f,
                                              mgp_stream_t stream) {
  if (!mu_f) return -1;
  if (!var_f) return -2;
  if (!mu_a) return -3;
  if (!var_a) return -4;
  if (ldf < N) return -5;
  if (!(epsilon > 0.f && epsilon < 1.f)) return -6;
  if (N < 0) return -7;
  if (K < 2) return -8;
  if (K > 32) return MGP_ERR_UNSUPPORTED;
  if (S < 1) return -9;
  if (!(tau > 0.f)) return -10;
  if (!(jitter >= 0.f)) return -16;
  const bool any = noise_zw || noise_uw || noise_zy, all = noise_zw && noise_uw && noise_zy;
  if (any && !all) return -11;
  if (n_offset < 0) return -15;
  const float keep = 1.f - epsilon, other = (float)((double)epsilon / (double)(K - 1));
  return predict_samples_run(mu_f, var_f, mu_a, var_a, ldf, nullptr, N, K, S, tau, jitter, noise_zw, noise_uw, noise_zy,
                             seed, n_offset, samples_y, samples_f, (hipStream_t)stream, true, keep, other);
}

extern "C" int mgp_multiclass_predict(const float* fmean, const float* fvar, int64_t ldf, int64_t N, int32_t K,
                                      float epsilon, float* y_mean, float* y_var, mgp_stream_t stream) {
  if (!fmean) return -1;
  if (!fvar) return -2;
  if (ldf < N) return -3;
  if (N < 0) return -4;
  if (K < 2) return -5;
  if (K > 32) return MGP_ERR_UNSUPPORTED;
  if (!(epsilon > 0.f && epsilon < 1.f)) return -6;
  if (!y_mean && !y_var) return -7;
  if (N == 0) return MGP_OK;
  const float keep = 1.f - epsilon, other = (float)((double)epsilon / (double)(K - 1));
  const dim3 grid((unsigned)((N + 255) / 256)), block(256);
  hipStream_t s = (hipStream_t)stream;
#define MGP_MCP_CASE(KM)                                                                                  \
  if (K <= KM) {                                                                                           \
    hipLaunchKernelGGL(multiclass_predict_kernel<KM>, grid, block, 0, s, fmean, fvar, ldf, N, K, keep, other, \
                       y_mean, y_var);                                                                     \
  } else
  MGP_MCP_CASE(2) MGP_MCP_CASE(4) MGP_MCP_CASE(8) MGP_MCP_CASE(16) MGP_MCP_CASE(32) {}
#undef MGP_MCP_CASE
  return launch_status();
}

extern "C" int mgp_philox_normal2(uint64_t seed, int64_t n_offset, int64_t N, int32_t K, int32_t S,
                                  float* z, mgp_stream_t stream) {
  if (n_offset < 0) return -2;
  if (N < 0) return -3;
  if (K < 1) return -4;
  if (S < 1) return -5;
  if (!z) return -6;
  if (N == 0) return MGP_OK;
  const int64_t total = N * (int64_t)S;
  hipLaunchKernelGGL(philox_normal2_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, (uint32_t)(seed & 0xffffffffu), (uint32_t)(seed >> 32),
                     n_offset, N, K, S, z);
  return launch_status();
}

// K6 and its backward: kElboLanes lanes per point (MultiClass: one -- its per-point
// Gauss-Hermite var-exp and its gradient would be repeated by every lane)
constexpr int kElboLanes = 4;
// The backward keeps one lane per point: its lane-split form (LANES = 4, the samples'
// accumulators summed by shuffles) reorders the float32 sums of G, and the kernel
// variance gradients, differences of large Kuf / Kuu terms through the Cholesky
// backward, amplify that reordering past their test bound at small M (measured:
// assign.variance 9.6e-4 vs 6.8e-4 at N = 1000, M = 25, K = 3, D = 1).
#ifndef MGP_K6B_LANES
#define MGP_K6B_LANES 1
#endif
constexpr int kElboBwdLanes = MGP_K6B_LANES;
static int64_t elbo_fwd_blocks(int64_t N, int lanes) { return (N * lanes + kElboThreads - 1) / kElboThreads; }
// The forward's lanes per point by N: 4 from N = 65536 (c3: 262144 threads), 8 or 16 below,
// so that a small per-rank N (c4's 8192) still gives the latency-bound sample chain
// 2^17 - 2^18 threads (MGP_K6_ADAPTIVE_LANES = 0: 4 always).
#ifndef MGP_K6_ADAPTIVE_LANES
#define MGP_K6_ADAPTIVE_LANES 1
#endif
static int elbo_fwd_lanes(int64_t N) {
  if (!MGP_K6_ADAPTIVE_LANES) return kElboLanes;
  return N >= 65536 ? 4 : N >= 32768 ? 8 : 16;
}

extern "C" size_t mgp_elbo_workspace_bytes(int64_t N) {
  const int64_t nb = elbo_fwd_blocks(N, std::max(kElboLanes, elbo_fwd_lanes(N)));
  return (size_t)(nb > 0 ? nb : 1) * sizeof(double);
}

template <int KM, bool MOD, bool MC>
static void launch_elbo_terms(int nb, int lanes, hipStream_t s, const float* mu_f, const float* var_f,
                              const float* mu_a, const float* var_a, int64_t ldf, const float* Y,
                              const float* lik_var, const float* lik_var_a, int64_t N, int K, int S, float inv_tau,
                              float jitter, const float* noise_z, const float* noise_u, uint32_t k0, uint32_t k1,
                              int64_t n_offset, double* partials, float mc_a, float mc_b) {
  if constexpr (MC) {
    hipLaunchKernelGGL((elbo_terms_kernel<KM, MOD, MC, 1>), dim3(nb), dim3(kElboThreads), 0, s, mu_f, var_f, mu_a,
                       var_a, ldf, Y, lik_var, lik_var_a, N, K, S, inv_tau, jitter, noise_z, noise_u, k0, k1,
                       n_offset, partials, mc_a, mc_b);
  } else if (lanes == 16) {
    hipLaunchKernelGGL((elbo_terms_kernel<KM, MOD, MC, 16>), dim3(nb), dim3(kElboThreads), 0, s, mu_f, var_f, mu_a,
                       var_a, ldf, Y, lik_var, lik_var_a, N, K, S, inv_tau, jitter, noise_z, noise_u, k0, k1,
                       n_offset, partials, mc_a, mc_b);
  } else if (lanes == 8) {
    hipLaunchKernelGGL((elbo_terms_kernel<KM, MOD, MC, 8>), dim3(nb), dim3(kElboThreads), 0, s, mu_f, var_f, mu_a,
                       var_a, ldf, Y, lik_var, lik_var_a, N, K, S, inv_tau, jitter, noise_z, noise_u, k0, k1,
                       n_offset, partials, mc_a, mc_b);
  } else {
    hipLaunchKernelGGL((elbo_terms_kernel<KM, MOD, MC, kElboLanes>), dim3(nb), dim3(kElboThreads), 0, s, mu_f, var_f,
                       mu_a, var_a, ldf, Y, lik_var, lik_var_a, N, K, S, inv_tau, jitter, noise_z, noise_u, k0, k1,
                       n_offset, partials, mc_a, mc_b);
  }
}

// mc: the pred likelihood is MultiClass(K)/RobustMax(eps) with mc_a = log(1 - eps),
// mc_b = log(eps / (K - 1)) (lik_var unused); lik_var_a != NULL: SMGPModified.
static int elbo_terms_run(const float* mu_f, const float* var_f, const float* mu_a, const float* var_a,
                          int64_t ldf, const float* Y, const float* lik_var, const float* lik_var_a,
                          int64_t N, int32_t K, int32_t S, float tau, float jitter, const float* noise_z,
                          const float* noise_u, uint64_t seed, int64_t n_offset, double* data_sum,
                          void* workspace, size_t workspace_bytes, hipStream_t s, bool mc = false,
                          float mc_a = 0.f, float mc_b = 0.f) {
  if (!workspace || workspace_bytes < mgp_elbo_workspace_bytes(N)) return MGP_ERR_WORKSPACE;
  double* partials = (double*)workspace;
  const int lanes = mc ? 1 : elbo_fwd_lanes(N);
  const int nb = (int)elbo_fwd_blocks(N, lanes);
  const uint32_t k0 = (uint32_t)(seed & 0xffffffffu), k1 = (uint32_t)(seed >> 32);
  if (nb > 0) {
#define MGP_ELBO_CASE(KM)                                                                               \
  if (K <= KM) {                                                                                         \
    auto f = lik_var_a ? (mc ? launch_elbo_terms<KM, true, true> : launch_elbo_terms<KM, true, false>)   \
                       : (mc ? launch_elbo_terms<KM, false, true> : launch_elbo_terms<KM, false, false>); \
    f(nb, lanes, s, mu_f, var_f, mu_a, var_a, ldf, Y, lik_var, lik_var_a, N, K, S, 1.f / tau, jitter,    \
      noise_z,                                                                                           \
      noise_u, k0, k1, n_offset, partials, mc_a, mc_b);                                                  \
  } else
    MGP_ELBO_CASE(1) MGP_ELBO_CASE(2) MGP_ELBO_CASE(4) MGP_ELBO_CASE(8) MGP_ELBO_CASE(16)
    MGP_ELBO_CASE(32) {}
#undef MGP_ELBO_CASE
    int st = launch_status();
    if (st) return st;
  }
  hipLaunchKernelGGL(sum_partials_kernel, dim3(1), dim3(1024), 0, s, partials, nb, data_sum);
  return launch_status();
}

extern "C" int mgp_elbo_terms(const float* mu_f, const float* var_f, const float* mu_a,
                              const float* var_a, int64_t ldf, const float* Y, const float* lik_var,
                              int64_t N, int32_t K, int32_t S, float tau, float jitter,
                              const float* noise_z,
                              const float* noise_u, uint64_t seed, int64_t n_offset,
                              double* data_sum, void* workspace, size_t workspace_bytes,
                              mgp_stream_t stream) {
  if (!mu_f) return -1;
  if (!var_f) return -2;
  if (!mu_a) return -3;
  if (!var_a) return -4;
  if (ldf < N) return -5;
  if (!Y) return -6;
  if (!lik_var) return -7;
  if (N < 0) return -8;
  if (K < 1) return -9;
  if (K > 32) return MGP_ERR_UNSUPPORTED;
  if (S < 1) return -10;
  if (!(tau > 0.f)) return -11;
  if (!(jitter >= 0.f)) return -14;
  if ((noise_z == nullptr) != (noise_u == nullptr)) return -12;
  if (n_offset < 0) return -15;
  if (!data_sum) return -16;
  return elbo_terms_run(mu_f, var_f, mu_a, var_a, ldf, Y, lik_var, nullptr, N, K, S, tau, jitter, noise_z, noise_u,
                        seed, n_offset, data_sum, workspace, workspace_bytes, (hipStream_t)stream);
}

extern "C" int mgp_elbo_terms_modified(const float* mu_f, const float* var_f, const float* mu_a,
                                       const float* var_a, int64_t ldf, const float* Y,
                                       const float* lik_var, const float* assign_lik_var, int64_t N,
                                       int32_t K, int32_t S, float tau, float jitter,
                                       const float* noise_z,
                                       const float* noise_u, uint64_t seed, int64_t n_offset,
                                       double* data_sum, void* workspace, size_t workspace_bytes,
                                       mgp_stream_t stream) {
  if (!mu_f) return -1;
  if (!var_f) return -2;
  if (!mu_a) return -3;
  if (!var_a) return -4;
  if (ldf < N) return -5;
  if (!Y) return -6;
  if (!lik_var) return -7;
  if (!assign_lik_var) return -8;
  if (N < 0) return -9;
  if (K < 1) return -10;
  if (K > 32) return MGP_ERR_UNSUPPORTED;
  if (S < 1) return -11;
  if (!(tau > 0.f)) return -12;
  if (!(jitter >= 0.f)) return -15;
  if ((noise_z == nullptr) != (noise_u == nullptr)) return -13;
  if (n_offset < 0) return -16;
  if (!data_sum) return -17;
  return elbo_terms_run(mu_f, var_f, mu_a, var_a, ldf, Y, lik_var, assign_lik_var, N, K, S, tau, jitter, noise_z,
                        noise_u, seed, n_offset, data_sum, workspace, workspace_bytes, (hipStream_t)stream);
}

extern "C" int mgp_elbo_combine(const double* data_sum, const double* kl_f, const double* kl_a,
                                double n_batch, double num_data, float* elbo_out, double* elbo_out64,
                                mgp_stream_t stream) {
  if (!data_sum) return -1;
  if (!kl_f) return -2;
  if (!kl_a) return -3;
  if (!(n_batch > 0)) return -4;
  if (!(num_data > 0)) return -5;
  if (!elbo_out && !elbo_out64) return -6;
  hipLaunchKernelGGL(elbo_combine_kernel, dim3(1), dim3(1), 0, (hipStream_t)stream, data_sum, kl_f,
                     kl_a, n_batch, num_data, elbo_out, elbo_out64);
  return launch_status();
}

static int kl_row_blocks(int64_t M) { return (int)((M + kKlRows - 1) / kKlRows); }

extern "C" size_t mgp_kl_workspace_bytes(int64_t M, int32_t K) {
  return (size_t)(K * kl_row_blocks(M) + 1) * 3 * sizeof(double);
}

extern "C" int mgp_gauss_kl_white(const float* q_mu, int64_t ldq, const float* q_sqrt, int64_t ldqs,
                                  int64_t strideq, int64_t M, int32_t K, double* kl_out,
                                  void* workspace, size_t workspace_bytes, mgp_stream_t stream) {
  if (!q_mu) return -1;
  if (ldq < K) return -2;
  if (!q_sqrt) return -3;
  if (ldqs < M) return -4;
  if (K > 1 && strideq < ldqs * M) return -5;
  if (M < 1) return -6;
  if (K < 1) return -7;
  if (!kl_out) return -8;
  if ((ldqs & 3) || (strideq & 3) || !aligned16(q_sqrt)) return MGP_ERR_ALIGN;  // float4 rows
  if (!workspace || workspace_bytes < mgp_kl_workspace_bytes(M, K)) return MGP_ERR_WORKSPACE;
  hipStream_t s = (hipStream_t)stream;
  const int nrb = kl_row_blocks(M);
  const int nblk = K * nrb + 1;
  double* p = (double*)workspace;
  hipLaunchKernelGGL(kl_partials_kernel, dim3(nblk), dim3(256), 0, s, q_mu, ldq, q_sqrt, ldqs,
                     strideq, M, K, nrb, p);
  int st = launch_status();
  if (st) return st;
  hipLaunchKernelGGL(kl_final_kernel, dim3(1), dim3(1024), 0, s, p, nblk, (double)M * (double)K,
                     kl_out);
  return launch_status();
}

extern "C" int mgp_predict_epilogue(const float* fmean, const float* fvar, const float* amean,
                                    int64_t ldf, const float* lik_var, int64_t N, int32_t K,
                                    float* y_mean, float* y_var, float* assign, mgp_stream_t stream) {
  if ((y_mean || y_var) && !fmean) return -1;
  if (y_var && !fvar) return -2;
  if (assign && !amean) return -3;
  if (ldf < N) return -4;
  if (y_var && !lik_var) return -5;
  if (N < 0) return -6;
  if (K < 1) return -7;
  if (N == 0) return MGP_OK;
  hipLaunchKernelGGL(predict_epilogue_kernel, dim3((unsigned)((N + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, fmean, fvar, amean, ldf, lik_var, N, K, y_mean, y_var, assign);
  return launch_status();
}

extern "C" int mgp_philox_noise(uint64_t seed, int64_t n_offset, int64_t N, int32_t K, int32_t S,
                                float* z, float* u, mgp_stream_t stream) {
  if (n_offset < 0) return -2;
  if (N < 0) return -3;
  if (K < 1) return -4;
  if (S < 1) return -5;
  if (N == 0) return MGP_OK;
  const int64_t total = N * (int64_t)S;
  hipLaunchKernelGGL(philox_noise_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, (uint32_t)(seed & 0xffffffffu), (uint32_t)(seed >> 32),
                     n_offset, N, K, S, z, u);
  return launch_status();
}

extern "C" const char* mgp_version(void) { return "mgp_hip 0.1.0 gfx950"; }

extern "C" const char* mgp_status_string(int status) {
  if (status == MGP_OK) return "ok";
  if (status < 0) return "invalid argument (index = -status)";
  if (status == MGP_ERR_WORKSPACE) return "workspace missing or too small";
  if (status == MGP_ERR_ALIGN) return "leading dimension or pointer not 16-byte aligned";
  if (status == MGP_ERR_UNSUPPORTED) return "size outside the supported range";
  if (status >= MGP_ERR_HIP_BASE) return hipGetErrorString((hipError_t)(status - MGP_ERR_HIP_BASE));
  return "unknown status";
}

static int elbo_kmax(int K) { return K <= 1 ? 1 : K <= 2 ? 2 : K <= 4 ? 4 : K <= 8 ? 8 : K <= 16 ? 16 : 32; }

extern "C" size_t mgp_elbo_backward_workspace_bytes(int64_t N, int32_t K) {
  const int64_t nb = N > 0 ? elbo_fwd_blocks(N, kElboLanes) : 1;
  return (size_t)nb * 2 * (size_t)elbo_kmax(K) * sizeof(double);
}

template <int KM, bool MOD, bool MC>
static void launch_elbo_bwd(int nb, hipStream_t s, const float* mu_f, const float* var_f, const float* mu_a,
                            const float* var_a, int64_t ldf, const float* Y, const float* lik_var,
                            const float* lik_var_a, int64_t N, int K, int S, float inv_tau, float jitter,
                            const float* noise_z, const float* noise_u, uint32_t k0, uint32_t k1, int64_t n_offset, float scale,
                            float* G, int64_t ldg, double* partials, float mc_a, float mc_b) {
  constexpr int L = MC ? 1 : kElboBwdLanes;
  hipLaunchKernelGGL((elbo_terms_bwd_kernel<KM, MOD, MC, L>), dim3(nb), dim3(kElboThreads), 0, s, mu_f, var_f, mu_a,
                     var_a, ldf, Y, lik_var, lik_var_a, N, K, S, inv_tau, jitter, noise_z, noise_u, k0, k1, n_offset,
                     scale, G, ldg, partials, mc_a, mc_b);
}

static int elbo_bwd_run(const float* mu_f, const float* var_f, const float* mu_a, const float* var_a, int64_t ldf,
                        const float* Y, const float* lik_var, const float* assign_lik_var, int64_t N, int32_t K,
                        int32_t S, float tau, float jitter, const float* noise_z, const float* noise_u, uint64_t seed,
                        int64_t n_offset, float scale, float* G, int64_t ldg, double* g_lik_var,
                        double* g_assign_lik_var, void* workspace, size_t workspace_bytes, hipStream_t s, bool mc,
                        float mc_a, float mc_b) {
  if (!workspace || workspace_bytes < mgp_elbo_backward_workspace_bytes(N, K)) return MGP_ERR_WORKSPACE;
  double* partials = (double*)workspace;
  const int nb = (int)elbo_fwd_blocks(N, mc ? 1 : kElboBwdLanes);
  const int km = elbo_kmax(K);
  const uint32_t k0 = (uint32_t)(seed & 0xffffffffu), k1 = (uint32_t)(seed >> 32);
  if (nb == 0) {
    if (g_lik_var) hipMemsetAsync(g_lik_var, 0, (size_t)K * sizeof(double), s);
    if (assign_lik_var) hipMemsetAsync(g_assign_lik_var, 0, (size_t)K * sizeof(double), s);
    return launch_status();
  }
#define MGP_ELBO_BWD_CASE(KM)                                                                             \
  if (km == KM) {                                                                                         \
    auto f = assign_lik_var ? (mc ? launch_elbo_bwd<KM, true, true> : launch_elbo_bwd<KM, true, false>)  \
                            : (mc ? launch_elbo_bwd<KM, false, true> : launch_elbo_bwd<KM, false, false>); \
    f(nb, s, mu_f, var_f, mu_a, var_a, ldf, Y, lik_var, assign_lik_var, N, K, S, 1.f / tau, jitter, noise_z, \
      noise_u, k0, k1, n_offset, scale, G, ldg, partials, mc_a, mc_b);                                    \
  } else
  MGP_ELBO_BWD_CASE(1) MGP_ELBO_BWD_CASE(2) MGP_ELBO_BWD_CASE(4) MGP_ELBO_BWD_CASE(8) MGP_ELBO_BWD_CASE(16)
  MGP_ELBO_BWD_CASE(32) {}
#undef MGP_ELBO_BWD_CASE
  int st = launch_status();
  if (st) return st;
  if (g_lik_var)
    hipLaunchKernelGGL(column_sums_kernel, dim3(K), dim3(256), 0, s, partials, nb, (int64_t)2 * km, g_lik_var,
                       (int64_t)1);
  if (assign_lik_var)
    hipLaunchKernelGGL(column_sums_kernel, dim3(K), dim3(256), 0, s, partials + km, nb, (int64_t)2 * km,
                       g_assign_lik_var, (int64_t)1);
  return launch_status();
}

extern "C" int mgp_elbo_terms_backward(const float* mu_f, const float* var_f, const float* mu_a,
                                       const float* var_a, int64_t ldf, const float* Y,
                                       const float* lik_var, const float* assign_lik_var, int64_t N,
                                       int32_t K, int32_t S, float tau, float jitter,
                                       const float* noise_z,
                                       const float* noise_u, uint64_t seed, int64_t n_offset,
                                       float scale, float* G, int64_t ldg, double* g_lik_var,
                                       double* g_assign_lik_var, void* workspace,
                                       size_t workspace_bytes, mgp_stream_t stream) {
  if (!mu_f) return -1;
  if (!var_f) return -2;
  if (!mu_a) return -3;
  if (!var_a) return -4;
  if (ldf < N) return -5;
  if (!Y) return -6;
  if (!lik_var) return -7;
  if (N < 0) return -9;
  if (K < 1) return -10;
  if (K > 32) return MGP_ERR_UNSUPPORTED;
  if (S < 1) return -11;
  if (!(tau > 0.f)) return -12;
  if (!(jitter >= 0.f)) return -15;
  if ((noise_z == nullptr) != (noise_u == nullptr)) return -13;
  if (n_offset < 0) return -16;
  if (!G) return -18;
  if (ldg < N) return -19;
  if (!g_lik_var) return -20;
  if (assign_lik_var && !g_assign_lik_var) return -21;
  return elbo_bwd_run(mu_f, var_f, mu_a, var_a, ldf, Y, lik_var, assign_lik_var, N, K, S, tau, jitter, noise_z, noise_u,
                      seed, n_offset, scale, G, ldg, g_lik_var, g_assign_lik_var, workspace, workspace_bytes,
                      (hipStream_t)stream, false, 0.f, 0.f);
}

// ------------------------------------------------------------------ MultiClass entries
static bool mc_consts(int K, float epsilon, float& a, float& b) {
  if (K < 2 || !(epsilon > 0.f) || !(epsilon < 1.f)) return false;
  a = (float)log1p(-(double)epsilon);
  b = (float)log((double)epsilon / (double)(K - 1));
  return true;
}

extern "C" int mgp_elbo_terms_multiclass(const float* mu_f, const float* var_f, const float* mu_a,
                                         const float* var_a, int64_t ldf, const float* Y, float epsilon,
                                         const float* assign_lik_var, int64_t N, int32_t K, int32_t S, float tau,
                                         float jitter, const float* noise_z, const float* noise_u, uint64_t seed,
                                         int64_t n_offset, double* data_sum, void* workspace,
                                         size_t workspace_bytes, mgp_stream_t stream) {
  float a, b;
  if (!mu_f) return -1;
  if (!var_f) return -2;
  if (!mu_a) return -3;
  if (!var_a) return -4;
  if (ldf < N) return -5;
  if (!Y) return -6;
  if (!(epsilon > 0.f && epsilon < 1.f)) return -7;
  if (N < 0) return -9;
  if (K < 2) return -10;
  if (K > 32) return MGP_ERR_UNSUPPORTED;
  if (S < 1) return -11;
  if (!(tau > 0.f)) return -12;
  if (!(jitter >= 0.f)) return -15;
  if ((noise_z == nullptr) != (noise_u == nullptr)) return -13;
  if (n_offset < 0) return -16;
  if (!data_sum) return -17;
  mc_consts(K, epsilon, a, b);
  return elbo_terms_run(mu_f, var_f, mu_a, var_a, ldf, Y, nullptr, assign_lik_var, N, K, S, tau, jitter, noise_z, noise_u,
                        seed, n_offset, data_sum, workspace, workspace_bytes, (hipStream_t)stream, true, a, b);
}

extern "C" int mgp_elbo_terms_multiclass_backward(const float* mu_f, const float* var_f, const float* mu_a,
                                                  const float* var_a, int64_t ldf, const float* Y, float epsilon,
                                                  const float* assign_lik_var, int64_t N, int32_t K, int32_t S,
                                                  float tau, float jitter, const float* noise_z, const float* noise_u,
                                                  uint64_t seed, int64_t n_offset, float scale, float* G,
                                                  int64_t ldg, double* g_assign_lik_var, void* workspace,
                                                  size_t workspace_bytes, mgp_stream_t stream) {
  float a, b;
  if (!mu_f) return -1;
  if (!var_f) return -2;
  if (!mu_a) return -3;
  if (!var_a) return -4;
  if (ldf < N) return -5;
  if (!Y) return -6;
  if (!(epsilon > 0.f && epsilon < 1.f)) return -7;
  if (N < 0) return -9;
  if (K < 2) return -10;
  if (K > 32) return MGP_ERR_UNSUPPORTED;
  if (S < 1) return -11;
  if (!(tau > 0.f)) return -12;
  if (!(jitter >= 0.f)) return -15;
  if ((noise_z == nullptr) != (noise_u == nullptr)) return -13;
  if (n_offset < 0) return -16;
  if (!G) return -18;
  if (ldg < N) return -19;
  if (assign_lik_var && !g_assign_lik_var) return -20;
  mc_consts(K, epsilon, a, b);
  return elbo_bwd_run(mu_f, var_f, mu_a, var_a, ldf, Y, nullptr, assign_lik_var, N, K, S, tau, jitter, noise_z, noise_u,
                      seed, n_offset, scale, G, ldg, nullptr, g_assign_lik_var, workspace, workspace_bytes,
                      (hipStream_t)stream, true, a, b);
}
