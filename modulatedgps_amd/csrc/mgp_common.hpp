// Shared device helpers for the gfx950 SMGP kernels (MFMA fragments, wave
// reductions, guarded vector loads, Philox noise).  CDNA4 only: wave64,
// f32-input MFMA v_mfma_f32_32x32x2_f32.
#pragma once
#include <hip/hip_runtime.h>

#include <type_traits>
#include <stdint.h>

#include "mgp_hip.h"

namespace mgp {

typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef float floatx4 __attribute__((ext_vector_type(4)));

constexpr int kWave = 64;

// ------------------------------------------------------------------ errors
inline int hip_status(hipError_t e) { return e == hipSuccess ? MGP_OK : MGP_ERR_HIP_BASE + (int)e; }
inline int launch_status() { return hip_status(hipGetLastError()); }
inline bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }

// fmean[k][n] = sum over nTs stats tiles; fvar[k][n] = var - sum_t ||A||^2 part
// + sum over nTp expert partials (trigemm.hip; shared by the f32 and split-bf16 K5).
int mgp_launch_cond_finalize(const float* stats, int64_t lds, int nTs, const float* part, int64_t ldp, int nTp,
                             const float* variance, int64_t N, int K, float* fmean, float* fvar, int64_t ldf,
                             hipStream_t s);
// One layer's operands of the two-layer finalize (mgp_expert_conditional_f16_batch).
struct CondFinLayer {
  const float* stats;
  const float* part;
  const float* variance;
  float* fmean;
  float* fvar;
};
int mgp_launch_cond_finalize2(const CondFinLayer& l0, const CondFinLayer& l1, int64_t lds, int nTs, int64_t ldp,
                              int nTp, int64_t N, int K, int64_t ldf, hipStream_t s);

// ------------------------------------------------------------------ MFMA
// D(32x32) += A(32x2) * B(2x32), exact f32 (fmaf chain).  Lane l supplies
// A[i = l & 31][k = l >> 5] and B[k = l >> 5][j = l & 31].  Result register r of
// lane l holds D[row = (r & 3) + 8 * (r >> 2) + 4 * (l >> 5)][col = l & 31].
// Cross-lane moves on gfx950's permlane swaps (VALU ops; __shfl_xor compiles to an
// LDS-crossbar ds_bpermute whose latency every use then waits for).
// lane_half_swap: lanes 0-31 get (a, a of lane + 32), lanes 32-63 get (b of lane - 32, b)
// -- the two halves of an output fragment from the 16x16 accumulator layout.
__device__ __forceinline__ void lane_half_swap(uint32_t& a, uint32_t& b) {
  const auto r = __builtin_amdgcn_permlane32_swap(a, b, false, false);
  a = r[0];
  b = r[1];
}
__device__ __forceinline__ void lane_half_swap(float& a, float& b) {
  uint32_t x = __float_as_uint(a), y = __float_as_uint(b);
  lane_half_swap(x, y);
  a = __uint_as_float(x);
  b = __uint_as_float(y);
}
// the value of lane l ^ 32 / l ^ 16
__device__ __forceinline__ float lane_xor32(float v) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float((threadIdx.x & 32) ? r[0] : r[1]);
}
__device__ __forceinline__ float lane_xor16(float v) {
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float((threadIdx.x & 16) ? r[0] : r[1]);
}

// max over the 64 lanes of a wave, every lane gets it: DPP within rows of 16 (quad
// swaps, half-row and row mirrors pair the groups already reduced), then the
// permlane swaps across rows (no LDS round trips)
// max over each 32-lane half of a wave (every lane of the half gets it)
__device__ __forceinline__ float half_max_f32(float v) {
  auto dpp = [](float x, auto ctrl) {
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), decltype(ctrl)::value, 0xF, 0xF, false));
  };
  v = fmaxf(v, dpp(v, std::integral_constant<int, 0xB1>{}));   // quad_perm [1, 0, 3, 2]
  v = fmaxf(v, dpp(v, std::integral_constant<int, 0x4E>{}));   // quad_perm [2, 3, 0, 1]
  v = fmaxf(v, dpp(v, std::integral_constant<int, 0x141>{}));  // row_half_mirror
  v = fmaxf(v, dpp(v, std::integral_constant<int, 0x140>{}));  // row_mirror
  return fmaxf(v, lane_xor16(v));
}

__device__ __forceinline__ float wave_max_f32(float v) {
  auto dpp = [](float x, auto ctrl) {
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), decltype(ctrl)::value, 0xF, 0xF, false));
  };
  v = fmaxf(v, dpp(v, std::integral_constant<int, 0xB1>{}));   // quad_perm [1, 0, 3, 2]
  v = fmaxf(v, dpp(v, std::integral_constant<int, 0x4E>{}));   // quad_perm [2, 3, 0, 1]
  v = fmaxf(v, dpp(v, std::integral_constant<int, 0x141>{}));  // row_half_mirror
  v = fmaxf(v, dpp(v, std::integral_constant<int, 0x140>{}));  // row_mirror
  v = fmaxf(v, lane_xor16(v));
  return fmaxf(v, lane_xor32(v));
}

__device__ __forceinline__ floatx16 mfma32x32x2(float a, float b, floatx16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ int acc_row(int r, int lane) { return (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5); }

// ------------------------------------------------------------------ split-bf16 (x6) images
// See split3.hip.  A fragment is 64 lanes x 8 bf16 per plane (1 KiB); lane
// (r = lane & 31, h = lane >> 5), element j <-> k-row kperm(h, j) of a 16-row
// k-step, the order in which a 32x32 accumulator holds its rows.
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef unsigned int u32x4v __attribute__((ext_vector_type(4)));

__device__ __forceinline__ int kperm(int h, int j) { return (j & 3) + 8 * (j >> 2) + 4 * h; }

// x -> (hi, mid, lo) bf16 planes; both differences are exact in f32.
__device__ __forceinline__ void split3(float x, __bf16& hi, __bf16& mid, __bf16& lo) {
  hi = (__bf16)x;
  const float r1 = x - (float)hi;
  mid = (__bf16)r1;
  const float r2 = r1 - (float)mid;
  lo = (__bf16)r2;
}

// Split 8 values and store the three planes of one lane (dst = plane 0 of the
// lane; planes are 64 bf16x8 apart).
__device__ __forceinline__ void store_split(bf16x8* __restrict__ dst, const float (&v)[8]) {
  bf16x8 h, m, l;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    __bf16 a, b, c;
    split3(v[j], a, b, c);
    h[j] = a; m[j] = b; l[j] = c;
  }
  dst[0] = h;
  dst[64] = m;
  dst[128] = l;
}

__device__ __forceinline__ floatx16 mfma_bf16(bf16x8 a, bf16x8 b, floatx16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

// acc += (a_hi + a_mid + a_lo)(b_hi + b_mid + b_lo) without the three
// products of weight < 2^-16; smallest terms first.
__device__ __forceinline__ floatx16 mfma_x6(const bf16x8 (&a)[3], const bf16x8 (&b)[3], floatx16 acc) {
  acc = mfma_bf16(a[2], b[0], acc);
  acc = mfma_bf16(a[1], b[1], acc);
  acc = mfma_bf16(a[0], b[2], acc);
  acc = mfma_bf16(a[1], b[0], acc);
  acc = mfma_bf16(a[0], b[1], acc);
  return mfma_bf16(a[0], b[0], acc);
}

// Reduced-plane products (K5's "bf16 mixed" modes, BASELINE config 5):
// NPL = 2: a_hi b_hi + a_hi b_mid + a_mid b_hi (dropped terms <= 2^-16 of the
// leading one: ~16-bit operands); NPL = 1: a_hi b_hi (bf16 operands).
template <int NPL>
__device__ __forceinline__ floatx16 mfma_planes(const bf16x8 (&a)[3], const bf16x8 (&b)[3], floatx16 acc) {
  if constexpr (NPL == 3) {
    return mfma_x6(a, b, acc);
  } else if constexpr (NPL == 2) {
    acc = mfma_bf16(a[1], b[0], acc);
    acc = mfma_bf16(a[0], b[1], acc);
    return mfma_bf16(a[0], b[0], acc);
  } else {
    return mfma_bf16(a[0], b[0], acc);
  }
}

// ------------------------------------------------------------------ split-f16 ("f16x3") images
// Same fragment geometry, planes 0 and 1 hold fp16 hi / lo of x 2^e (plane 2
// unused): x 2^e = hi + lo + |x 2^e| 2^-22 at most, and the product
// a b ~ a_hi b_hi + a_hi b_lo + a_lo b_hi drops a_lo b_lo (<= 2^-22 of it):
// three v_mfma_f32_32x32x16_f16 per block instead of six bf16 ones.  The image
// scale e (a power of two, so exact) keeps the operand's largest magnitude in
// [2^13, 2^14): hi never overflows (4x headroom below 65504) and lo stays a
// normal fp16 down to 2^-16 of that maximum.  e comes from the image trailer
// (the float bound |x| <= trailer, see img_exp) that the producer writes.
typedef _Float16 halfx8 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ int img_exp(float bound) {
  if (!(bound > 0.f) || !(bound < 3.0e38f)) return 0;  // zero / inf / nan: unscaled
  return 13 - ilogbf(bound);
}

// X8: plane 2 also gets the fp8 cross-term plane of the same 8 values (K5's
// "f16x8" mode, mfma_f8x): dwords 0-1 = e4m3(hi 2^-6), dwords 2-3 = e4m3(lo 2^6).
// With the image maximum in [2^13, 2^14) both land in e4m3's range (<= 2^8):
// hi 2^-6 keeps 3 mantissa bits down to 2^-14 of the maximum, lo 2^6 likewise.
// write_lo = false (X8 only): plane 1 (f16 lo) is left unwritten -- the image then
// feeds only the f16x8 K5, which reads planes 0 and 2.
template <bool X8 = false>
__device__ __forceinline__ void store_split_f16(bf16x8* __restrict__ dst, const float (&v)[8], float scale,
                                                bool write_lo = true) {
  halfx8 h, l;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const float x = v[j] * scale;
    const _Float16 hi = (_Float16)x;
    h[j] = hi;
    l[j] = (_Float16)(x - (float)hi);  // exact difference in f32
  }
  dst[0] = __builtin_bit_cast(bf16x8, h);
  if (!X8 || write_lo) dst[64] = __builtin_bit_cast(bf16x8, l);
  if constexpr (X8) {
    u32x4v x8;
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      int wh = 0, wl = 0;
      wh = __builtin_amdgcn_cvt_pk_fp8_f32((float)h[4 * q] * 0x1p-6f, (float)h[4 * q + 1] * 0x1p-6f, wh, false);
      wh = __builtin_amdgcn_cvt_pk_fp8_f32((float)h[4 * q + 2] * 0x1p-6f, (float)h[4 * q + 3] * 0x1p-6f, wh, true);
      wl = __builtin_amdgcn_cvt_pk_fp8_f32((float)l[4 * q] * 0x1p6f, (float)l[4 * q + 1] * 0x1p6f, wl, false);
      wl = __builtin_amdgcn_cvt_pk_fp8_f32((float)l[4 * q + 2] * 0x1p6f, (float)l[4 * q + 3] * 0x1p6f, wl, true);
      x8[q] = (uint32_t)wh;
      x8[2 + q] = (uint32_t)wl;
    }
    dst[128] = __builtin_bit_cast(bf16x8, x8);
  }
}

__device__ __forceinline__ floatx16 mfma_f16(bf16x8 a, bf16x8 b, floatx16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(halfx8, a), __builtin_bit_cast(halfx8, b), c,
                                                0, 0, 0);
}

// Cross terms of two k-steps (k, k') of split-f16 images on one e4m3 MFMA
// (2x the f16 rate per flop): a_hi b_lo + a_lo b_hi over 64 k.  ax, bx are the
// X8 planes (store_split_f16<true>); b's hi/lo halves are swapped so that every
// a_hi 2^-6 byte meets the b_lo 2^6 byte of the same k (the scales cancel; A
// and B share the per-lane k distribution, so any consistent pairing works).
typedef int intx8 __attribute__((ext_vector_type(8)));
__device__ __forceinline__ floatx16 mfma_f8x(bf16x8 ax0, bf16x8 ax1, bf16x8 bx0, bf16x8 bx1, floatx16 acc) {
  const u32x4v a0 = __builtin_bit_cast(u32x4v, ax0), a1 = __builtin_bit_cast(u32x4v, ax1);
  const u32x4v b0 = __builtin_bit_cast(u32x4v, bx0), b1 = __builtin_bit_cast(u32x4v, bx1);
  const intx8 a = {(int)a0[0], (int)a0[1], (int)a0[2], (int)a0[3], (int)a1[0], (int)a1[1], (int)a1[2], (int)a1[3]};
  const intx8 b = {(int)b0[2], (int)b0[3], (int)b0[0], (int)b0[1], (int)b1[2], (int)b1[3], (int)b1[0], (int)b1[1]};
  return __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a, b, acc, 0, 0, 0, 127, 0, 127);
}

// F16 images (NPL = 2): a_hi b_hi + a_hi b_lo + a_lo b_hi, smallest first.
template <int NPL, bool F16>
__device__ __forceinline__ floatx16 mfma_fmt(const bf16x8 (&a)[3], const bf16x8 (&b)[3], floatx16 acc) {
  if constexpr (F16) {
    static_assert(NPL == 2, "f16 images have two planes");
    acc = mfma_f16(a[1], b[0], acc);
    acc = mfma_f16(a[0], b[1], acc);
    return mfma_f16(a[0], b[0], acc);
  } else {
    return mfma_planes<NPL>(a, b, acc);
  }
}

// ------------------------------------------------------------------ reductions
template <typename T>
__device__ __forceinline__ T wave_sum(T v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, kWave);
  return v;
}

// Block-wide sum (blockDim.x multiple of 64, <= 1024).  Result valid in thread 0.
template <typename T>
__device__ __forceinline__ T block_sum(T v, T* scratch /* >= 16 entries */) {
  v = wave_sum(v);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (lane == 0) scratch[w] = v;
  __syncthreads();
  T r = 0;
  if (threadIdx.x == 0) {
    const int nw = blockDim.x >> 6;
    for (int i = 0; i < nw; ++i) r += scratch[i];
  }
  __syncthreads();
  return r;
}

// ------------------------------------------------------------------ guarded loads
// Load 4 consecutive floats of row `row` starting at column `col` (col % 4 == 0)
// with zero fill outside [0, nrows) x [0, ncols).  Requires ld % 4 == 0 and a
// 16-byte aligned base.
__device__ __forceinline__ floatx4 load4_guarded(const float* __restrict__ base, int64_t ld,
                                                 int64_t row, int64_t col, int64_t nrows,
                                                 int64_t ncols) {
  floatx4 v = {0.f, 0.f, 0.f, 0.f};
  if (row < nrows) {
    const float* p = base + row * ld + col;
    if (col + 3 < ncols) {
      v = *reinterpret_cast<const floatx4*>(p);
    } else {
      if (col + 0 < ncols) v.x = p[0];
      if (col + 1 < ncols) v.y = p[1];
      if (col + 2 < ncols) v.z = p[2];
    }
  }
  return v;
}

// ------------------------------------------------------------------ Philox4x32-10
// Salmon et al. SC'11; constants from Random123.  Must match oracle/philox.py.
struct u32x4 { uint32_t x, y, z, w; };

__device__ __forceinline__ u32x4 philox4x32_10(u32x4 c, uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    const uint32_t hi0 = __umulhi(0xD2511F53u, c.x), lo0 = 0xD2511F53u * c.x;
    const uint32_t hi1 = __umulhi(0xCD9E8D57u, c.z), lo1 = 0xCD9E8D57u * c.z;
    c = u32x4{hi1 ^ c.y ^ k0, lo1, hi0 ^ c.w ^ k1, lo0};
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return c;
}

// uint32 -> (0,1): ((w >> 9) + 0.5) * 2^-23 (exact in fp32).
__device__ __forceinline__ float u01(uint32_t w) { return ((float)(w >> 9) + 0.5f) * 1.1920928955078125e-07f; }

// Four normals from one stream-0 block (Box-Muller on word pairs (x,y), (z,w)).
__device__ __forceinline__ void box_muller4(u32x4 w, float out[4]) {
  // Precise logf/sincosf (not the __ intrinsics): parity with the float64 oracle.
  const float r0 = sqrtf(-2.f * logf(u01(w.x)));
  const float r1 = sqrtf(-2.f * logf(u01(w.z)));
  float s0, c0, s1, c1;
  sincosf(6.283185307179586f * u01(w.y), &s0, &c0);
  sincosf(6.283185307179586f * u01(w.w), &s1, &c1);
  out[0] = r0 * c0;
  out[1] = r0 * s0;
  out[2] = r1 * c1;
  out[3] = r1 * s1;
}

}  // namespace mgp
