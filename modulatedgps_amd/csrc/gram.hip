// Backward "gram" products: contractions over the data dimension N.
//
//   out[i][j] = alpha * sum_n X[i][n] Y[j][n]        (X: [MI][ldx], Y: [MJ][ldy], f32)
//
// used for the gradients that sum over data points (the GradientTape pass of
// GPflow base_conditional, MixtureGPs/models.py:141-143):
//   dL_k   = 2 tril(A diag(Gv_k) (L_k^T A)^T)   X = A, Y = CG_k         (q_sqrt)
//   dLm    = -tril(gKuf A^T)                     X = gKuf, Y = A          (Cholesky factor)
//   dq_mu  = A G_mu^T                            X = A, Y = G_mu          (q_mu)
//
// gfx950 mapping: 128 x 128 output tile per workgroup (4 waves of 64 x 64 =
// 2 x 2 tiles of v_mfma_f32_32x32x2_f32, exact f32), 16-deep n-chunks
// global -> registers -> LDS ([row][16 + 1] images, conflict-free column
// reads), double-buffered.  The n range is split over blockIdx.z (split-K) for
// parallelism; partial tiles go to a workspace and gram_reduce_kernel sums
// them in a fixed order (deterministic), applies alpha and the triangle.
// Roofline: f32 MFMA (2 MI MJ N flops, half for the triangular outputs).
#include "mgp_common.hpp"

namespace mgp {

constexpr int kGT = 128;   // output tile
constexpr int kGK = 16;    // n per chunk
constexpr int kGP = kGK + 1;

__device__ __forceinline__ floatx4 gload4(const float* __restrict__ p, int64_t ld, int64_t r, int64_t c,
                                          int64_t R, int64_t C) {
  if (r < R && c + 3 < C) return *reinterpret_cast<const floatx4*>(p + r * ld + c);
  floatx4 v = {0.f, 0.f, 0.f, 0.f};
  if (r < R) {
#pragma unroll
    for (int e = 0; e < 4; ++e)
      if (c + e < C) v[e] = p[r * ld + c + e];
  }
  return v;
}

// grid: x = tile pair (TRI: bj <= bi only), z = n split.
template <bool TRI>
__global__ __launch_bounds__(256) void gram_kernel(const float* __restrict__ X, int64_t ldx, int64_t MI,
                                                   const float* __restrict__ Y, int64_t ldy, int64_t MJ,
                                                   int64_t N, int64_t nper, int nbj, float* __restrict__ ws,
                                                   int64_t ldw, int64_t split_stride) {
  __shared__ float sx[2][kGT * kGP], sy[2][kGT * kGP];
  int bi, bj;
  if (TRI) {
    int q = blockIdx.x;
    bi = 0;
    while ((bi + 1) * (bi + 2) / 2 <= q) ++bi;
    bj = q - bi * (bi + 1) / 2;
  } else {
    bi = blockIdx.x / nbj;
    bj = blockIdx.x % nbj;
  }
  const int64_t i0 = (int64_t)bi * kGT, j0 = (int64_t)bj * kGT;
  const int64_t nb = (int64_t)blockIdx.z * nper;
  const int64_t ne = (nb + nper < N) ? nb + nper : N;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wi = (w >> 1) * 64, wj = (w & 1) * 64;
  floatx16 acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[a][b][e] = 0.f;
  // thread t loads rows t / 4 and t / 4 + 64, columns 4 (t % 4) .. + 3 of the chunk
  const int lr = tid >> 2, lc = (tid & 3) * 4;
  floatx4 rx[2], ry[2];
  auto load = [&](int64_t n0) {
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      rx[q] = gload4(X, ldx, i0 + lr + 64 * q, n0 + lc, MI, ne);
      ry[q] = gload4(Y, ldy, j0 + lr + 64 * q, n0 + lc, MJ, ne);
    }
  };
  auto store = [&](int buf) {
#pragma unroll
    for (int q = 0; q < 2; ++q)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        sx[buf][(lr + 64 * q) * kGP + lc + e] = rx[q][e];
        sy[buf][(lr + 64 * q) * kGP + lc + e] = ry[q][e];
      }
  };
  if (nb < ne) {
    load(nb);
    store(0);
    __syncthreads();
    int buf = 0;
    for (int64_t n0 = nb; n0 < ne; n0 += kGK) {
      const bool more = n0 + kGK < ne;
      if (more) load(n0 + kGK);
      const float* px = sx[buf];
      const float* py = sy[buf];
#pragma unroll
      for (int ks = 0; ks < kGK / 2; ++ks) {
        const int kk = 2 * ks + (lane >> 5);
        float a[2], b[2];
#pragma unroll
        for (int t2 = 0; t2 < 2; ++t2) {
          a[t2] = px[(wi + 32 * t2 + (lane & 31)) * kGP + kk];
          b[t2] = py[(wj + 32 * t2 + (lane & 31)) * kGP + kk];
        }
#pragma unroll
        for (int ta = 0; ta < 2; ++ta)
#pragma unroll
          for (int tb = 0; tb < 2; ++tb) acc[ta][tb] = mfma32x32x2(a[ta], b[tb], acc[ta][tb]);
      }
      if (more) store(buf ^ 1);
      __syncthreads();
      buf ^= 1;
    }
  }
  float* out = ws + (int64_t)blockIdx.z * split_stride;
#pragma unroll
  for (int ta = 0; ta < 2; ++ta)
#pragma unroll
    for (int tb = 0; tb < 2; ++tb) {
      const int64_t j = j0 + wj + 32 * tb + (lane & 31);
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int64_t i = i0 + wi + 32 * ta + acc_row(e, lane);
        if (i < MI && j < MJ) out[i * ldw + j] = acc[ta][tb][e];
      }
    }
}

// out[i][j] = alpha * sum_z ws[z][i][j]  (TRI: j <= i only, zero above).
__global__ __launch_bounds__(256) void gram_reduce_kernel(const float* __restrict__ ws, int64_t ldw,
                                                          int64_t split_stride, int nsplit, int64_t MI, int64_t MJ,
                                                          float alpha, int tri, float* __restrict__ out,
                                                          int64_t ldo) {
  const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (idx >= MI * MJ) return;
  const int64_t i = idx / MJ, j = idx % MJ;
  float v = 0.f;
  if (!tri || j <= i) {
    for (int z = 0; z < nsplit; ++z) v += ws[(int64_t)z * split_stride + i * ldw + j];
    v *= alpha;
  }
  out[i * ldo + j] = v;
}

// Narrow grams (MJ <= 16, e.g. g_q_mu = A G_mu^T with K columns): a 128-column
// MFMA tile would be 1/16 used, so lanes stride over n instead: wave w keeps RW
// rows x JMAX columns of sums (RW JMAX = 64 registers), each X element is read
// once, Y's rows per 4 RW-row block; the lane and chunk sums are float64.
template <int JMAX>
__global__ __launch_bounds__(256) void gram_narrow_kernel(const float* __restrict__ X, int64_t ldx, int64_t MI,
                                                          const float* __restrict__ Y, int64_t ldy, int64_t MJ,
                                                          int64_t N, int64_t chunk, double* __restrict__ part) {
  constexpr int RW = 64 / JMAX;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t i0 = ((int64_t)blockIdx.x * 4 + w) * RW;
  const int64_t nb = (int64_t)blockIdx.y * chunk, ne = nb + chunk < N ? nb + chunk : N;
  float acc[RW][JMAX];
#pragma unroll
  for (int r = 0; r < RW; ++r)
#pragma unroll
    for (int j = 0; j < JMAX; ++j) acc[r][j] = 0.f;
  for (int64_t n = nb + lane; n < ne; n += 64) {
    float y[JMAX], x[RW];
#pragma unroll
    for (int j = 0; j < JMAX; ++j) y[j] = j < MJ ? Y[(int64_t)j * ldy + n] : 0.f;
#pragma unroll
    for (int r = 0; r < RW; ++r) x[r] = i0 + r < MI ? X[(i0 + r) * ldx + n] : 0.f;
#pragma unroll
    for (int r = 0; r < RW; ++r)
#pragma unroll
      for (int j = 0; j < JMAX; ++j) acc[r][j] = fmaf(x[r], y[j], acc[r][j]);
  }
#pragma unroll
  for (int r = 0; r < RW; ++r)
#pragma unroll
    for (int j = 0; j < JMAX; ++j) {
      double v = (double)acc[r][j];
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
      if (lane == 0 && i0 + r < MI && j < MJ) part[((int64_t)blockIdx.y * MI + i0 + r) * MJ + j] = v;
    }
}

// out[i][j] = alpha * sum over the chunks of part[ch][i][j] (fixed order).
__global__ __launch_bounds__(256) void gram_narrow_fold_kernel(const double* __restrict__ part, int nch, int64_t MI,
                                                               int64_t MJ, float alpha, float* __restrict__ out,
                                                               int64_t ldo) {
  const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (idx >= MI * MJ) return;
  double v = 0.0;
  for (int ch = 0; ch < nch; ++ch) v += part[(int64_t)ch * MI * MJ + idx];
  out[(idx / MJ) * ldo + idx % MJ] = (float)(alpha * v);
}


// ------------------------------------------------------------------ x6 gram
// out[b][i][j] = alpha * sum_n X_b[i][n] (w_b[n]) Y_b[j][n] at f32 accuracy on
// the bf16 MFMA: each 32-wide n chunk is loaded as f32 (optionally scaled by
// the weight w_b[n]), split into hi/mid/lo bf16 planes on the fly and staged
// in LDS as 32x32x16 operand fragments; six plane products per fragment pair
// (mfma_x6).  The contraction is over n, so both operands use the same lane
// -> k assignment (lane (r, h), element j <-> n0 + 16 s + 8 h + j) and no
// permutation is needed.  128 x 128 output tile per workgroup (4 waves of
// 64 x 64), split-K over blockIdx.z into a workspace, batch over blockIdx.y;
// gram_x6_reduce_kernel sums the splits in a fixed order (deterministic).
constexpr int kXC = 32;    // n per chunk = two bf16 k-steps
constexpr int kXG = 3200;  // LDS bytes per (32-row block, k-step) group: 3 planes x 1 KiB + 128 B pad

// Split 4 consecutive n-values of one row into the three planes and store them
// as half of a lane's 16-B fragment slot (plane stride 1 KiB).
__device__ __forceinline__ void stash4(char* dst, floatx4 v) {
  typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
  bf16x4 h, m, l;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    __bf16 a, b, c;
    split3(v[j], a, b, c);
    h[j] = a; m[j] = b; l[j] = c;
  }
  *reinterpret_cast<bf16x4*>(dst) = h;
  *reinterpret_cast<bf16x4*>(dst + 1024) = m;
  *reinterpret_cast<bf16x4*>(dst + 2048) = l;
}

// Split-f16 variant: 4 consecutive values, scaled by a power of two, as fp16
// hi / lo planes (see mgp_common.hpp, split-f16 images).
__device__ __forceinline__ void stash4h(char* dst, floatx4 v, float scale) {
  typedef _Float16 halfx4 __attribute__((ext_vector_type(4)));
  halfx4 h, l;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const float x = v[j] * scale;
    const _Float16 hi = (_Float16)x;
    h[j] = hi;
    l[j] = (_Float16)(x - (float)hi);
  }
  *reinterpret_cast<halfx4*>(dst) = h;
  *reinterpret_cast<halfx4*>(dst + 1024) = l;
}

// 768 threads in two roles, three waves per SIMD: one consumer (waves 0-3)
// multiplies one LDS buffer (64 x 64 of the tile each) while two producers
// (waves 4-11; two waves per SIMD double the VALU issue rate of one) load the
// next f32 chunks (two chunks ahead, in registers), split them and store the
// fragments into the other buffer.  One barrier per chunk.
// F16: the chunks are split into scaled fp16 hi / lo planes instead (xb, yb, wb:
// device bounds of |X|, |Y| and |W|, the scales 2^img_exp(xb), 2^img_exp(yb wb)),
// three f16 products per fragment pair; the accumulators are unscaled on store.
// RS (with F16): xb / yb are per-row bounds (xb[i] >= max_n |X[i][n]|, yb[j] likewise),
// each row split at its own scale 2^min(img_exp, 120) and the output unscaled per row
// and column -- rows of very different size (g_Kuf, A = L^-1 Kuf) keep their 22 bits.
template <bool TRI, bool WEIGHT, bool F16 = false, bool RS = false>
__global__ __launch_bounds__(768, 1) void gram_x6_kernel(const float* __restrict__ X, int64_t ldx, int64_t sx,
                                                         int64_t MI, const float* __restrict__ Y, int64_t ldy,
                                                         int64_t sy, int64_t MJ, const float* __restrict__ W,
                                                         int64_t sw, int64_t N, int64_t nper, int nbj, int tiles,
                                                         int batch, int nsplit, float* __restrict__ ws,
                                                         int64_t bstride, int64_t zstride,
                                                         const float* __restrict__ xb = nullptr,
                                                         const float* __restrict__ yb = nullptr,
                                                         const float* __restrict__ wb = nullptr) {
  // per buffer: [32-row block][k-step] groups of [plane][lane] 16-B fragment slots
  __shared__ __attribute__((aligned(16))) char sX[2][8 * kXG], sY[2][8 * kXG];
  // item: when the splits come in multiples of 8, split z runs on XCD z % 8 and
  // every (tile, batch) item of a split is adjacent there (one n-slab per L2)
  int q, b, z;
  {
    const int id = blockIdx.x, items = tiles * batch;
    if (nsplit % 8 == 0) {
      const int x = id & 7, j = id >> 3;
      z = x + 8 * (j / items);
      const int rem = j % items;
      q = rem % tiles;
      b = rem / tiles;
    } else {
      q = id % tiles;
      b = (id / tiles) % batch;
      z = id / items;
    }
  }
  int bi, bj;
  if (TRI) {
    bi = (int)((sqrtf(8.f * q + 1.f) - 1.f) * 0.5f);
    while ((bi + 1) * (bi + 2) / 2 <= q) ++bi;
    while (bi * (bi + 1) / 2 > q) --bi;
    bj = q - bi * (bi + 1) / 2;
  } else {
    bi = q / nbj;
    bj = q % nbj;
  }
  X += b * sx;
  Y += b * sy;
  if (WEIGHT) W += b * sw;
  const int64_t i0 = (int64_t)bi * kGT, j0 = (int64_t)bj * kGT;
  const int64_t nb = (int64_t)z * nper;
  const int64_t ne = (nb + nper < N) ? nb + nper : N;
  const int64_t nch = nb < ne ? (ne - nb + kXC - 1) / kXC : 0;
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const bool producer = w >= 4;
  float xs = 1.f, ys = 1.f, unscale = 1.f;
  if constexpr (F16 && !RS) {
    const int ex = img_exp(*xb), ey = img_exp(*yb * (WEIGHT ? *wb : 1.f));
    xs = ldexpf(1.f, ex);
    ys = ldexpf(1.f, ey);
    unscale = ldexpf(1.f, -(ex + ey));
  }

  // ---- producer state: thread loads 4 consecutive n (column group cg) of rows
  // 32 q + rr (q = q0, q0 + 1) of both tiles.  Lane l of producer wave pw (0..7):
  // rr = 8 (pw % 4) + (l / 2) % 8, q0 = 2 (pw / 4), cg = 2 (l / 16) + l % 2, so a
  // wave reads 8 rows x 128 B per load and each 16-lane group of a ds_write_b64
  // (one (k-step, lane half) pair: cg / 4, (cg / 2) % 2) stores 8 rows x 16 B =
  // 128 contiguous bytes.
  const int pw = w - 4;
  const int rr = 8 * (pw & 3) + ((lane >> 1) & 7), cg = 2 * (lane >> 4) + (lane & 1);
  const int q0 = 2 * ((pw >> 2) & 1);
  const int soff = (cg >> 2) * kXG + (rr + 32 * ((cg >> 1) & 1)) * 16 + (cg & 1) * 8;
  float xsq[2] = {xs, xs}, ysq[2] = {ys, ys};  // this producer thread's two rows of each tile
  if constexpr (RS) {
    if (producer) {
#pragma unroll
      for (int qq = 0; qq < 2; ++qq) {
        const int64_t ri = i0 + 32 * (q0 + qq) + rr, rj = j0 + 32 * (q0 + qq) + rr;
        xsq[qq] = ldexpf(1.f, ri < MI ? min(img_exp(xb[ri]), 120) : 0);
        ysq[qq] = ldexpf(1.f, rj < MJ ? min(img_exp(yb[rj]), 120) : 0);
      }
    }
  }
  // buffer loads: rows beyond the matrix fall outside the resource and read 0;
  // the one partial chunk at the end of n is masked when it is stashed
  const int64_t rows_x = MI - i0 < kGT ? MI - i0 : kGT, rows_y = MJ - j0 < kGT ? MJ - j0 : kGT;
  const __amdgpu_buffer_rsrc_t rX =
      __builtin_amdgcn_make_buffer_rsrc((void*)(X + i0 * ldx), (short)0, (int)(uint32_t)(rows_x * ldx * 4), 0x00020000);
  const __amdgpu_buffer_rsrc_t rY =
      __builtin_amdgcn_make_buffer_rsrc((void*)(Y + j0 * ldy), (short)0, (int)(uint32_t)(rows_y * ldy * 4), 0x00020000);
  const __amdgpu_buffer_rsrc_t rW =
      __builtin_amdgcn_make_buffer_rsrc((void*)W, (short)0, (int)(uint32_t)(WEIGHT ? N * 4 : 0), 0x00020000);
  const uint32_t vx = (uint32_t)((32 * q0 + rr) * ldx + 4 * cg) * 4u;
  const uint32_t vy = (uint32_t)((32 * q0 + rr) * ldy + 4 * cg) * 4u;
  const uint32_t qx = (uint32_t)(32 * ldx * 4), qy = (uint32_t)(32 * ldy * 4);
  struct Regs { floatx4 x[2], y[2], w; };
  Regs ra, rb;
  auto load = [&](Regs& r, int64_t c) {
    const uint32_t so = (uint32_t)((nb + c * kXC) * 4);
#pragma unroll
    for (int qq = 0; qq < 2; ++qq) {
      r.x[qq] = __builtin_bit_cast(floatx4, __builtin_amdgcn_raw_buffer_load_b128(rX, vx + qq * qx, so, 0));
      r.y[qq] = __builtin_bit_cast(floatx4, __builtin_amdgcn_raw_buffer_load_b128(rY, vy + qq * qy, so, 0));
    }
    if (WEIGHT) r.w = __builtin_bit_cast(floatx4, __builtin_amdgcn_raw_buffer_load_b128(rW, 16u * cg, so, 0));
  };
  auto stash = [&](Regs& r, int64_t c, int buf) {
    const int64_t n0 = nb + c * kXC;
    if (n0 + kXC > ne) {  // the last, partial chunk: zero the columns >= ne
#pragma unroll
      for (int e = 0; e < 4; ++e)
        if (n0 + 4 * cg + e >= ne) {
#pragma unroll
          for (int qq = 0; qq < 2; ++qq) {
            r.x[qq][e] = 0.f;
            r.y[qq][e] = 0.f;
          }
        }
    }
#pragma unroll
    for (int qq = 0; qq < 2; ++qq) {
      if constexpr (F16) {
        stash4h(sX[buf] + 2 * (q0 + qq) * kXG + soff, r.x[qq], xsq[qq]);
        stash4h(sY[buf] + 2 * (q0 + qq) * kXG + soff, WEIGHT ? r.y[qq] * r.w : r.y[qq], ysq[qq]);
      } else {
        stash4(sX[buf] + 2 * (q0 + qq) * kXG + soff, r.x[qq]);
        stash4(sY[buf] + 2 * (q0 + qq) * kXG + soff, WEIGHT ? r.y[qq] * r.w : r.y[qq]);
      }
    }
  };

  // ---- consumer state: wave w multiplies X blocks wb, wb + 1 by Y blocks vb, vb + 1
  const int wb_ = (w >> 1) * 2, vb = (w & 1) * 2;
  floatx16 acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[a][c][e] = 0.f;
  auto compute = [&](int buf) {
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      constexpr int NP = F16 ? 2 : 3;
      bf16x8 c[2][3];
#pragma unroll
      for (int t2 = 0; t2 < 2; ++t2)
#pragma unroll
        for (int p = 0; p < NP; ++p)
          c[t2][p] = *reinterpret_cast<const bf16x8*>(sY[buf] + (2 * (vb + t2) + ks) * kXG + p * 1024 + lane * 16);
#pragma unroll
      for (int ta = 0; ta < 2; ++ta) {
        bf16x8 a[3];
#pragma unroll
        for (int p = 0; p < NP; ++p)
          a[p] = *reinterpret_cast<const bf16x8*>(sX[buf] + (2 * (wb_ + ta) + ks) * kXG + p * 1024 + lane * 16);
#pragma unroll
        for (int tb = 0; tb < 2; ++tb) {
          if constexpr (F16)
            acc[ta][tb] = mfma_fmt<2, true>(a, c[tb], acc[ta][tb]);
          else
            acc[ta][tb] = mfma_x6(a, c[tb], acc[ta][tb]);
        }
      }
      // x6: keep the next k-step's fragment reads after these MFMAs (registers)
      if constexpr (!F16) __builtin_amdgcn_sched_barrier(0);
    }
  };

  // chunk c lives in register set c % 4 and LDS buffer c % 2; the load of chunk
  // c + 4 is issued as soon as chunk c is stashed (four chunk phases cover its
  // latency).  The two roles run separate loops with the same barriers (one per
  // chunk), so neither role's registers are live in the other's loop.
  if (producer) {
    Regs r2, r3;
    // phase of chunk c: stash it (set c % 4, buffer c % 2), load chunk c + 4 (past the
    // data the buffer resources read zeros; never stashed), one barrier.  Full rounds
    // of four phases in the loop, the rest after it (no exit inside the loop body, so
    // the register sets need no copies at the back edge)
    auto phase = [&](Regs& r, int64_t c, int buf) {
      if (c < nch) stash(r, c, buf);
      load(r, c + 4);
      __syncthreads();
    };
    load(ra, 0);
    load(rb, 1);
    load(r2, 2);
    load(r3, 3);
    if (nch > 0) stash(ra, 0, 0);
    load(ra, 4);
    __syncthreads();
    int64_t c = 1;
    for (; c + 3 <= nch; c += 4) {
      phase(rb, c, 1);
      phase(r2, c + 1, 0);
      phase(r3, c + 2, 1);
      phase(ra, c + 3, 0);
    }
    if (c <= nch) phase(rb, c, 1);
    if (c + 1 <= nch) phase(r2, c + 1, 0);
    if (c + 2 <= nch) phase(r3, c + 2, 1);
    return;
  }
  __syncthreads();
  // chunk pairs, then the odd chunk after the loop: a break between the two halves
  // made the compiler copy all accumulators at every back edge (64 moves behind a
  // drained MFMA pipe per chunk pair)
  int64_t i = 0;
  for (; i + 1 < nch; i += 2) {
    compute(0);
    __syncthreads();
    compute(1);
    __syncthreads();
  }
  if (i < nch) {
    compute(0);
    __syncthreads();
  }
  float* out = ws + (int64_t)z * zstride + (int64_t)b * bstride;
#pragma unroll
  for (int ta = 0; ta < 2; ++ta)
#pragma unroll
    for (int tb = 0; tb < 2; ++tb) {
      const int64_t j = j0 + 32 * (vb + tb) + (lane & 31);
      float uj = unscale;
      if constexpr (RS) uj = ldexpf(1.f, j < MJ ? -min(img_exp(yb[j]), 120) : 0);
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int64_t i = i0 + 32 * (wb_ + ta) + acc_row(e, lane);
        if (i < MI && j < MJ) {
          if constexpr (RS)
            out[i * MJ + j] = acc[ta][tb][e] * ldexpf(1.f, -min(img_exp(xb[i]), 120)) * uj;
          else
            out[i * MJ + j] = F16 ? acc[ta][tb][e] * unscale : acc[ta][tb][e];
        }
      }
    }
}

// ------------------------------------------------------------------ weighted gram on a row image, entry pairs
// ws[z][b][i][j] = sum_n X[i][n] W_b[n] Y[j][n] over split z (the P_k grams of the
// conditional backward): X (as its row image, split once) and the f32 Y are
// shared by the batch, so one workgroup takes TWO batch entries of a tile: X's
// fragments and Y's chunk are loaded once per chunk and Y is weighted and split
// per entry (half the L2 -> CU traffic and a third less split work than one
// entry per workgroup on gram_x6_kernel).  768 threads: consumer waves 0-7
// (entry e = w / 4, 64 x 64 of the tile each, two per SIMD), producer waves 8-15
// (kRows2PW; 8-11 with 4).
// Chunks of 32 n, double-buffered, one barrier each.
#ifndef MGP_ROWS2_PW
#define MGP_ROWS2_PW 8
#endif
constexpr int kRows2PW = MGP_ROWS2_PW;
constexpr int kXG2 = 2176;  // LDS bytes per (32-row block, k-step) group: 2 planes x 1 KiB + 128 B pad

// PW: producer waves (4: 768 threads; 8, the default: 1024 threads, each producer
// thread taking half the row groups and image units of a chunk, 118 VGPRs, four
// waves per SIMD -- the P_k gram 2.06 -> 1.92 ms in the training step,
// profiles/r05zd_rows2_pw8_train_ab.log)
template <bool TRI, int PW = 4>
__global__ __launch_bounds__(512 + 64 * PW, 1) void gram_rows2_kernel(const char* __restrict__ Ximg, int64_t nns, int64_t MI,
                                                            const float* __restrict__ Y, int64_t ldy, int64_t MJ,
                                                           const float* __restrict__ W, int64_t sw, int64_t N,
                                                           int64_t nper, int nbj, int tiles, int pairs, int batch,
                                                           int nsplit, float* __restrict__ ws, int64_t bstride,
                                                           int64_t zstride, const float* __restrict__ xb,
                                                           const float* __restrict__ yb,
                                                           const float* __restrict__ wb) {
  __shared__ __attribute__((aligned(16))) char sX[2][8 * kXG2], sY[2][2][8 * kXG2];
  int q, pr, z;
  {
    // the entry pairs of a tile are adjacent (one XCD, in flight together): A's chunks
    // are fetched into L2 once for all of them (tile-outer order fetched them once per
    // pair, 2.85 GB per launch at c3)
    const int id = blockIdx.x, items = tiles * pairs;
    if (nsplit % 8 == 0) {
      const int x = id & 7, j = id >> 3;
      z = x + 8 * (j / items);
      const int rem = j % items;
      pr = rem % pairs;
      q = rem / pairs;
    } else {
      pr = id % pairs;
      q = (id / pairs) % tiles;
      z = id / items;
    }
  }
  int bi, bj;
  if (TRI) {
    bi = (int)((sqrtf(8.f * q + 1.f) - 1.f) * 0.5f);
    while ((bi + 1) * (bi + 2) / 2 <= q) ++bi;
    while (bi * (bi + 1) / 2 > q) --bi;
    bj = q - bi * (bi + 1) / 2;
  } else {
    bi = q / nbj;
    bj = q % nbj;
  }
  const int b0 = 2 * pr;
  const bool two = b0 + 1 < batch;
  const int64_t i0 = (int64_t)bi * kGT, j0 = (int64_t)bj * kGT;
  const int64_t nb = (int64_t)z * nper;
  const int64_t ne = (nb + nper < N) ? nb + nper : N;
  const int64_t nch = nb < ne ? (ne - nb + kXC - 1) / kXC : 0;
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  // X's image carries 2^ex; the weighted Y is split at 2^ey (bound |Y| |W|)
  const int ex = img_exp(*xb), ey = img_exp(*yb * *wb);
  const float ys = ldexpf(1.f, ey), unscale = ldexpf(1.f, -(ex + ey));

  // ---- producer state.  Y: thread pt (0..255) of wave pw = pt / 64 loads 4
  // consecutive n (column group cg) of rows 32 qq + rr, qq = 0..3, rr = 8 pw +
  // (lane / 2) % 8, cg = 2 (lane / 16) + lane % 2 (gram_x6_kernel's lane pattern).
  // X: 16-B image units u = pt + 256 s of the chunk's 8 blocks (row block u / 256,
  // k-step (u / 128) % 2) -> LDS group u / 128, byte (u % 128) 16.
  constexpr int QN = 16 / PW;   // row groups of Y (and 16-B X units) per producer thread per chunk
  const int pt = tid - 512, pw = pt >> 6, ph = pw >> 2;
  const int rr = 8 * (pw & 3) + ((lane >> 1) & 7), cg = 2 * (lane >> 4) + (lane & 1);
  const int soff = (cg >> 2) * kXG2 + (rr + 32 * ((cg >> 1) & 1)) * 16 + (cg & 1) * 8;
  const int64_t rows_x = MI - i0 < kGT ? MI - i0 : kGT, rows_y = MJ - j0 < kGT ? MJ - j0 : kGT;
  const __amdgpu_buffer_rsrc_t rX = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(Ximg + 4 * (int64_t)bi * nns * 2048), (short)0, (int)(uint32_t)((rows_x + 31) / 32 * nns * 2048),
      0x00020000);
  const __amdgpu_buffer_rsrc_t rY =
      __builtin_amdgcn_make_buffer_rsrc((void*)(Y + j0 * ldy), (short)0, (int)(uint32_t)(rows_y * ldy * 4), 0x00020000);
  const __amdgpu_buffer_rsrc_t rW0 =
      __builtin_amdgcn_make_buffer_rsrc((void*)(W + b0 * sw), (short)0, (int)(uint32_t)(N * 4), 0x00020000);
  const __amdgpu_buffer_rsrc_t rW1 = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(W + (two ? b0 + 1 : b0) * sw), (short)0, (int)(uint32_t)(N * 4), 0x00020000);
  const uint32_t vy = (uint32_t)(rr * ldy + 4 * cg) * 4u, qy = (uint32_t)(32 * ldy * 4);
  uint32_t vxi[QN];
  int dxi[QN];
#pragma unroll
  for (int s = 0; s < QN; ++s) {
    const int u = (pt & 255) + 256 * (s + QN * ph), g = u >> 7;
    vxi[s] = (uint32_t)(((g >> 1) * nns + (g & 1)) * 2048 + (u & 127) * 16);
    dxi[s] = g * kXG2 + (u & 127) * 16;
  }
  struct Regs { u32x4v x[QN]; floatx4 y[QN], w0, w1; };
  Regs ra, rb;
  // loads are unconditional (past the data the resources read zeros or unused
  // bytes): every path issues the same count, so the wait counts stay tight
  auto load = [&](Regs& r, int64_t c) {
    const int64_t n0 = nb + c * kXC;
    const uint32_t so = (uint32_t)(n0 * 4), xso = (uint32_t)(n0 / 16 * 2048);
#pragma unroll
    for (int s = 0; s < QN; ++s) r.x[s] = __builtin_amdgcn_raw_buffer_load_b128(rX, vxi[s], xso, 0);
#pragma unroll
    for (int qi = 0; qi < QN; ++qi)
      r.y[qi] = __builtin_bit_cast(floatx4,
                                   __builtin_amdgcn_raw_buffer_load_b128(rY, vy + (qi + QN * ph) * qy, so, 0));
    r.w0 = __builtin_bit_cast(floatx4, __builtin_amdgcn_raw_buffer_load_b128(rW0, 16u * cg, so, 0));
    r.w1 = __builtin_bit_cast(floatx4, __builtin_amdgcn_raw_buffer_load_b128(rW1, 16u * cg, so, 0));
  };
  auto stash = [&](Regs& r, int64_t c, int buf) {
    // Y's columns >= ne are zeroed (the last chunk; X's image is zero there) by
    // selects, not branches: a branch here costs the loads' wait-count tracking
    const int lim = (int)(ne - (nb + c * kXC)) - 4 * cg;
#pragma unroll
    for (int e2 = 0; e2 < 4; ++e2)
#pragma unroll
      for (int qi = 0; qi < QN; ++qi) r.y[qi][e2] = e2 < lim ? r.y[qi][e2] : 0.f;
#pragma unroll
    for (int s = 0; s < QN; ++s) *reinterpret_cast<u32x4v*>(sX[buf] + dxi[s]) = r.x[s];
#pragma unroll
    for (int qi = 0; qi < QN; ++qi) {
      const int qq = qi + QN * ph;
      stash4h(sY[buf][0] + 2 * qq * kXG2 + soff, r.y[qi] * r.w0, ys);
      stash4h(sY[buf][1] + 2 * qq * kXG2 + soff, r.y[qi] * r.w1, ys);
    }
  };

  // ---- consumer state: wave w (entry e) multiplies X blocks wb_, wb_ + 1 by the
  // weighted Y blocks vb, vb + 1
  const int e = w >> 2, wl = w & 3;
  const int wb_ = (wl >> 1) * 2, vb = (wl & 1) * 2;
  floatx16 acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
      for (int k = 0; k < 16; ++k) acc[a][c][k] = 0.f;
  auto compute = [&](int buf) {
    const char* sy_ = sY[buf][e];
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      // all 8 fragment reads of the k-step in flight before its first MFMA
      bf16x8 c[2][3], a[2][3];
#pragma unroll
      for (int t2 = 0; t2 < 2; ++t2)
#pragma unroll
        for (int p = 0; p < 2; ++p) {
          c[t2][p] = *reinterpret_cast<const bf16x8*>(sy_ + (2 * (vb + t2) + ks) * kXG2 + p * 1024 + lane * 16);
          a[t2][p] = *reinterpret_cast<const bf16x8*>(sX[buf] + (2 * (wb_ + t2) + ks) * kXG2 + p * 1024 + lane * 16);
        }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int ta = 0; ta < 2; ++ta)
#pragma unroll
        for (int tb = 0; tb < 2; ++tb) acc[ta][tb] = mfma_fmt<2, true>(a[ta], c[tb], acc[ta][tb]);
    }
  };

  // chunk c in register set c % 3 and LDS buffer c % 2; the load of chunk c + 3
  // is issued as soon as chunk c is stashed (three chunk phases cover it)
  if (w >= 8) {
    Regs rc;
    auto phase = [&](Regs& r, int64_t c, int buf) {
      if (c < nch) stash(r, c, buf);
      load(r, c + 3);
      __syncthreads();
    };
    load(ra, 0);
    load(rb, 1);
    load(rc, 2);
    if (nch > 0) stash(ra, 0, 0);
    load(ra, 3);
    __syncthreads();
    // phases of chunks 1 .. nch: full rounds of six in the loop, the rest after it
    int64_t c = 1;
    for (; c + 5 <= nch; c += 6) {
      phase(rb, c, 1);
      phase(rc, c + 1, 0);
      phase(ra, c + 2, 1);
      phase(rb, c + 3, 0);
      phase(rc, c + 4, 1);
      phase(ra, c + 5, 0);
    }
    if (c <= nch) phase(rb, c, 1);
    if (c + 1 <= nch) phase(rc, c + 1, 0);
    if (c + 2 <= nch) phase(ra, c + 2, 1);
    if (c + 3 <= nch) phase(rb, c + 3, 0);
    if (c + 4 <= nch) phase(rc, c + 4, 1);
    return;
  }
  __syncthreads();
  // chunk pairs, then the odd chunk after the loop: a break between the two halves
  // made the compiler copy all accumulators at every back edge (64 moves behind a
  // drained MFMA pipe per chunk pair)
  int64_t i = 0;
  for (; i + 1 < nch; i += 2) {
    compute(0);
    __syncthreads();
    compute(1);
    __syncthreads();
  }
  if (i < nch) {
    compute(0);
    __syncthreads();
  }
  if (e == 1 && !two) return;
  float* out = ws + (int64_t)z * zstride + (int64_t)(b0 + e) * bstride;
#pragma unroll
  for (int ta = 0; ta < 2; ++ta)
#pragma unroll
    for (int tb = 0; tb < 2; ++tb) {
      const int64_t j = j0 + 32 * (vb + tb) + (lane & 31);
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        const int64_t i = i0 + 32 * (wb_ + ta) + acc_row(k, lane);
        if (i < MI && j < MJ) out[i * MJ + j] = acc[ta][tb][k] * unscale;
      }
    }
}

// out[b][i][j] = alpha * sum_z ws[z][b][i][j]; mode 0 full, 1 lower triangle
// (zero above), 2 symmetric (the upper triangle mirrors the lower).  Grid
// (32-column tile, 32-row tile, batch), 256 threads = 32 rows x 8 four-column
// groups: the source tile (the mirrored one above the diagonal in mode 2) is
// summed with 16-B row-contiguous loads, four splits in flight per thread (fixed
// order: split z into partial z % 4, then (p0 + p1) + (p2 + p3)), into LDS and
// written out transposed where needed -- coalesced both ways, no index divisions.
__global__ __launch_bounds__(256) void gram_x6_reduce_kernel(const float* __restrict__ ws, int64_t bstride,
                                                             int64_t zstride, int nsplit, int64_t MI, int64_t MJ,
                                                             float alpha, int mode, float* __restrict__ out,
                                                             int64_t ldo, int64_t so) {
  __shared__ float sT[32][33];
  const int tx = threadIdx.x & 7, ty = threadIdx.x >> 3;
  const int64_t bi = blockIdx.y, bj = blockIdx.x, b = blockIdx.z;
  const bool mirror = mode == 2 && bj > bi;
  const bool skip = mode == 1 && bj > bi;  // a zero tile
  const int64_t ti = mirror ? bj : bi, tj = mirror ? bi : bj;
  if (!skip) {
    const int64_t r = 32 * ti + ty, c = 32 * tj + 4 * tx;
    floatx4 v = {0.f, 0.f, 0.f, 0.f};
    if (r < MI && c < MJ) {
      const float* src = ws + b * bstride + r * MJ + c;
      if (c + 4 <= MJ && (MJ & 3) == 0) {  // 16-B aligned rows (zstride, bstride are multiples of MJ)
        floatx4 p[4] = {v, v, v, v};
        int z = 0;
        for (; z + 4 <= nsplit; z += 4) {
#pragma unroll
          for (int u = 0; u < 4; ++u) p[u] += *reinterpret_cast<const floatx4*>(src + (int64_t)(z + u) * zstride);
        }
        for (; z < nsplit; ++z) p[z & 3] += *reinterpret_cast<const floatx4*>(src + (int64_t)z * zstride);
        v = (p[0] + p[1]) + (p[2] + p[3]);
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e)
          if (c + e < MJ)
            for (int z = 0; z < nsplit; ++z) v[e] += src[(int64_t)z * zstride + e];
      }
    }
#pragma unroll
    for (int e = 0; e < 4; ++e) sT[ty][4 * tx + e] = v[e] * alpha;
  }
  __syncthreads();
  const int64_t i = 32 * bi + ty, j0 = 32 * bj + 4 * tx;
  if (i >= MI || j0 >= MJ) return;
  floatx4 o;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const int lj = 4 * tx + e;
    const int64_t j = j0 + e;
    if (skip || (mode == 1 && j > i))
      o[e] = 0.f;
    else if (mirror || (mode == 2 && bi == bj && j > i))
      o[e] = sT[lj][ty];
    else
      o[e] = sT[ty][lj];
  }
  float* dst = out + b * so + i * ldo + j0;
  if (j0 + 4 <= MJ && ((ldo | so) & 3) == 0 && ((uintptr_t)out & 15) == 0) {
    *reinterpret_cast<floatx4*>(dst) = o;
  } else {
#pragma unroll
    for (int e = 0; e < 4; ++e)
      if (j0 + e < MJ) dst[e] = o[e];
  }
}

// Row image of X (M x N f32) for the gram's X side: [row block rb][k-step ns]
// blocks of [plane][lane] 16-B units, lane (r, h) <- row 32 rb + r, element j <-
// n = 16 ns + 8 h + j (the gram's lane -> n assignment), scaled by
// 2^img_exp(*bound) and split into fp16 hi / lo (planes 0 / 1); zero beyond M, N.
// Workgroup: one row block, 8 k-steps; thread: units u = tid + 256 s.
__global__ __launch_bounds__(256) void split_rows_f16_kernel(const float* __restrict__ X, int64_t ldx, int64_t M,
                                                             int64_t N, int nns, const float* __restrict__ bound,
                                                             bf16x8* __restrict__ img) {
  const int64_t rb = blockIdx.y;
  const float scale = ldexpf(1.f, img_exp(*bound));
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    const int u = threadIdx.x + 256 * s, lane = u & 63;
    const int64_t ns = 8 * (int64_t)blockIdx.x + (u >> 6);
    if (ns >= nns) continue;
    const int64_t row = 32 * rb + (lane & 31), n = 16 * ns + 8 * (lane >> 5);
    float v[8];
    if (row < M && n + 7 < N) {
      const floatx4 a = *reinterpret_cast<const floatx4*>(X + row * ldx + n);
      const floatx4 b = *reinterpret_cast<const floatx4*>(X + row * ldx + n + 4);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        v[j] = a[j];
        v[4 + j] = b[j];
      }
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = (row < M && n + j < N) ? X[row * ldx + n + j] : 0.f;
    }
    store_split_f16(img + (rb * nns + ns) * 128 + lane, v, scale);
  }
}

}  // namespace mgp

using namespace mgp;

extern "C" int64_t mgp_rows_f16_ksteps(int64_t N) { return N <= 0 ? 0 : (N + kXC - 1) / kXC * (kXC / 16); }

extern "C" size_t mgp_rows_f16_bytes(int64_t M, int64_t N) {
  if (M <= 0 || N <= 0) return 16;
  return (size_t)((M + 31) / 32) * (size_t)mgp_rows_f16_ksteps(N) * 2048;
}

extern "C" int mgp_split_rows_f16(const float* X, int64_t ldx, int64_t M, int64_t N, const float* bound, void* img,
                                  size_t img_bytes, mgp_stream_t stream) {
  if (!X) return -1;
  if (ldx < N || ldx % 4) return -2;
  if (M < 0) return -3;
  if (N < 0) return -4;
  if (!bound) return -5;
  if (!img) return -6;
  if (M == 0 || N == 0) return MGP_OK;
  if (img_bytes < mgp_rows_f16_bytes(M, N)) return MGP_ERR_WORKSPACE;
  if (!aligned16(X) || !aligned16(img)) return MGP_ERR_ALIGN;
  const int64_t nns = mgp_rows_f16_ksteps(N);
  if (nns >= ((int64_t)1 << 30) || (M + 31) / 32 > 65535) return MGP_ERR_UNSUPPORTED;
  hipLaunchKernelGGL(split_rows_f16_kernel, dim3((unsigned)((nns + 7) / 8), (unsigned)((M + 31) / 32)), dim3(256), 0,
                     (hipStream_t)stream, X, ldx, M, N, (int)nns, bound, (bf16x8*)img);
  return launch_status();
}

static int gram_splits(int64_t N, int tiles) {
  // aim for >= 1024 workgroups, each with >= 1024 points
  int s = 1;
  while ((int64_t)tiles * s < 1024 && N / (2 * s) >= 1024) s *= 2;
  return s;
}

constexpr int64_t kNarrowChunk = 2048;  // n per workgroup of gram_narrow_kernel
static bool gram_narrow(int64_t MJ, int32_t tri) { return !tri && MJ <= 16; }

extern "C" size_t mgp_gram_workspace_bytes(int64_t MI, int64_t MJ, int64_t N, int32_t tri) {
  if (MI <= 0 || MJ <= 0 || N <= 0) return 16;
  if (gram_narrow(MJ, tri))
    return (size_t)((N + kNarrowChunk - 1) / kNarrowChunk) * (size_t)MI * (size_t)MJ * sizeof(double);
  const int nbi = (int)((MI + kGT - 1) / kGT), nbj = (int)((MJ + kGT - 1) / kGT);
  const int tiles = tri ? nbi * (nbi + 1) / 2 : nbi * nbj;
  return (size_t)gram_splits(N, tiles) * (size_t)MI * (size_t)MJ * sizeof(float);
}

extern "C" int mgp_gram(const float* X, int64_t ldx, int64_t MI, const float* Y, int64_t ldy, int64_t MJ,
                        int64_t N, float alpha, int32_t tri, float* out, int64_t ldo, void* workspace,
                        size_t workspace_bytes, mgp_stream_t stream) {
  if (!X) return -1;
  if (ldx < N) return -2;
  if (MI < 0) return -3;
  if (!Y) return -4;
  if (ldy < N) return -5;
  if (MJ < 0) return -6;
  if (N < 0) return -7;
  if (tri && MI != MJ) return -9;
  if (!out) return -10;
  if (ldo < MJ) return -11;
  if (MI == 0 || MJ == 0) return MGP_OK;
  if (!workspace || workspace_bytes < mgp_gram_workspace_bytes(MI, MJ, N, tri)) return MGP_ERR_WORKSPACE;
  hipStream_t s = (hipStream_t)stream;
  if (gram_narrow(MJ, tri)) {
    const int64_t nch = N > 0 ? (N + kNarrowChunk - 1) / kNarrowChunk : 0;
    if (nch > 65535 || (MI + 15) / 16 > ((int64_t)1 << 31)) return MGP_ERR_UNSUPPORTED;
    double* part = (double*)workspace;
    if (nch == 0) {
      int st = hip_status(hipMemsetAsync(part, 0, MI * MJ * sizeof(double), s));
      if (st) return st;
    } else if (MJ <= 8) {
      hipLaunchKernelGGL(gram_narrow_kernel<8>, dim3((unsigned)((MI + 31) / 32), (unsigned)nch), dim3(256), 0, s, X,
                         ldx, MI, Y, ldy, MJ, N, kNarrowChunk, part);
    } else {
      hipLaunchKernelGGL(gram_narrow_kernel<16>, dim3((unsigned)((MI + 15) / 16), (unsigned)nch), dim3(256), 0, s,
                         X, ldx, MI, Y, ldy, MJ, N, kNarrowChunk, part);
    }
    int st = launch_status();
    if (st) return st;
    hipLaunchKernelGGL(gram_narrow_fold_kernel, dim3((unsigned)((MI * MJ + 255) / 256)), dim3(256), 0, s, part,
                       (int)(nch > 0 ? nch : 1), MI, MJ, alpha, out, ldo);
    return launch_status();
  }
  const int nbi = (int)((MI + kGT - 1) / kGT), nbj = (int)((MJ + kGT - 1) / kGT);
  const int tiles = tri ? nbi * (nbi + 1) / 2 : nbi * nbj;
  const int nsplit = N > 0 ? gram_splits(N, tiles) : 1;
  int64_t nper = (N + nsplit - 1) / nsplit;
  nper = (nper + kGK - 1) / kGK * kGK;
  float* ws = (float*)workspace;
  const int64_t stride = MI * MJ;
  if (tri)
    hipLaunchKernelGGL(gram_kernel<true>, dim3(tiles, 1, nsplit), dim3(256), 0, s, X, ldx, MI, Y, ldy, MJ, N, nper,
                       nbj, ws, MJ, stride);
  else
    hipLaunchKernelGGL(gram_kernel<false>, dim3(tiles, 1, nsplit), dim3(256), 0, s, X, ldx, MI, Y, ldy, MJ, N,
                       nper, nbj, ws, MJ, stride);
  int st = launch_status();
  if (st) return st;
  hipLaunchKernelGGL(gram_reduce_kernel, dim3((unsigned)((MI * MJ + 255) / 256)), dim3(256), 0, s, ws, MJ, stride,
                     nsplit, MI, MJ, alpha, tri, out, ldo);
  return launch_status();
}

// The split-K count is costed for the MI355X's 256 CUs whatever device is current:
// a fixed count keeps the workspace size (mgp_*_workspace_bytes) and the fixed-order
// split reduction -- so the result bits -- the same on every device and CU partition
// mode (round 4; the count used to follow hipDeviceAttributeMultiprocessorCount).
constexpr int kGramCUs = 256;

// Split-K count of the 768-thread grams (items = workgroups per split, out_tiles =
// 128 x 128 output tiles the reduction sums): every workgroup of a launch holds
// the same n-count, so the launch lasts (workgroup rounds) x (chunks per workgroup
// + ~4 chunks of pipeline fill and store); the reduction reads one more tile set
// per split (~0.009 chunk times per tile, measured at c3).  Among 1, 2, 4 and the multiples
// of 8 up to 64 (one n-slab per XCD), with >= 512 points per workgroup, the
// cheapest count wins (a larger count only when >= 1 % cheaper).  The earlier
// rule (double until 2048 workgroups) left c3's P_k gram 4.5 rounds deep: 16
// splits instead of 8 take it from 2.28 to 2.12 ms (profiles/r03_gram_splits_probe.log).
static int gram_x6_splits(int64_t N, int64_t items, int64_t out_tiles) {
  const int cus = kGramCUs;
  int best = 1;
  double best_cost = 1e300;
  static const int cand[] = {1, 2, 4, 8, 16, 24, 32, 40, 48, 56, 64};
  for (int s : cand) {
    if (s > 1 && N / s < 512) break;
    const int64_t rounds = (items * s + cus - 1) / cus;
    const int64_t nch = (N + (int64_t)s * kXC - 1) / ((int64_t)s * kXC);
    const double cost = (double)rounds * (double)(nch + 4) + 0.009 * (double)out_tiles * s;
    if (cost < best_cost * 0.99) {
      best_cost = cost;
      best = s;
    }
  }
  return best;
}

static int gram_x6_tiles(int64_t MI, int64_t MJ, int tri) {
  const int nbi = (int)((MI + kGT - 1) / kGT), nbj = (int)((MJ + kGT - 1) / kGT);
  return tri ? nbi * (nbi + 1) / 2 : nbi * nbj;
}

extern "C" size_t mgp_gram_x6_workspace_bytes(int64_t MI, int64_t MJ, int64_t N, int32_t batch, int32_t mode) {
  if (MI <= 0 || MJ <= 0 || N <= 0 || batch <= 0) return 16;
  const int64_t tiles = gram_x6_tiles(MI, MJ, mode != 0);
  // the larger of the x6 kernel's count and the row-image kernel's (entry pairs)
  const int s1 = gram_x6_splits(N, tiles * batch, tiles * batch);
  const int s2 = gram_x6_splits(N, tiles * ((batch + 1) / 2), tiles * batch);
  return (size_t)(s1 > s2 ? s1 : s2) * (size_t)batch * (size_t)MI * (size_t)MJ * sizeof(float);
}

static int gram_x6_launch(const float* X, int64_t ldx, int64_t sx, int64_t MI, const float* Y, int64_t ldy,
                          int64_t sy, int64_t MJ, const float* W, int64_t sw, int64_t N, int32_t batch, float alpha,
                          int32_t mode, float* out, int64_t ldo, int64_t so, void* workspace,
                          size_t workspace_bytes, mgp_stream_t stream, const float* xb, const float* yb,
                          const float* wb, bool rs = false) {
  const bool f16 = xb != nullptr;
  if (rs && (W || !f16)) return MGP_ERR_UNSUPPORTED;
  if (!X) return -1;
  if (ldx < N || ldx % 4) return -2;
  if (batch > 1 && sx % 4) return -3;
  if (MI < 0) return -4;
  if (!Y) return -5;
  if (ldy < N || ldy % 4) return -6;
  if (batch > 1 && sy % 4) return -7;
  if (MJ < 0) return -8;
  if (W && batch > 1 && sw % 4) return -10;
  if (W && N * 4 >= ((int64_t)1 << 31)) return MGP_ERR_UNSUPPORTED;
  if (N < 0) return -11;
  if (batch < 0) return -12;
  if (mode < 0 || mode > 2) return -14;
  if (mode && MI != MJ) return -14;
  if ((int64_t)kGT * (ldx > ldy ? ldx : ldy) * 4 >= ((int64_t)1 << 32)) return MGP_ERR_UNSUPPORTED;
  if (!out) return -15;
  if (ldo < MJ) return -16;
  if (batch > 1 && so < ldo * MI) return -17;
  if (MI == 0 || MJ == 0 || batch == 0) return MGP_OK;
  if (batch > 65535) return MGP_ERR_UNSUPPORTED;  // the reduction's grid
  if (!aligned16(X) || !aligned16(Y) || (W && !aligned16(W))) return MGP_ERR_ALIGN;
  if (!workspace || workspace_bytes < mgp_gram_x6_workspace_bytes(MI, MJ, N, batch, mode)) return MGP_ERR_WORKSPACE;
  hipStream_t s = (hipStream_t)stream;
  const int tiles = gram_x6_tiles(MI, MJ, mode != 0);
  const int nbj = (int)((MJ + kGT - 1) / kGT);
  const int nsplit = N > 0 ? gram_x6_splits(N, (int64_t)tiles * batch, (int64_t)tiles * batch) : 1;
  int64_t nper = (N + nsplit - 1) / nsplit;
  nper = (nper + kXC - 1) / kXC * kXC;
  float* ws = (float*)workspace;
  const int64_t bstride = MI * MJ, zstride = (int64_t)batch * MI * MJ;
  const dim3 grid((unsigned)(tiles * batch * nsplit));
  if (rs && mode != 0)
    hipLaunchKernelGGL((gram_x6_kernel<true, false, true, true>), grid, dim3(768), 0, s, X, ldx, sx, MI, Y, ldy, sy,
                       MJ, W, sw, N, nper, nbj, tiles, (int)batch, nsplit, ws, bstride, zstride, xb, yb, wb);
  else if (rs)
    hipLaunchKernelGGL((gram_x6_kernel<false, false, true, true>), grid, dim3(768), 0, s, X, ldx, sx, MI, Y, ldy, sy,
                       MJ, W, sw, N, nper, nbj, tiles, (int)batch, nsplit, ws, bstride, zstride, xb, yb, wb);
  else {
#define MGP_GRAM_X6(TRI, WT, F16)                                                                              \
  if ((mode != 0) == TRI && (W != nullptr) == WT && f16 == F16)                                               \
    hipLaunchKernelGGL((gram_x6_kernel<TRI, WT, F16>), grid, dim3(768), 0, s, X, ldx, sx, MI, Y, ldy, sy, MJ, W, sw, \
                       N, nper, nbj, tiles, (int)batch, nsplit, ws, bstride, zstride, xb, yb, wb);
  MGP_GRAM_X6(true, true, false)
  MGP_GRAM_X6(true, false, false)
  MGP_GRAM_X6(false, true, false)
  MGP_GRAM_X6(false, false, false)
  MGP_GRAM_X6(true, true, true)
  MGP_GRAM_X6(true, false, true)
  MGP_GRAM_X6(false, true, true)
  MGP_GRAM_X6(false, false, true)
#undef MGP_GRAM_X6
  }
  int st = launch_status();
  if (st) return st;
  hipLaunchKernelGGL(gram_x6_reduce_kernel, dim3((unsigned)((MJ + 31) / 32), (unsigned)((MI + 31) / 32), (unsigned)batch),
                     dim3(256), 0, s, ws, bstride, zstride, nsplit, MI, MJ, alpha, (int)mode, out, ldo, so);
  return launch_status();
}

extern "C" int mgp_gram_x6(const float* X, int64_t ldx, int64_t sx, int64_t MI, const float* Y, int64_t ldy,
                           int64_t sy, int64_t MJ, const float* W, int64_t sw, int64_t N, int32_t batch, float alpha,
                           int32_t mode, float* out, int64_t ldo, int64_t so, void* workspace,
                           size_t workspace_bytes, mgp_stream_t stream) {
  return gram_x6_launch(X, ldx, sx, MI, Y, ldy, sy, MJ, W, sw, N, batch, alpha, mode, out, ldo, so, workspace,
                        workspace_bytes, stream, nullptr, nullptr, nullptr);
}

extern "C" int mgp_gram_f16(const float* X, int64_t ldx, int64_t sx, int64_t MI, const float* Y, int64_t ldy,
                            int64_t sy, int64_t MJ, const float* W, int64_t sw, int64_t N, int32_t batch, float alpha,
                            int32_t mode, float* out, int64_t ldo, int64_t so, const float* x_bound,
                            const float* y_bound, const float* w_bound, void* workspace, size_t workspace_bytes,
                            mgp_stream_t stream) {
  if (!x_bound) return -18;
  if (!y_bound) return -19;
  if (W && !w_bound) return -20;
  return gram_x6_launch(X, ldx, sx, MI, Y, ldy, sy, MJ, W, sw, N, batch, alpha, mode, out, ldo, so, workspace,
                        workspace_bytes, stream, x_bound, y_bound, w_bound);
}

// mgp_gram_f16 (unweighted) with per-row bounds xb[MI], yb[MJ] instead of two scalars
// (gram_x6_kernel<., false, true, true>; the conditional backward's g_Lm gram).
int gram_f16_rowscaled(const float* X, int64_t ldx, int64_t MI, const float* Y, int64_t ldy, int64_t MJ, int64_t N,
                       float alpha, int32_t mode, float* out, int64_t ldo, const float* xb, const float* yb,
                       void* workspace, size_t workspace_bytes, mgp_stream_t stream) {
  if (!xb || !yb) return MGP_ERR_UNSUPPORTED;
  return gram_x6_launch(X, ldx, 0, MI, Y, ldy, 0, MJ, nullptr, 0, N, 1, alpha, mode, out, ldo, MI * ldo, workspace,
                        workspace_bytes, stream, xb, yb, nullptr, true);
}

// mgp_gram_f16 (weighted) with X given as its row image (mgp_split_rows_f16 of X
// with bound x_bound) and the f32 Y shared by the batch: X's split is done once,
// and one workgroup serves two batch entries (gram_rows2_kernel).
extern "C" int mgp_gram_f16_rows(const void* ximg, size_t ximg_bytes, int64_t MI, const float* Y, int64_t ldy,
                                 int64_t MJ, const float* W, int64_t sw, int64_t N, int32_t batch, float alpha,
                                 int32_t mode, float* out, int64_t ldo, int64_t so, const float* x_bound,
                                 const float* y_bound, const float* w_bound, void* workspace, size_t workspace_bytes,
                                 mgp_stream_t stream) {
  if (!ximg) return -1;
  if (!Y) return -4;
  if (ldy < N || ldy % 4) return -5;
  if (!W) return -10;
  if (!x_bound) return -18;
  if (!y_bound) return -19;
  if (!w_bound) return -20;
  if (MI < 0 || MJ < 0 || N < 0 || batch < 0) return -3;
  if (mode < 0 || mode > 2 || (mode && MI != MJ)) return -14;
  if (batch > 1 && sw % 4) return -10;
  if (MI > 0 && N > 0 && ximg_bytes < mgp_rows_f16_bytes(MI, N)) return MGP_ERR_WORKSPACE;
  if (N * 4 >= ((int64_t)1 << 31) || (int64_t)kGT * ldy * 4 >= ((int64_t)1 << 32)) return MGP_ERR_UNSUPPORTED;
  const int64_t nns = mgp_rows_f16_ksteps(N);
  if (4 * nns * 2048 >= ((int64_t)1 << 32)) return MGP_ERR_UNSUPPORTED;
  if (!out) return -15;
  if (ldo < MJ) return -16;
  if (batch > 1 && so < ldo * MI) return -17;
  if (MI == 0 || MJ == 0 || batch == 0) return MGP_OK;
  if (batch > 65535) return MGP_ERR_UNSUPPORTED;  // the reduction's grid
  if (!aligned16(ximg) || !aligned16(Y) || !aligned16(W)) return MGP_ERR_ALIGN;
  if (!workspace || workspace_bytes < mgp_gram_x6_workspace_bytes(MI, MJ, N, batch, mode)) return MGP_ERR_WORKSPACE;
  hipStream_t s = (hipStream_t)stream;
  const int tiles = gram_x6_tiles(MI, MJ, mode != 0);
  const int nbj = (int)((MJ + kGT - 1) / kGT);
  const int pairs = (batch + 1) / 2;
  const int nsplit = N > 0 ? gram_x6_splits(N, (int64_t)tiles * pairs, (int64_t)tiles * batch) : 1;
  int64_t nper = (N + nsplit - 1) / nsplit;
  nper = (nper + kXC - 1) / kXC * kXC;
  float* ws = (float*)workspace;
  const int64_t bstride = MI * MJ, zstride = (int64_t)batch * MI * MJ;
  const dim3 grid((unsigned)(tiles * pairs * nsplit)), block(512 + 64 * kRows2PW);
  if (mode != 0)
    hipLaunchKernelGGL((gram_rows2_kernel<true, kRows2PW>), grid, block, 0, s, (const char*)ximg, nns, MI, Y, ldy, MJ,
                       W, sw, N, nper, nbj, tiles, pairs, (int)batch, nsplit, ws, bstride, zstride, x_bound, y_bound,
                       w_bound);
  else
    hipLaunchKernelGGL((gram_rows2_kernel<false, kRows2PW>), grid, block, 0, s, (const char*)ximg, nns, MI, Y, ldy,
                       MJ, W, sw, N, nper, nbj, tiles, pairs, (int)batch, nsplit, ws, bstride, zstride, x_bound,
                       y_bound, w_bound);
  int st = launch_status();
  if (st) return st;
  hipLaunchKernelGGL(gram_x6_reduce_kernel, dim3((unsigned)((MJ + 31) / 32), (unsigned)((MI + 31) / 32), (unsigned)batch),
                     dim3(256), 0, s, ws, bstride, zstride, nsplit, MI, MJ, alpha, (int)mode, out, ldo, so);
  return launch_status();
}
