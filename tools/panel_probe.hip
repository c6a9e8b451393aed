// K3 panel-sweep probe: cycles of one 64 x 16 panel factorisation (wave 0 of a
// 64-thread workgroup) for variants of the sweep, stamped with sched-barrier
// fenced s_memtime.  Build and run on the GPU box:
//   hipcc -O3 --offload-arch=gfx950 -I include -I modulatedgps_amd/csrc -o tools/panel_probe tools/panel_probe.hip \
//     -Lmodulatedgps_amd -lmgp_hip -Wl,-rpath,'$ORIGIN/../modulatedgps_amd'
//   tools/panel_probe
#include <cstring>
#include <type_traits>

#include "../modulatedgps_amd/csrc/chol.hip"

namespace probe {
using namespace mgp;

__device__ __forceinline__ double rcp_f64_chain(double p) {
  const double r = __builtin_amdgcn_rcp(p);
  return fma(r, fma(-p, r, 1.0), r);
}
__device__ __forceinline__ double rsqrt1_f64(double p) {
  const double r = __builtin_amdgcn_rsq(p);
  return r * fma(-0.5 * p * r, r, 1.5);
}

// LDS-broadcast sweep with an rcp pivot chain (measured slower than the kernel's readlane sweep)
__device__ void lds_sweep(double* sF, double* col, double* sb, int r, int& bad) {
  double a[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) a[j] = sF[r * LDT + j];
  double rs[16], pv[16];
  double vcur[16], vnext[16];
  int zb;
  asm volatile("v_mov_b32 %0, 0" : "=v"(zb));
  const double* sbz = sb + zb;
  sb[r] = a[0];
#pragma unroll
  for (int s2 = 2; s2 < 16; ++s2) vcur[s2] = sbz[s2];
#pragma unroll
  for (int c = 0; c < 16; ++c) {
    const double piv = read_lane_f64(a[c], c);
    pv[c] = piv;
    rs[c] = rsqrt1_f64(piv);
    if (c + 1 < 16) {
      const double v1 = read_lane_f64(a[c], c + 1);
      const double t = a[c] * rcp_f64_chain(piv);
      a[c + 1] = fma(-t, v1, a[c + 1]);
      if (c + 2 < 16) {
        sb[((c + 1) & 1) * CB + r] = a[c + 1];
#pragma unroll
        for (int s2 = c + 3; s2 < 16; ++s2) vnext[s2] = sbz[((c + 1) & 1) * CB + s2];
        __builtin_amdgcn_sched_barrier(0);
      }
#pragma unroll
      for (int s2 = c + 2; s2 < 16; ++s2) a[s2] = fma(-t, vcur[s2], a[s2]);
#pragma unroll
      for (int s2 = c + 3; s2 < 16; ++s2) vcur[s2] = vnext[s2];
    }
  }
#pragma unroll
  for (int c = 0; c < 16; ++c) if (!(pv[c] > 0.0) && bad == 0) bad = c + 1;
#pragma unroll
  for (int c = 0; c < 16; ++c) sF[r * LDT + c] = (r >= c) ? a[c] * rs[c] : 0.0;
}

__device__ __forceinline__ unsigned long long stamp() {
  __builtin_amdgcn_sched_barrier(0);
  unsigned long long t;
  asm volatile("s_memtime %0\n s_waitcnt lgkmcnt(0)" : "=s"(t) : : "memory");
  __builtin_amdgcn_sched_barrier(0);
  return t;
}

// chain only: the pivot recurrence without the off-chain trailing updates
__device__ void chain_only(double* sF, double* col, int r, int& bad) {
  double a[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) a[j] = sF[r * LDT + j];
#pragma unroll
  for (int c = 0; c < 15; ++c) {
    const double piv = read_lane_f64(a[c], c);
    const double v1 = read_lane_f64(a[c], c + 1);
    const double t = a[c] * rcp_f64_chain(piv);
    a[c + 1] = fma(-t, v1, a[c + 1]);
  }
#pragma unroll
  for (int c = 0; c < 16; ++c) sF[r * LDT + c] = a[c];
}

// trailing updates only: fixed t, LDS broadcast as in panel_factor
__device__ void updates_only(double* sF, double* sb, int r) {
  double a[16], vcur[16], vnext[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) a[j] = sF[r * LDT + j];
  int zb;
  asm volatile("v_mov_b32 %0, 0" : "=v"(zb));
  const double* sbz = sb + zb;
  sb[r] = a[0];
#pragma unroll
  for (int s2 = 2; s2 < 16; ++s2) vcur[s2] = sbz[s2];
#pragma unroll
  for (int c = 0; c < 15; ++c) {
    const double t = a[c] * 0.01;
    if (c + 2 < 16) {
      sb[((c + 1) & 1) * CB + r] = a[c + 1];
#pragma unroll
      for (int s2 = c + 3; s2 < 16; ++s2) vnext[s2] = sbz[((c + 1) & 1) * CB + s2];
      __builtin_amdgcn_sched_barrier(0);
    }
#pragma unroll
    for (int s2 = c + 2; s2 < 16; ++s2) a[s2] = fma(-t, vcur[s2], a[s2]);
#pragma unroll
    for (int s2 = c + 3; s2 < 16; ++s2) vcur[s2] = vnext[s2];
  }
#pragma unroll
  for (int c = 0; c < 16; ++c) sF[r * LDT + c] = a[c];
}

// previous sweep: all broadcasts by readlane, rsq + two Newton steps on the chain
__device__ void readlane_sweep(double* sF, double* col, int r, int& bad) {
  double a[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) a[j] = sF[r * LDT + j];
  double rs[16];
  double piv = read_lane_f64(a[0], 0);
  rs[0] = rsqrt_f64(piv);
#pragma unroll
  for (int c = 0; c < 16; ++c) {
    double v[16];
#pragma unroll
    for (int s2 = c + 1; s2 < 16; ++s2) v[s2] = read_lane_f64(a[c], s2);
    const double t = a[c] * (rs[c] * rs[c]);
    if (c + 1 < 16) {
      a[c + 1] = fma(-t, v[c + 1], a[c + 1]);
      piv = read_lane_f64(a[c + 1], c + 1);
      rs[c + 1] = rsqrt_f64(piv);
    }
#pragma unroll
    for (int s2 = c + 2; s2 < 16; ++s2) a[s2] = fma(-t, v[s2], a[s2]);
  }
#pragma unroll
  for (int c = 0; c < 16; ++c) sF[r * LDT + c] = (r >= c) ? a[c] * rs[c] : 0.0;
}


// V2: readlane broadcasts, rcp chain, rs (one Newton) per column, bad deferred
__device__ void rl_rcp(double* sF, double* col, int r, int& bad) {
  double a[16], rs[16], pv[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) a[j] = sF[r * LDT + j];
#pragma unroll
  for (int c = 0; c < 16; ++c) {
    const double piv = read_lane_f64(a[c], c);
    pv[c] = piv;
    rs[c] = rsqrt1_f64(piv);
    if (c + 1 < 16) {
      double v[16];
#pragma unroll
      for (int s2 = c + 1; s2 < 16; ++s2) v[s2] = read_lane_f64(a[c], s2);
      const double t = a[c] * rcp_f64_chain(piv);
      a[c + 1] = fma(-t, v[c + 1], a[c + 1]);
#pragma unroll
      for (int s2 = c + 2; s2 < 16; ++s2) a[s2] = fma(-t, v[s2], a[s2]);
    }
  }
#pragma unroll
  for (int c = 0; c < 16; ++c) if (!(pv[c] > 0.0) && bad == 0) bad = c + 1;
#pragma unroll
  for (int c = 0; c < 16; ++c) sF[r * LDT + c] = (r >= c) ? a[c] * rs[c] : 0.0;
}

// V5/V6: pipelined -- column c-1's deferred trailing updates are issued inside
// column c's pivot chain (PIN: sched barriers between the groups)
template <bool PIN>
__device__ void rl_pipe(double* sF, double* col, int r, int& bad) {
  double a[16], rs[16], pv[16], vp[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) a[j] = sF[r * LDT + j];
  double tp = 0.0;
#pragma unroll
  for (int c = 0; c < 16; ++c) {
    const double piv = read_lane_f64(a[c], c);
    const double v1 = (c + 1 < 16) ? read_lane_f64(a[c], c + 1) : 0.0;
    if (PIN) __builtin_amdgcn_sched_barrier(0);
    if (c >= 1) {   // deferred updates of column c - 1 (s >= c + 1; s = c + 1 first: the chain needs it)
#pragma unroll
      for (int s2 = c + 1; s2 < 16; ++s2) a[s2] = fma(-tp, vp[s2], a[s2]);
    }
    if (PIN) __builtin_amdgcn_sched_barrier(0);
    pv[c] = piv;
    if (c + 1 < 16) {
      const double t = a[c] * rcp_f64_chain(piv);
      a[c + 1] = fma(-t, v1, a[c + 1]);
#pragma unroll
      for (int s2 = c + 2; s2 < 16; ++s2) vp[s2] = read_lane_f64(a[c], s2);
      tp = t;
    }
    if (PIN) __builtin_amdgcn_sched_barrier(0);
    rs[c] = rsqrt1_f64(piv);
  }
#pragma unroll
  for (int c = 0; c < 16; ++c) if (!(pv[c] > 0.0) && bad == 0) bad = c + 1;
#pragma unroll
  for (int c = 0; c < 16; ++c) sF[r * LDT + c] = (r >= c) ? a[c] * rs[c] : 0.0;
}


// V7: one rsq (one Newton) per column: L = a rs on the chain, t = L rs
template <bool PIPE>
__device__ void rs1(double* sF, double* col, int r, int& bad) {
  double a[16], pv[16], vp[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) a[j] = sF[r * LDT + j];
  double tp = 0.0;
#pragma unroll
  for (int c = 0; c < 16; ++c) {
    const double piv = read_lane_f64(a[c], c);
    pv[c] = piv;
    const double r0 = __builtin_amdgcn_rsq(piv);
    const double hp = 0.5 * piv;
    double v[16];
    if (!PIPE) {
#pragma unroll
      for (int s2 = c + 1; s2 < 16; ++s2) v[s2] = read_lane_f64(a[c], s2);
    } else {
      if (c + 1 < 16) v[c + 1] = read_lane_f64(a[c], c + 1);
      if (c >= 1) {
#pragma unroll
        for (int s2 = c + 1; s2 < 16; ++s2) a[s2] = fma(-tp, vp[s2], a[s2]);
      }
    }
    const double rs = r0 * fma(-hp * r0, r0, 1.5);
    if (r == 0) col[c] = rs;
    const double L = a[c] * rs;
    a[c] = (r >= c) ? L : 0.0;
    if (c + 1 < 16) {
      const double t = L * rs;
      a[c + 1] = fma(-t, v[c + 1], a[c + 1]);
      if (!PIPE) {
#pragma unroll
        for (int s2 = c + 2; s2 < 16; ++s2) a[s2] = fma(-t, v[s2], a[s2]);
      } else {
#pragma unroll
        for (int s2 = c + 2; s2 < 16; ++s2) vp[s2] = read_lane_f64(a[c] * 0.0 + L / rs, s2);
        tp = t;
      }
    }
  }
#pragma unroll
  for (int c = 0; c < 16; ++c) if (!(pv[c] > 0.0) && bad == 0) bad = c + 1;
#pragma unroll
  for (int c = 0; c < 16; ++c) sF[r * LDT + c] = a[c];
}


// V8-V10: the previous readlane sweep with a cheaper pivot chain.
// MODE 0: v_rsq_f64 + 1 Newton; 1: f32 rsq + 2 Newton (f64); 2: f32 rsq + 1 Newton
template <int MODE>
__device__ __forceinline__ double rsq_mode(double p) {
  double r;
  if (MODE == 0) r = __builtin_amdgcn_rsq(p);
  else r = (double)__builtin_amdgcn_rsqf((float)p);
  const double h = 0.5 * p;
  r = r * fma(-h * r, r, 1.5);
  if (MODE == 1) r = r * fma(-h * r, r, 1.5);
  return r;
}
template <int MODE>
__device__ void rl_mode(double* sF, double* col, int r, int& bad) {
  double a[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) a[j] = sF[r * LDT + j];
  double rs[16];
  double piv = read_lane_f64(a[0], 0);
  rs[0] = rsq_mode<MODE>(piv);
#pragma unroll
  for (int c = 0; c < 16; ++c) {
    double v[16];
#pragma unroll
    for (int s2 = c + 1; s2 < 16; ++s2) v[s2] = read_lane_f64(a[c], s2);
    const double t = a[c] * (rs[c] * rs[c]);
    if (c + 1 < 16) {
      a[c + 1] = fma(-t, v[c + 1], a[c + 1]);
      piv = read_lane_f64(a[c + 1], c + 1);
      rs[c + 1] = rsq_mode<MODE>(piv);
    }
#pragma unroll
    for (int s2 = c + 2; s2 < 16; ++s2) a[s2] = fma(-t, v[s2], a[s2]);
  }
#pragma unroll
  for (int c = 0; c < 16; ++c) sF[r * LDT + c] = (r >= c) ? a[c] * rs[c] : 0.0;
}

// V11: DPP broadcasts.  Every lane keeps, beside its own row a[], a copy d[] of row (lane & 15)
// of the panel's diagonal block; the column values a row needs come from the copy in its own
// 16-lane row by v_mov_b64_dpp row_newbcast (one op per value instead of two readlanes), and
// the copy gets the same update (one more FMA per value).
template <int S>
__device__ __forceinline__ double bcast16(double x) {
  return __builtin_amdgcn_update_dpp(0.0, x, 0x150 + S, 0xF, 0xF, false);
}
template <int C, int S>
__device__ __forceinline__ void dpp_upd(double (&a)[16], double (&d)[16], double t, double td) {
  if constexpr (S < 16) {
    const double v = bcast16<S>(d[C]);
    a[S] = fma(-t, v, a[S]);
    d[S] = fma(-td, v, d[S]);
    dpp_upd<C, S + 1>(a, d, t, td);
  }
}
template <int C>
__device__ __forceinline__ void dpp_col(double (&a)[16], double (&d)[16], double (&rs)[16]) {
  if constexpr (C < 16) {
    const double piv = bcast16<C>(d[C]);
    rs[C] = rsqrt_f64(piv);
    const double rs2 = rs[C] * rs[C];
    const double t = a[C] * rs2, td = d[C] * rs2;
    dpp_upd<C, C + 1>(a, d, t, td);
    dpp_col<C + 1>(a, d, rs);
  }
}
__device__ void dpp_sweep(double* sF, double* col, int r, int& bad) {
  double a[16], d[16], rs[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    a[j] = sF[r * LDT + j];
    d[j] = sF[(r & 15) * LDT + j];
  }
  dpp_col<0>(a, d, rs);
#pragma unroll
  for (int c = 0; c < 16; ++c) sF[r * LDT + c] = (r >= c) ? a[c] * rs[c] : 0.0;
}

// V13: the kernel's numerics (rsq + two Newton steps, t = a rs^2) with the column
// broadcasts through LDS, one column ahead: right after column c's first FMA makes
// a[c + 1] final, every lane stores it and reads rows c + 2 .. 15 back (uniform
// addresses: LDS broadcasts), consumed after column c + 1's pivot chain; the
// pivot check deferred.  VEC: the reads as 16-B pairs.
template <bool VEC>
__device__ void lds_rsq(double* sF, double* col, double* sb, int r, int& bad) {
  double a[16], rs[16], pv[16], vcur[16], vnext[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) a[j] = sF[r * LDT + j];
  int zb;
  asm volatile("v_mov_b32 %0, 0" : "=v"(zb));
  double* sbz = sb + zb;
  sbz[r] = a[0];
#pragma unroll
  for (int s2 = 1; s2 < 16; ++s2) vcur[s2] = sbz[s2];
  pv[0] = read_lane_f64(a[0], 0);
  rs[0] = rsqrt_f64(pv[0]);
#pragma unroll
  for (int c = 0; c < 16; ++c) {
    const double t = a[c] * (rs[c] * rs[c]);
    if (c + 1 < 16) {
      a[c + 1] = fma(-t, vcur[c + 1], a[c + 1]);
      if (c + 2 < 16) {
        double* buf = sbz + ((c + 1) & 1) * CB;
        buf[r] = a[c + 1];
        if (VEC) {
          const int s0 = (c + 2) & ~1;
#pragma unroll
          for (int s2 = s0; s2 < 16; s2 += 2) {
            const double2 v2 = *reinterpret_cast<const double2*>(buf + s2);
            vnext[s2] = v2.x;
            vnext[s2 + 1] = v2.y;
          }
        } else {
#pragma unroll
          for (int s2 = c + 2; s2 < 16; ++s2) vnext[s2] = buf[s2];
        }
      }
      pv[c + 1] = read_lane_f64(a[c + 1], c + 1);
      rs[c + 1] = rsqrt_f64(pv[c + 1]);
#pragma unroll
      for (int s2 = c + 2; s2 < 16; ++s2) a[s2] = fma(-t, vcur[s2], a[s2]);
#pragma unroll
      for (int s2 = c + 2; s2 < 16; ++s2) vcur[s2] = vnext[s2];
    }
  }
#pragma unroll
  for (int c = 0; c < 16; ++c) if (!(pv[c] > 0.0) && bad == 0) bad = c + 1;
#pragma unroll
  for (int c = 0; c < 16; ++c) sF[r * LDT + c] = (r >= c) ? a[c] * rs[c] : 0.0;
  if (r == 0) {
#pragma unroll
    for (int c = 0; c < 16; ++c) col[c] = rs[c];
  }
}

// V15: as V13 with the broadcasts by ds_bpermute (two per value, no LDS storage)
__device__ __forceinline__ double bperm_f64(double v, int lane) {
  const uint64_t u = (uint64_t)__double_as_longlong(v);
  const uint32_t lo = (uint32_t)__builtin_amdgcn_ds_bpermute(4 * lane, (int)(uint32_t)u);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_ds_bpermute(4 * lane, (int)(uint32_t)(u >> 32));
  return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}
__device__ void bperm_rsq(double* sF, double* col, int r, int& bad) {
  double a[16], rs[16], pv[16], vcur[16], vnext[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) a[j] = sF[r * LDT + j];
#pragma unroll
  for (int s2 = 1; s2 < 16; ++s2) vcur[s2] = bperm_f64(a[0], s2);
  pv[0] = read_lane_f64(a[0], 0);
  rs[0] = rsqrt_f64(pv[0]);
#pragma unroll
  for (int c = 0; c < 16; ++c) {
    const double t = a[c] * (rs[c] * rs[c]);
    if (c + 1 < 16) {
      a[c + 1] = fma(-t, vcur[c + 1], a[c + 1]);
#pragma unroll
      for (int s2 = c + 2; s2 < 16; ++s2) vnext[s2] = bperm_f64(a[c + 1], s2);
      pv[c + 1] = read_lane_f64(a[c + 1], c + 1);
      rs[c + 1] = rsqrt_f64(pv[c + 1]);
#pragma unroll
      for (int s2 = c + 2; s2 < 16; ++s2) a[s2] = fma(-t, vcur[s2], a[s2]);
#pragma unroll
      for (int s2 = c + 2; s2 < 16; ++s2) vcur[s2] = vnext[s2];
    }
  }
#pragma unroll
  for (int c = 0; c < 16; ++c) if (!(pv[c] > 0.0) && bad == 0) bad = c + 1;
#pragma unroll
  for (int c = 0; c < 16; ++c) sF[r * LDT + c] = (r >= c) ? a[c] * rs[c] : 0.0;
  if (r == 0) {
#pragma unroll
    for (int c = 0; c < 16; ++c) col[c] = rs[c];
  }
}

// V16: panel_factor<0> with the pivot check after the sweep (pv[] kept)
__device__ void pf_deferred(double* __restrict__ sF, double* __restrict__ col, int r, int& bad) {
  double a[16], rs[16], pv[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) a[j] = sF[r * LDT + j];
  pv[0] = read_lane_f64(a[0], 0);
  rs[0] = rsqrt_f64(pv[0]);
#pragma unroll
  for (int c = 0; c < 16; ++c) {
    double v[16];
#pragma unroll
    for (int s2 = c + 1; s2 < 16; ++s2) v[s2] = read_lane_f64(a[c], s2);
    const double t = a[c] * (rs[c] * rs[c]);
    if (c + 1 < 16) {
      a[c + 1] = fma(-t, v[c + 1], a[c + 1]);
      pv[c + 1] = read_lane_f64(a[c + 1], c + 1);
      rs[c + 1] = rsqrt_f64(pv[c + 1]);
    }
#pragma unroll
    for (int s2 = c + 2; s2 < 16; ++s2) a[s2] = fma(-t, v[s2], a[s2]);
  }
#pragma unroll
  for (int c = 0; c < 16; ++c) if (!(pv[c] > 0.0) && bad == 0) bad = c + 1;
#pragma unroll
  for (int c = 0; c < 16; ++c) sF[r * LDT + c] = (r >= c) ? a[c] * rs[c] : 0.0;
  if (r == 0) {
#pragma unroll
    for (int c = 0; c < 16; ++c) col[c] = rs[c];
  }
}

// V17: the bare readlane sweep plus the col[] writes of rs (no pivot check)
// V18: the same plus a lane-wise pivot check: lane c keeps its own pivot (a cndmask pair
// per column, no VALU -> SALU round trip in the sweep), one compare and ballot after it
template <bool CHECK>
__device__ void rl_col(double* __restrict__ sF, double* __restrict__ col, int r, int& bad) {
  double a[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) a[j] = sF[r * LDT + j];
  double rs[16];
  double piv = read_lane_f64(a[0], 0);
  double mine = a[0];   // lane c: the pivot of column c (lane 0's is a[0] now)
  rs[0] = rsqrt_f64(piv);
#pragma unroll
  for (int c = 0; c < 16; ++c) {
    double v[16];
#pragma unroll
    for (int s2 = c + 1; s2 < 16; ++s2) v[s2] = read_lane_f64(a[c], s2);
    const double t = a[c] * (rs[c] * rs[c]);
    if (c + 1 < 16) {
      a[c + 1] = fma(-t, v[c + 1], a[c + 1]);
      if (CHECK) mine = (r == c + 1) ? a[c + 1] : mine;
      piv = read_lane_f64(a[c + 1], c + 1);
      rs[c + 1] = rsqrt_f64(piv);
    }
#pragma unroll
    for (int s2 = c + 2; s2 < 16; ++s2) a[s2] = fma(-t, v[s2], a[s2]);
  }
#pragma unroll
  for (int c = 0; c < 16; ++c) sF[r * LDT + c] = (r >= c) ? a[c] * rs[c] : 0.0;
  if (r == 0) {
#pragma unroll
    for (int c = 0; c < 16; ++c) col[c] = rs[c];
  }
  if (CHECK) {
    const unsigned long long nonpos = __ballot(r < 16 && !(mine > 0.0));
    if (nonpos && bad == 0) bad = __ffsll(nonpos);   // 1-based column of the first
  }
}

// V19: two-level panel, the kernel's numerics: the left 8 columns swept (updating
// columns <= 7 only), the right half's updates from them applied afterwards as one
// batch with the column values broadcast through LDS (each a[s] gets the same FMAs
// in the same c order as in the one-level sweep: bit-identical), then the right 8
// columns swept.  sb: 64 doubles of LDS.
__device__ void two_level(double* __restrict__ sF, double* __restrict__ col, double* __restrict__ sb, int r,
                          int& bad) {
  double a[16], rs[16], tl[8];
#pragma unroll
  for (int j = 0; j < 16; ++j) a[j] = sF[r * LDT + j];
  auto sweep = [&](auto C0c) {
    constexpr int C0 = decltype(C0c)::value;   // 0: left half, 8: right half
    double piv = read_lane_f64(a[C0], C0);
    rs[C0] = rsqrt_f64(piv);
#pragma unroll
    for (int c = C0; c < C0 + 8; ++c) {
      double v[16];
#pragma unroll
      for (int s2 = c + 1; s2 < C0 + 8; ++s2) v[s2] = read_lane_f64(a[c], s2);
      const double t = a[c] * (rs[c] * rs[c]);
      if (C0 == 0) tl[c] = t;
      if (c + 1 < C0 + 8) {
        a[c + 1] = fma(-t, v[c + 1], a[c + 1]);
        piv = read_lane_f64(a[c + 1], c + 1);
        rs[c + 1] = rsqrt_f64(piv);
      }
#pragma unroll
      for (int s2 = c + 2; s2 < C0 + 8; ++s2) a[s2] = fma(-t, v[s2], a[s2]);
    }
  };
  sweep(std::integral_constant<int, 0>());
  // right half from the left columns: rows 8..15 publish a[s][c] (c < 8), c-major
  if (r >= 8 && r < 16) {
#pragma unroll
    for (int c = 0; c < 8; ++c) sb[c * 8 + (r - 8)] = a[c];
  }
  __builtin_amdgcn_s_waitcnt(0xc07f);   // lgkmcnt(0): the wave's own LDS writes land first
  __builtin_amdgcn_wave_barrier();
  // column 8's first update must precede its pivot: a[8] gets all 8 FMAs first
#pragma unroll
  for (int c = 0; c < 8; ++c) {
    const double2 p0 = *reinterpret_cast<const double2*>(sb + c * 8 + 0);
    const double2 p1 = *reinterpret_cast<const double2*>(sb + c * 8 + 2);
    const double2 p2 = *reinterpret_cast<const double2*>(sb + c * 8 + 4);
    const double2 p3 = *reinterpret_cast<const double2*>(sb + c * 8 + 6);
    const double vv[8] = {p0.x, p0.y, p1.x, p1.y, p2.x, p2.y, p3.x, p3.y};
#pragma unroll
    for (int s = 0; s < 8; ++s) a[8 + s] = fma(-tl[c], vv[s], a[8 + s]);
  }
  sweep(std::integral_constant<int, 8>());
#pragma unroll
  for (int c = 0; c < 16; ++c) sF[r * LDT + c] = (r >= c) ? a[c] * rs[c] : 0.0;
  if (r == 0) {
#pragma unroll
    for (int c = 0; c < 16; ++c) col[c] = rs[c];
  }
}

__global__ void run(const double* src, double* dst, unsigned long long* t, int variant) {
  __shared__ double sF[CB * LDT], col[3 * CB];
  const int r = threadIdx.x;
  for (int j = 0; j < 64; ++j) sF[r * LDT + j] = src[r * 64 + j];
  __syncthreads();
  int bad = 0;
  unsigned long long t0 = stamp();
  if (variant == 0) lds_sweep(sF, col, col + CB, r, bad);
  else if (variant == 1) readlane_sweep(sF, col, r, bad);
  else if (variant == 2) chain_only(sF, col, r, bad);
  else if (variant == 3) updates_only(sF, col + CB, r);
  else if (variant == 4) rl_rcp(sF, col, r, bad);
  else if (variant == 5) rl_pipe<true>(sF, col, r, bad);
  else if (variant == 6) rl_pipe<false>(sF, col, r, bad);
  else if (variant == 7) rs1<false>(sF, col, r, bad);
  else if (variant == 8) rl_mode<0>(sF, col, r, bad);
  else if (variant == 11) dpp_sweep(sF, col, r, bad);
  else if (variant == 12) panel_factor<0>(sF, col, r);
  else if (variant == 9) rl_mode<1>(sF, col, r, bad);
  else if (variant == 13) lds_rsq<false>(sF, col, col + CB, r, bad);
  else if (variant == 14) lds_rsq<true>(sF, col, col + CB, r, bad);
  else if (variant == 15) bperm_rsq(sF, col, r, bad);
  else if (variant == 16) pf_deferred(sF, col, r, bad);
  else if (variant == 17) rl_col<false>(sF, col, r, bad);
  else if (variant == 18) rl_col<true>(sF, col, r, bad);
  else if (variant == 19) two_level(sF, col, col + CB, r, bad);
  else rl_mode<2>(sF, col, r, bad);
  unsigned long long t1 = stamp();
  if (r == 0) t[variant] = t1 - t0;
  __syncthreads();
  for (int j = 0; j < 64; ++j) dst[r * 64 + j] = sF[r * LDT + j] + bad;
}
}  // namespace probe

int main() {
  double h[64 * 64];
  for (int i = 0; i < 64; ++i)
    for (int j = 0; j < 64; ++j) h[i * 64 + j] = (i == j ? 64.0 : 0.0) + 1.0 / (1.0 + i + j);
  double *src, *dst;
  unsigned long long* t;
  (void)hipMalloc(&src, sizeof(h));
  (void)hipMalloc(&dst, sizeof(h));
  (void)hipMalloc(&t, 32 * sizeof(unsigned long long));
  constexpr int NV = 20;
  (void)hipMemcpy(src, h, sizeof(h), hipMemcpyHostToDevice);
  unsigned long long ht[32] = {0};
  const char* names[NV] = {"panel_factor (LDS broadcast, rcp chain)", "readlane sweep (kernel)", "chain only",
                          "trailing updates only", "readlane + rcp chain", "pipelined, pinned", "pipelined", "rsq1 chain", "readlane, rsq f64 + 1 Newton", "readlane, rsq f32 + 2 Newton", "readlane, rsq f32 + 1 Newton", "DPP row_newbcast + row copies", "panel_factor<0> (kernel)",
                          "LDS column broadcast, kernel chain", "LDS column broadcast (16-B pairs)", "ds_bpermute broadcast, kernel chain",
                          "panel_factor, pivot check after the sweep", "readlane sweep + col writes",
                          "col writes + lane-wise pivot check", "two-level (8 + LDS batch + 8)"};
  for (int rep = 0; rep < 3; ++rep)
    for (int v = 0; v < NV; ++v) hipLaunchKernelGGL(probe::run, dim3(1), dim3(64), 0, 0, src, dst, t, v);
  (void)hipMemcpy(ht, t, sizeof(ht), hipMemcpyDeviceToHost);
  // agreement of the variants' L panels
  double ref[64 * 64], out[64 * 64], ref1[64 * 64];
  for (int v = 0; v < NV; ++v) {
    if (v == 2 || v == 3) continue;
    hipLaunchKernelGGL(probe::run, dim3(1), dim3(64), 0, 0, src, dst, t, v);
    (void)hipMemcpy(v == 0 ? ref : out, dst, sizeof(ref), hipMemcpyDeviceToHost);
    if (v == 0) continue;
    if (v == 1) memcpy(ref1, out, sizeof(ref1));
    double e = 0, e1 = 0;
    for (int i = 0; i < 64; ++i)
      for (int j = 0; j < 16; ++j) {
        e = fmax(e, fabs(out[i * 64 + j] - ref[i * 64 + j]));
        e1 = fmax(e1, fabs(out[i * 64 + j] - ref1[i * 64 + j]));
      }
    printf("variant %d max |diff| vs 0: %.3e, vs 1 (the kernel's numerics): %.3e\n", v, e, e1);
  }
  for (int v = 0; v < NV; ++v) printf("%-42s %6llu cycles (%.0f per column)\n", names[v], ht[v], ht[v] / 16.0);
  return 0;
}
