// Does f64 MFMA work on the other waves of K3's look-ahead workgroup slow its VALU
// panel sweep?  One 512-thread workgroup (8 waves; the SIMD of each wave is read from
// HW_ID): wave 0 runs K3's panel_factor<0> (64 x 16 f64 panel, readlane broadcasts)
// `reps` times and stamps its cycles; the waves in `mask` meanwhile run independent
// v_mfma_f64_16x16x4_f64 chains (mode 1) or f64 VALU FMAs (mode 2) until wave 0 is done
// (LDS flag), and report how many they issued.  Build and run on the GPU box:
//   hipcc -O3 --offload-arch=gfx950 -I include -I modulatedgps_amd/csrc -o tools/simd_share_probe tools/simd_share_probe.hip
//   tools/simd_share_probe
#include <cstdio>
#include <vector>

#include "../modulatedgps_amd/csrc/chol.hip"

namespace probe {
using namespace mgp;

__device__ __forceinline__ unsigned long long stamp() {
  __builtin_amdgcn_sched_barrier(0);
  unsigned long long t;
  asm volatile("s_memtime %0\n s_waitcnt lgkmcnt(0)" : "=s"(t) : : "memory");
  __builtin_amdgcn_sched_barrier(0);
  return t;
}

__global__ __launch_bounds__(512) void share_kernel(const double* __restrict__ A, int reps, int mask, int mode,
                                                    unsigned long long* __restrict__ out) {
  __shared__ double sF[CB * LDT], sB[CB * LDT], col[CB];
  __shared__ volatile int done;
  const int w = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6)), lane = threadIdx.x & 63;
  const unsigned simd = (__builtin_amdgcn_s_getreg((1 << 11) | (4 << 6) | 4)) & 3;   // HW_ID.SIMD_ID
  for (int i = threadIdx.x; i < CB * CB; i += 512) {
    sB[(i >> 6) * LDT + (i & 63)] = A[i];
    sF[(i >> 6) * LDT + (i & 63)] = A[i];
  }
  if (threadIdx.x == 0) done = 0;
  __syncthreads();
  unsigned long long t0 = 0, t1 = 0, work = 0;
  if (w == 0) {
    int bad = 0;
    t0 = stamp();
    for (int r = 0; r < reps; ++r) {
#pragma unroll
      for (int c = 0; c < 16; ++c) sF[lane * LDT + c] = sB[lane * LDT + c];
      panel_factor<0>(sF, col, lane, bad);
    }
    t1 = stamp();
    if (lane == 0) done = 1;
    work = bad;
  } else if ((mask >> w) & 1) {
    if (mode == 1) {
      doublex4 acc[4] = {};
      double a = sB[lane], b = sB[LDT + lane];
      while (!done) {
#pragma unroll
        for (int k = 0; k < 16; ++k) acc[k & 3] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[k & 3], 0, 0, 0);
        work += 16;
      }
      out[1024 + threadIdx.x] = (unsigned long long)(acc[0][0] + acc[1][1] + acc[2][2] + acc[3][3] != 1.5);
    } else {
      double x[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) x[k] = sB[lane + k];
      while (!done) {
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int k = 0; k < 8; ++k) x[k] = fma(x[k], 0.999, 1e-3);
        work += 32;
      }
      out[1024 + threadIdx.x] = (unsigned long long)(x[0] + x[7] != 1.5);
    }
  }
  if (lane == 0) {
    out[w * 4 + 0] = t1 - t0;
    out[w * 4 + 1] = work;
    out[w * 4 + 2] = simd;
  }
  for (int i = threadIdx.x; i < CB * 16; i += 512) out[2048 + i] = __double_as_longlong(sF[(i >> 4) * LDT + (i & 15)]);
}
}  // namespace probe

int main() {
  const int n = 64;
  std::vector<double> A(n * n);
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < n; ++j) A[i * n + j] = (i == j ? 64.0 : 0.0) + 1.0 / (1.0 + i + j);
  double* dA;
  unsigned long long* dO;
  if (hipMalloc(&dA, sizeof(double) * n * n) || hipMalloc(&dO, 8 * 4096)) return 1;
  if (hipMemcpy(dA, A.data(), sizeof(double) * n * n, hipMemcpyHostToDevice)) return 1;
  const int reps = 200;
  struct Cfg { const char* name; int mask, mode; };
  const Cfg cfgs[] = {{"alone", 0, 0},
                      {"mfma wave4 (same SIMD as wave 0)", 1 << 4, 1},
                      {"mfma waves 1-3 (other SIMDs)", 0xE, 1},
                      {"mfma waves 5-7", 0xE0, 1},
                      {"mfma waves 1-7", 0xFE, 1},
                      {"valu wave4", 1 << 4, 2},
                      {"valu waves 5-7", 0xE0, 2}};
  std::vector<unsigned long long> o(4096);
  for (int pass = 0; pass < 2; ++pass)
    for (const Cfg& c : cfgs) {
      hipLaunchKernelGGL(probe::share_kernel, dim3(1), dim3(512), 0, 0, dA, reps, c.mask, c.mode, dO);
      if (hipDeviceSynchronize() || hipMemcpy(o.data(), dO, 8 * 4096, hipMemcpyDeviceToHost)) return 2;
      if (pass == 0) continue;
      std::printf("%-36s wave0 %.0f cyc/panel (simd %llu)", c.name, (double)o[0] / reps, o[2]);
      for (int w = 1; w < 8; ++w)
        if ((c.mask >> w) & 1) std::printf("  w%d(simd %llu): %llu ops", w, o[w * 4 + 2], o[w * 4 + 1]);
      std::printf("\n");
    }
  return 0;
}
