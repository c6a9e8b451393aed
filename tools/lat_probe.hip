// Dependent-latency probe for the K3 panel-sweep primitives (one wave,
// s_memtime around 64-long dependent chains).  Build and run on the GPU box:
//   hipcc -O3 --offload-arch=gfx950 -o tools/lat_probe tools/lat_probe.hip && tools/lat_probe
#include <hip/hip_runtime.h>
#include <stdio.h>

__device__ __forceinline__ double rl(double v, int lane) {
  const unsigned long long u = (unsigned long long)__double_as_longlong(v);
  const unsigned lo = __builtin_amdgcn_readlane((unsigned)u, lane);
  const unsigned hi = __builtin_amdgcn_readlane((unsigned)(u >> 32), lane);
  return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}

__global__ void probe(double* out, unsigned long long* t, double x0) {
  const int l = threadIdx.x;
  double x = x0 + l * 1e-3;
  unsigned long long t0, t1;
  // 1. dependent v_fma_f64
  t0 = __builtin_amdgcn_s_memtime();
#pragma unroll
  for (int i = 0; i < 64; ++i) x = fma(x, 0.999, 1e-3);
  asm volatile("" ::"v"(x));
  t1 = __builtin_amdgcn_s_memtime();
  if (l == 0) t[0] = t1 - t0;
  // 2. readlane -> fma (SGPR operand) -> readlane
  double y = x;
  t0 = __builtin_amdgcn_s_memtime();
#pragma unroll
  for (int i = 0; i < 64; ++i) {
    const double p = rl(y, i & 63);
    y = fma(y, p, 1e-3);
  }
  asm volatile("" ::"v"(y));
  t1 = __builtin_amdgcn_s_memtime();
  if (l == 0) t[1] = t1 - t0;
  // 3. dependent v_rcp_f64
  double z = x + 2.0;
  t0 = __builtin_amdgcn_s_memtime();
#pragma unroll
  for (int i = 0; i < 64; ++i) z = __builtin_amdgcn_rcp(z) + 1.0;
  asm volatile("" ::"v"(z));
  t1 = __builtin_amdgcn_s_memtime();
  if (l == 0) t[2] = t1 - t0;
  // 4. dependent v_rsq_f64
  double w = x + 2.0;
  t0 = __builtin_amdgcn_s_memtime();
#pragma unroll
  for (int i = 0; i < 64; ++i) w = __builtin_amdgcn_rsq(w) + 1.0;
  asm volatile("" ::"v"(w));
  t1 = __builtin_amdgcn_s_memtime();
  if (l == 0) t[3] = t1 - t0;
  // 5. independent v_fma_f64 throughput (8 chains)
  double a[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) a[k] = x + k;
  t0 = __builtin_amdgcn_s_memtime();
#pragma unroll
  for (int i = 0; i < 16; ++i)
#pragma unroll
    for (int k = 0; k < 8; ++k) a[k] = fma(a[k], 0.999, 1e-3);
  double s = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k) asm volatile("" ::"v"(a[k]));
  t1 = __builtin_amdgcn_s_memtime();
  if (l == 0) t[4] = t1 - t0;
  // 6. readlane only chain: v_readlane -> v_mov from sgpr -> readlane
  double q = x;
  t0 = __builtin_amdgcn_s_memtime();
#pragma unroll
  for (int i = 0; i < 64; ++i) q = rl(q, (i * 7) & 63) + (double)l;
  asm volatile("" ::"v"(q));
  t1 = __builtin_amdgcn_s_memtime();
  if (l == 0) t[5] = t1 - t0;
  // 7. LDS write -> read round trip chain
  __shared__ double sh[64];
  double u = x;
  t0 = __builtin_amdgcn_s_memtime();
#pragma unroll
  for (int i = 0; i < 32; ++i) {
    sh[l] = u;
    __builtin_amdgcn_s_waitcnt(0xc07f);
    u = sh[(l + 1) & 63] + 1.0;
  }
  asm volatile("" ::"v"(u));
  t1 = __builtin_amdgcn_s_memtime();
  if (l == 0) t[6] = t1 - t0;
  // 8. memrealtime calibration: 200 dependent fma f64 against the 100 MHz clock
  unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
  t0 = __builtin_amdgcn_s_memtime();
  double v = x;
  for (int i = 0; i < 20000; ++i) v = fma(v, 0.999, 1e-3);
  asm volatile("" ::"v"(v));
  t1 = __builtin_amdgcn_s_memtime();
  unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
  if (l == 0) { t[7] = t1 - t0; t[8] = r1 - r0; }
  out[l] = x + y + z + w + s + q + u + v;
}

int main() {
  double* out;
  unsigned long long* t;
  hipMalloc(&out, 64 * sizeof(double));
  hipMalloc(&t, 16 * sizeof(unsigned long long));
  unsigned long long h[16];
  for (int rep = 0; rep < 3; ++rep) {
    hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, out, t, 1.5);
    hipMemcpy(h, t, sizeof(h), hipMemcpyDeviceToHost);
  }
  printf("per-op cycles: fma_f64 dep %.1f | readlane->fma(sgpr)->readlane %.1f | rcp_f64+add dep %.1f | rsq_f64+add dep %.1f | fma_f64 indep (8 chains) %.1f per op | readlane->add %.1f | lds write->read %.1f\n",
         h[0] / 64.0, h[1] / 64.0, h[2] / 64.0, h[3] / 64.0, h[4] / 128.0, h[5] / 64.0, h[6] / 32.0);
  printf("clock: %llu memtime ticks in %llu memrealtime ticks (100 MHz) -> %.3f GHz\n", h[7], h[8],
         h[7] / (h[8] * 10.0));
  return 0;
}
