// Issue rate of v_mfma_f64_16x16x4_f64 (K3's matrix instruction): NACC independent
// accumulators per wave, 64 rounds, timed by s_memtime; one wave per SIMD (256
// threads) and two (512 threads) on one CU.
//   hipcc -O3 --offload-arch=gfx950 -o tools/f64_mfma_probe tools/f64_mfma_probe.hip && tools/f64_mfma_probe
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef double doublex4 __attribute__((ext_vector_type(4)));

template <int NACC>
__global__ void probe(double* out, unsigned long long* t) {
  doublex4 acc[NACC];
#pragma unroll
  for (int i = 0; i < NACC; ++i) acc[i] = doublex4{0.0, 0.0, 0.0, 0.0};
  double a = 1.0 + threadIdx.x * 1e-6, b = 0.999;
  __syncthreads();
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
#pragma nounroll
  for (int r = 0; r < 64; ++r) {
#pragma unroll
    for (int i = 0; i < NACC; ++i) acc[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[i], 0, 0, 0);
  }
  double s = 0.0;
#pragma unroll
  for (int i = 0; i < NACC; ++i) s += acc[i][0] + acc[i][3];
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if ((threadIdx.x & 63) == 0) t[threadIdx.x >> 6] = t1 - t0;
}

template <int NACC>
static void run(int threads) {
  double* out;
  unsigned long long* t;
  hipMalloc(&out, threads * sizeof(double));
  hipMalloc(&t, 16 * sizeof(unsigned long long));
  for (int rep = 0; rep < 3; ++rep) hipLaunchKernelGGL(probe<NACC>, dim3(1), dim3(threads), 0, 0, out, t);
  hipDeviceSynchronize();
  unsigned long long h[16];
  hipMemcpy(h, t, sizeof(h), hipMemcpyDeviceToHost);
  unsigned long long mx = 0;
  for (int w = 0; w < threads / 64; ++w) mx = h[w] > mx ? h[w] : mx;
  const double per_simd = (double)(64 * NACC) * (threads / 256);
  printf("{\"nacc\": %d, \"waves_per_simd\": %d, \"cycles\": %llu, \"cycles_per_mfma_per_simd\": %.2f}\n", NACC,
         threads / 256, mx, mx / per_simd);
  hipFree(out);
  hipFree(t);
}

int main() {
  run<1>(256);
  run<2>(256);
  run<4>(256);
  run<8>(256);
  run<4>(512);
  run<8>(512);
  return 0;
}
