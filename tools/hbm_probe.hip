// HBM write-ceiling probe for K1 (the Kuf image is a pure 404.8 MB write at c3).
// Times store-only kernels of the same byte count and per-wave store pattern as
// rbf_kuf_x6_kernel: plain / nontemporal 16-B stores, grid-stride vs 24 KiB
// contiguous per wave.  Build: hipcc --offload-arch=gfx950 -O3 -o tools/hbm_probe tools/hbm_probe.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

template <bool NT>
__global__ __launch_bounds__(256) void fill_stride(u32x4* __restrict__ p, size_t n16) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  u32x4 v = {threadIdx.x, 1u, 2u, 3u};
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += stride) {
    if (NT)
      __builtin_nontemporal_store(v, p + i);
    else
      p[i] = v;
  }
}

// K1's pattern: a wave owns CH contiguous 1 KiB fragments (64 lanes x 16 B),
// written fragment after fragment.
template <bool NT, int CH>
__global__ __launch_bounds__(256) void fill_wave_chunks(u32x4* __restrict__ p, size_t n16) {
  const int lane = threadIdx.x & 63;
  const size_t wave = (size_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  u32x4 v = {threadIdx.x, 1u, 2u, 3u};
  u32x4* q = p + wave * CH * 64 + lane;
#pragma unroll
  for (int f = 0; f < CH; ++f) {
    if (wave * CH * 64 + f * 64 + lane >= n16) return;
    if (NT)
      __builtin_nontemporal_store(v, q + f * 64);
    else
      q[f * 64] = v;
  }
}

#define CHK(x)                                                             \
  do {                                                                     \
    hipError_t e = (x);                                                    \
    if (e != hipSuccess) {                                                 \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));               \
      exit(1);                                                             \
    }                                                                      \
  } while (0)

template <typename F>
static float timeit(F f, int reps) {
  hipEvent_t a, b;
  CHK(hipEventCreate(&a));
  CHK(hipEventCreate(&b));
  f();
  CHK(hipDeviceSynchronize());
  CHK(hipEventRecord(a));
  for (int i = 0; i < reps; ++i) f();
  CHK(hipEventRecord(b));
  CHK(hipEventSynchronize(b));
  float ms;
  CHK(hipEventElapsedTime(&ms, a, b));
  return ms * 1000.f / reps;
}

int main() {
  const size_t bytes = 404783104;  // c3 Kuf image: 6 B x 1024 x 65536 + X, Z reads
  const size_t n16 = bytes / 16;
  u32x4* p;
  CHK(hipMalloc(&p, bytes));
  const int reps = 20;
  auto report = [&](const char* name, float us) {
    printf("%-28s %8.1f us  %6.0f GB/s  %.3f of 8 TB/s\n", name, us, bytes / us * 1e-3, bytes / us * 1e-3 / 8000.0);
  };
  for (int g : {1024, 2048, 4096, 8192}) {
    char nm[64];
    snprintf(nm, sizeof nm, "stride plain g=%d", g);
    report(nm, timeit([&] { fill_stride<false><<<g, 256>>>(p, n16); }, reps));
    snprintf(nm, sizeof nm, "stride nt g=%d", g);
    report(nm, timeit([&] { fill_stride<true><<<g, 256>>>(p, n16); }, reps));
  }
  {
    const size_t waves24 = (n16 + 24 * 64 - 1) / (24 * 64);
    const int g24 = (int)((waves24 + 3) / 4);
    report("chunk24 plain", timeit([&] { fill_wave_chunks<false, 24><<<g24, 256>>>(p, n16); }, reps));
    report("chunk24 nt", timeit([&] { fill_wave_chunks<true, 24><<<g24, 256>>>(p, n16); }, reps));
    const size_t waves6 = (n16 + 6 * 64 - 1) / (6 * 64);
    const int g6 = (int)((waves6 + 3) / 4);
    report("chunk6 plain", timeit([&] { fill_wave_chunks<false, 6><<<g6, 256>>>(p, n16); }, reps));
    report("chunk6 nt", timeit([&] { fill_wave_chunks<true, 6><<<g6, 256>>>(p, n16); }, reps));
    const size_t waves96 = (n16 + 96 * 64 - 1) / (96 * 64);
    const int g96 = (int)((waves96 + 3) / 4);
    report("chunk96 plain", timeit([&] { fill_wave_chunks<false, 96><<<g96, 256>>>(p, n16); }, reps));
    report("chunk96 nt", timeit([&] { fill_wave_chunks<true, 96><<<g96, 256>>>(p, n16); }, reps));
  }
  CHK(hipFree(p));
  return 0;
}
