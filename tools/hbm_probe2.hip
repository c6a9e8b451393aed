// HBM write-ceiling probe, round 2: store width per lane (4 / 8 / 16 B), waves per
// CU (grid size, one-shot vs grid-stride), and K1's split-f16 image pattern
// (2 of every 3 KiB written: planes 0 and 1 of each fragment triple).
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/hbm_probe2 tools/hbm_probe2.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));

// one-shot: every thread stores ITEMS elements of type T, a wave covering
// consecutive 64-element (64 * sizeof(T) byte) rows
template <typename T, int ITEMS>
__global__ __launch_bounds__(256) void fill_oneshot(T* __restrict__ p, size_t n) {
  const size_t wave = ((size_t)blockIdx.x * 256 + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  T v;
  memset(&v, 0, sizeof(T));
  ((unsigned*)&v)[0] = threadIdx.x;
  T* q = p + wave * ITEMS * 64 + lane;
#pragma unroll
  for (int f = 0; f < ITEMS; ++f) {
    const size_t i = wave * ITEMS * 64 + (size_t)f * 64 + lane;
    if (i < n) q[f * 64] = v;
  }
}

// K1 f16 pattern: a wave owns 8 fragment triples (3 KiB each), writes planes 0 and 1
template <int TRIPLES>
__global__ __launch_bounds__(256) void fill_k1f16(u32x4* __restrict__ p, size_t n16) {
  const int lane = threadIdx.x & 63;
  const size_t wave = (size_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  u32x4 v = {threadIdx.x, 1u, 2u, 3u};
  u32x4* q = p + wave * TRIPLES * 192 + lane;
#pragma unroll
  for (int f = 0; f < TRIPLES; ++f) {
    if (wave * TRIPLES * 192 + f * 192 + 128 > n16) return;
    q[f * 192] = v;
    q[f * 192 + 64] = v;
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
  const size_t bytes = 268435456;  // 256 MiB written (c3 split-f16 Kuf payload: 4 B x 1024 x 65536)
  char* p;
  CHK(hipMalloc(&p, (size_t)3 * bytes / 2 + (1 << 20)));
  const int reps = 20;
  auto report = [&](const char* name, size_t b, float us) {
    printf("%-34s %8.1f us  %6.0f GB/s  %.3f of 8 TB/s\n", name, us, b / us * 1e-3, b / us * 1e-3 / 8000.0);
  };
  char nm[96];
#define ONESHOT(T, ITEMS)                                                                        \
  {                                                                                               \
    const size_t n = bytes / sizeof(T);                                                           \
    const size_t waves = (n + ITEMS * 64 - 1) / (ITEMS * 64);                                     \
    const int g = (int)((waves + 3) / 4);                                                         \
    snprintf(nm, sizeof nm, "oneshot %dB x %d per lane (g=%d)", (int)sizeof(T), ITEMS, g);       \
    report(nm, bytes, timeit([&] { fill_oneshot<T, ITEMS><<<g, 256>>>((T*)p, n); }, reps));       \
  }
  ONESHOT(unsigned, 1) ONESHOT(unsigned, 4) ONESHOT(unsigned, 16) ONESHOT(unsigned, 64)
  ONESHOT(u32x2, 1) ONESHOT(u32x2, 4) ONESHOT(u32x2, 16)
  ONESHOT(u32x4, 1) ONESHOT(u32x4, 2) ONESHOT(u32x4, 4) ONESHOT(u32x4, 8) ONESHOT(u32x4, 16)
  {
    const size_t n16 = (size_t)3 * bytes / 2 / 16;   // image span: 3 KiB per 2 KiB written
    const size_t waves = n16 / (8 * 192);
    const int g = (int)((waves + 3) / 4);
    report("k1 f16 pattern (8 triples/wave)", bytes, timeit([&] { fill_k1f16<8><<<g, 256>>>((u32x4*)p, n16); }, reps));
    const size_t w2 = n16 / (2 * 192);
    report("k1 f16 pattern (2 triples/wave)", bytes,
           timeit([&] { fill_k1f16<2><<<(int)((w2 + 3) / 4), 256>>>((u32x4*)p, n16); }, reps));
  }
  CHK(hipFree(p));
  return 0;
}
