// Does a tile written by one launch stay in its XCD's L2 for the next launch?
// Launch W: workgroup b writes 32 KiB tile b (plain stores).  Launch R (next on
// the stream): workgroup b reads tile perm(b) and stamps the cycles from its start
// until all of its loads returned.  perm = identity (reader on the writer's XCD,
// assuming blockIdx % 8 placement), shift by one (another XCD), or a tile region
// nobody wrote for many launches.  Build and run on the GPU box:
//   hipcc -O3 --offload-arch=gfx950 -o tools/xcd_reuse_probe tools/xcd_reuse_probe.hip && tools/xcd_reuse_probe
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

constexpr int kTiles = 64, kTileBytes = 32768, kThreads = 256;
constexpr int kPer = kTileBytes / 16 / kThreads;  // 16-B loads per thread

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(kThreads) void write_tiles(u32x4* buf, unsigned v) {
  u32x4* t = buf + (size_t)blockIdx.x * (kTileBytes / 16);
#pragma unroll
  for (int i = 0; i < kPer; ++i) t[threadIdx.x + kThreads * i] = u32x4{v, v + 1, v + 2, (unsigned)i};
}

__global__ __launch_bounds__(kThreads) void read_tiles(const u32x4* buf, int shift, int base, long long* cyc,
                                                       unsigned* sink) {
  const long long t0 = __builtin_amdgcn_s_memtime();
  const int tile = base + (blockIdx.x + shift) % kTiles;
  const u32x4* t = buf + (size_t)tile * (kTileBytes / 16);
  u32x4 acc = {0, 0, 0, 0};
  u32x4 r[kPer];
#pragma unroll
  for (int i = 0; i < kPer; ++i) r[i] = t[threadIdx.x + kThreads * i];
#pragma unroll
  for (int i = 0; i < kPer; ++i) acc += r[i];
  __syncthreads();
  const long long t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
  if (acc.x == 0xdeadbeef) sink[0] = acc.y;  // keeps the loads
}

int main() {
  u32x4* buf;
  long long* cyc;
  unsigned* sink;
  // tiles [0, 64): written each round; [64, 8256): the eviction stream; [9000, 9064):
  // never written after the first fill
  constexpr size_t kAll = 9216;
  hipMalloc(&buf, kAll * kTileBytes);
  hipMalloc(&cyc, kTiles * sizeof(long long));
  hipMalloc(&sink, 4);
  hipMemset(buf, 0, kAll * kTileBytes);
  std::vector<long long> h(kTiles);
  const char* names[3] = {"same XCD as the writer", "next XCD (shift 1)", "cold tiles (not written)"};
  for (int mode = 0; mode < 3; ++mode) {
    std::vector<double> med;
    for (int rep = 0; rep < 30; ++rep) {
      // evict: stream 256 MiB through the caches
      write_tiles<<<8192, kThreads>>>(buf + (size_t)(kTiles) * (kTileBytes / 16), rep);
      write_tiles<<<kTiles, kThreads>>>(buf, rep);
      read_tiles<<<kTiles, kThreads>>>(buf, mode == 1 ? 1 : 0, mode == 2 ? 9000 : 0, cyc, sink);
      hipMemcpy(h.data(), cyc, kTiles * sizeof(long long), hipMemcpyDeviceToHost);
      std::sort(h.begin(), h.end());
      if (rep >= 5) med.push_back((double)h[kTiles / 2]);
    }
    std::sort(med.begin(), med.end());
    printf("%-28s median WG load time %.0f cycles (min %.0f, max %.0f over 25 reps)\n", names[mode], med[med.size() / 2],
           med.front(), med.back());
  }
  return 0;
}
