// Issue / latency probe of the VALU instructions of the K3 panel sweep, timed by
// s_memtime around fixed inline-asm sequences (one wave, nothing else running).
//   hipcc -O3 --offload-arch=gfx950 -o tools/isa_probe tools/isa_probe.hip && tools/isa_probe
#include <hip/hip_runtime.h>
#include <stdio.h>

#define REP8(x) x x x x x x x x
#define REP32(x) REP8(x) REP8(x) REP8(x) REP8(x)

__device__ __forceinline__ unsigned long long tick() {
  unsigned long long t;
  asm volatile("s_memtime %0\n s_waitcnt lgkmcnt(0)" : "=s"(t) : : "memory");
  return t;
}

__global__ void probe(double* out, unsigned long long* t) {
  double x = 1.0 + threadIdx.x * 1e-3, y = 2.0, z = 3.0, w = 0.5;
  unsigned long long t0, t1;
  // 0: 32 independent v_readlane_b32 (distinct destination SGPRs)
  t0 = tick();
  asm volatile(
      "v_readlane_b32 s20, %0, 1\n v_readlane_b32 s21, %0, 2\n v_readlane_b32 s22, %0, 3\n v_readlane_b32 s23, %0, 4\n"
      "v_readlane_b32 s24, %0, 5\n v_readlane_b32 s25, %0, 6\n v_readlane_b32 s26, %0, 7\n v_readlane_b32 s27, %0, 8\n"
      "v_readlane_b32 s28, %0, 9\n v_readlane_b32 s29, %0, 10\n v_readlane_b32 s30, %0, 11\n v_readlane_b32 s31, %0, 12\n"
      "v_readlane_b32 s32, %0, 13\n v_readlane_b32 s33, %0, 14\n v_readlane_b32 s34, %0, 15\n v_readlane_b32 s35, %0, 16\n"
      "v_readlane_b32 s20, %0, 1\n v_readlane_b32 s21, %0, 2\n v_readlane_b32 s22, %0, 3\n v_readlane_b32 s23, %0, 4\n"
      "v_readlane_b32 s24, %0, 5\n v_readlane_b32 s25, %0, 6\n v_readlane_b32 s26, %0, 7\n v_readlane_b32 s27, %0, 8\n"
      "v_readlane_b32 s28, %0, 9\n v_readlane_b32 s29, %0, 10\n v_readlane_b32 s30, %0, 11\n v_readlane_b32 s31, %0, 12\n"
      "v_readlane_b32 s32, %0, 13\n v_readlane_b32 s33, %0, 14\n v_readlane_b32 s34, %0, 15\n v_readlane_b32 s35, %0, 16\n"
      "s_nop 0\n" ::"v"(threadIdx.x)
      : "s20", "s21", "s22", "s23", "s24", "s25", "s26", "s27", "s28", "s29", "s30", "s31", "s32", "s33", "s34",
        "s35");
  t1 = tick();
  if (threadIdx.x == 0) t[0] = t1 - t0;
  // 1: 32 dependent v_fma_f64
  t0 = tick();
  asm volatile(REP32("v_fma_f64 %0, %0, %1, %2\n") : "+v"(x) : "v"(w), "v"(y));
  t1 = tick();
  if (threadIdx.x == 0) t[1] = t1 - t0;
  // 2: 32 independent v_fma_f64 (4 chains)
  double a0 = x, a1 = y, a2 = z, a3 = w;
  t0 = tick();
  asm volatile(REP8("v_fma_f64 %0, %0, %4, %5\n v_fma_f64 %1, %1, %4, %5\n v_fma_f64 %2, %2, %4, %5\n v_fma_f64 %3, %3, %4, %5\n")
               : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3)
               : "v"(w), "v"(y));
  t1 = tick();
  if (threadIdx.x == 0) t[2] = t1 - t0;
  // 3: 32 x (v_readlane_b32 pair -> v_fma_f64 with the SGPR pair) dependent through the VGPR
  t0 = tick();
  unsigned u0 = threadIdx.x, u1 = threadIdx.x + 7;
  asm volatile(REP32("v_readlane_b32 s40, %0, 3\n v_readlane_b32 s41, %1, 3\n v_fma_f64 %2, s[40:41], %2, %2\n")
               : "+v"(u0), "+v"(u1), "+v"(x)
               :
               : "s40", "s41");
  t1 = tick();
  if (threadIdx.x == 0) t[3] = t1 - t0;
  // 4: 32 dependent v_rsq_f64
  double r = x * x + 1.0;
  t0 = tick();
  asm volatile(REP32("v_rsq_f64 %0, %0\n") : "+v"(r));
  t1 = tick();
  if (threadIdx.x == 0) t[4] = t1 - t0;
  // 5: 32 independent v_rsq_f64 (4 chains)
  double q0 = x + 1, q1 = y + 1, q2 = z + 1, q3 = w + 1;
  t0 = tick();
  asm volatile(REP8("v_rsq_f64 %0, %0\n v_rsq_f64 %1, %1\n v_rsq_f64 %2, %2\n v_rsq_f64 %3, %3\n")
               : "+v"(q0), "+v"(q1), "+v"(q2), "+v"(q3));
  t1 = tick();
  if (threadIdx.x == 0) t[5] = t1 - t0;
  // 6: 32 v_fma_f64 reading an SGPR pair written by readlanes long before
  asm volatile("v_readlane_b32 s40, %0, 3\n v_readlane_b32 s41, %1, 3\n s_nop 7\n s_nop 7\n" ::"v"(u0), "v"(u1)
               : "s40", "s41");
  t0 = tick();
  asm volatile(REP8("v_fma_f64 %0, s[40:41], %4, %0\n v_fma_f64 %1, s[40:41], %4, %1\n v_fma_f64 %2, s[40:41], %4, %2\n v_fma_f64 %3, s[40:41], %4, %3\n")
               : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3)
               : "v"(w)
               : "s40", "s41");
  t1 = tick();
  if (threadIdx.x == 0) t[6] = t1 - t0;
  // 7: 32 x (v_readlane pair of a fresh FMA result -> next FMA): the sweep's chain
  t0 = tick();
  asm volatile(REP32("v_add_u32 %0, %0, %1\n v_readlane_b32 s40, %0, 3\n v_add_u32 %0, s40, %0\n")
               : "+v"(u0)
               : "v"(u1)
               : "s40");
  t1 = tick();
  if (threadIdx.x == 0) t[7] = t1 - t0;
  // 8: 32 readlanes, lane 3, alternating destinations s40 / s41 (no consumer)
  t0 = tick();
  asm volatile(REP8("v_readlane_b32 s40, %0, 3\n v_readlane_b32 s41, %1, 3\n v_readlane_b32 s40, %0, 3\n v_readlane_b32 s41, %1, 3\n")
               ::"v"(u0), "v"(u1) : "s40", "s41");
  t1 = tick();
  if (threadIdx.x == 0) t[8] = t1 - t0;
  // 9: 32 readlanes, lane 3, distinct destinations
  t0 = tick();
  asm volatile(REP8("v_readlane_b32 s40, %0, 3\n v_readlane_b32 s41, %1, 3\n v_readlane_b32 s42, %0, 3\n v_readlane_b32 s43, %1, 3\n")
               ::"v"(u0), "v"(u1) : "s40", "s41", "s42", "s43");
  t1 = tick();
  if (threadIdx.x == 0) t[9] = t1 - t0;
  // 10: 32 readlanes, lanes 17 / 45 / 60 / 33
  t0 = tick();
  asm volatile(REP8("v_readlane_b32 s40, %0, 17\n v_readlane_b32 s41, %1, 45\n v_readlane_b32 s42, %0, 60\n v_readlane_b32 s43, %1, 33\n")
               ::"v"(u0), "v"(u1) : "s40", "s41", "s42", "s43");
  t1 = tick();
  if (threadIdx.x == 0) t[10] = t1 - t0;
  // 11: 32 x (readlane pair + independent fma f64 with VGPR operands)
  t0 = tick();
  asm volatile(REP32("v_readlane_b32 s40, %4, 5\n v_readlane_b32 s41, %5, 5\n v_fma_f64 %0, %0, %6, %1\n")
               : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3) : "v"(u0), "v"(u1), "v"(w) : "s40", "s41");
  t1 = tick();
  if (threadIdx.x == 0) t[11] = t1 - t0;
  // 12: 32 ds_read2_b64 uniform address (broadcast) + waits at the end
  __shared__ double sh[256];
  sh[threadIdx.x] = x;
  __syncthreads();
  typedef double d2v __attribute__((ext_vector_type(2)));
  d2v bb;
  unsigned addr = 0;
  t0 = tick();
  asm volatile(REP32("ds_read2_b64 %0, %1 offset1:1\n") "s_waitcnt lgkmcnt(0)\n" : "=v"(bb) : "v"(addr));
  const double b0 = bb[0], b1 = bb[1];
  t1 = tick();
  if (threadIdx.x == 0) t[12] = t1 - t0;
  // 13: 32 v_fma_f64 with an SGPR operand written long before (repeat of 6, 2 chains)
  t0 = tick();
  asm volatile(REP32("v_fma_f64 %0, s[40:41], %2, %0\n v_fma_f64 %1, s[40:41], %2, %1\n")
               : "+v"(a0), "+v"(a1) : "v"(w) : "s40", "s41");
  t1 = tick();
  if (threadIdx.x == 0) t[13] = t1 - t0;
  // 14: 32 v_fma_f64 with a VGPR-held broadcast (v_mov from SGPR beforehand)
  double bv = 0.25;
  t0 = tick();
  asm volatile(REP32("v_fma_f64 %0, %3, %2, %0\n v_fma_f64 %1, %3, %2, %1\n")
               : "+v"(a0), "+v"(a1) : "v"(w), "v"(bv));
  t1 = tick();
  if (threadIdx.x == 0) t[14] = t1 - t0;
  out[threadIdx.x] = b0 + b1 + (double)(u0 + u1) + x + y + z + w + a0 + a1 + a2 + a3 + r + q0 + q1 + q2 + q3;
}

int main() {
  double* out;
  unsigned long long* t;
  (void)hipMalloc(&out, 64 * sizeof(double));
  (void)hipMalloc(&t, 16 * sizeof(unsigned long long));
  unsigned long long h[16];
  for (int rep = 0; rep < 3; ++rep) {
    hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, out, t);
    (void)hipMemcpy(h, t, sizeof(h), hipMemcpyDeviceToHost);
  }
  const char* n[15] = {"v_readlane_b32 independent", "v_fma_f64 dependent", "v_fma_f64 independent",
                      "readlane pair -> fma(sgpr) dependent", "v_rsq_f64 dependent", "v_rsq_f64 independent",
                      "fma(sgpr operand) independent", "add_u32 -> readlane -> add_u32(sgpr) chain",
                      "readlane lane 3, dest s40/s41", "readlane lane 3, 4 dests", "readlane lanes 17/45/60/33",
                      "readlane pair + independent fma (vgpr)", "ds_read2_b64 broadcast (+1 wait)",
                      "2 x fma(sgpr) per step", "2 x fma(vgpr) per step"};
  for (int i = 0; i < 15; ++i) printf("%-44s %5.1f cycles per step (%llu / 32)\n", n[i], h[i] / 32.0, h[i]);
  return 0;
}
