// Accuracy of the K3 pivot chain's reciprocal square root: v_rsq_f64 + one Newton
// step (panel_factor since round 5) and + two (before), against 1 / sqrt(p) in
// float64 on the host, over 2^22 positive values spread across the exponent range.
//   hipcc -O3 --offload-arch=gfx950 -o tools/rsq_probe tools/rsq_probe.hip && tools/rsq_probe
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdint>
#include <cstring>
#include <vector>

__global__ void rsq_kernel(const double* p, double* r1, double* r2, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const double x = p[i];
  double r = __builtin_amdgcn_rsq(x);
  const double h = 0.5 * x;
  r = r * fma(-h * r, r, 1.5);
  r1[i] = r;
  r2[i] = r * fma(-h * r, r, 1.5);
}

static double ulps(double a, double ref) {
  return std::fabs(a - ref) / (std::nextafter(std::fabs(ref), INFINITY) - std::fabs(ref));
}

int main() {
  const int n = 1 << 22;
  std::vector<double> h(n), o1(n), o2(n);
  uint64_t s = 88172645463325252ull;
  for (int i = 0; i < n; ++i) {
    s ^= s << 13, s ^= s >> 7, s ^= s << 17;
    const double m = 1.0 + (double)(s >> 11) * 0x1.0p-53;   // [1, 2)
    const int e = (int)((s >> 3) % 1201) - 600;              // 2^-600 .. 2^600
    h[i] = std::ldexp(m, e);
  }
  double *p, *r1, *r2;
  (void)hipMalloc(&p, n * sizeof(double));
  (void)hipMalloc(&r1, n * sizeof(double));
  (void)hipMalloc(&r2, n * sizeof(double));
  (void)hipMemcpy(p, h.data(), n * sizeof(double), hipMemcpyHostToDevice);
  hipLaunchKernelGGL(rsq_kernel, dim3(n / 256), dim3(256), 0, 0, p, r1, r2, n);
  (void)hipMemcpy(o1.data(), r1, n * sizeof(double), hipMemcpyDeviceToHost);
  (void)hipMemcpy(o2.data(), r2, n * sizeof(double), hipMemcpyDeviceToHost);
  double m1 = 0, m2 = 0, s1 = 0, s2 = 0;
  for (int i = 0; i < n; ++i) {
    const double ref = 1.0 / std::sqrt(h[i]);
    const double u1 = ulps(o1[i], ref), u2 = ulps(o2[i], ref);
    m1 = std::fmax(m1, u1), m2 = std::fmax(m2, u2), s1 += u1, s2 += u2;
  }
  printf("rsq + 1 Newton: max %.2f ulp, mean %.3f ulp\n", m1, s1 / n);
  printf("rsq + 2 Newton: max %.2f ulp, mean %.3f ulp\n", m2, s2 / n);
  return 0;
}
