// Accuracy of the hardware fp64 reciprocal / rsqrt estimates and their Newton refinements.
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <vector>
__global__ void k(const double* x, double* out, int n) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  double a = x[i];
  double r0 = __builtin_amdgcn_rcp(a);
  double r1 = fma(r0, fma(-a, r0, 1.0), r0);
  double r2 = fma(r1, fma(-a, r1, 1.0), r1);
  double s0 = __builtin_amdgcn_rsq(a);
  double s1 = s0 * fma(-0.5 * a * s0, s0, 1.5);
  double s2 = s1 * fma(-0.5 * a * s1, s1, 1.5);
  out[6 * i + 0] = r0; out[6 * i + 1] = r1; out[6 * i + 2] = r2;
  out[6 * i + 3] = s0; out[6 * i + 4] = s1; out[6 * i + 5] = s2;
}
int main() {
  const int n = 1 << 20;
  std::vector<double> x(n), o(6 * n);
  unsigned long long s = 88172645463325252ull;
  for (int i = 0; i < n; ++i) {
    s ^= s << 13; s ^= s >> 7; s ^= s << 17;
    double u = (s >> 11) * 0x1.0p-53;
    x[i] = std::exp((u - 0.5) * 180.0);  // 1e-39 .. 1e39
  }
  double *dx, *dout;
  (void)hipMalloc(&dx, n * 8); (void)hipMalloc(&dout, 6 * n * 8);
  (void)hipMemcpy(dx, x.data(), n * 8, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, dim3(n / 256), dim3(256), 0, 0, dx, dout, n);
  (void)hipMemcpy(o.data(), dout, 6 * n * 8, hipMemcpyDeviceToHost);
  double e[6] = {0};
  for (int i = 0; i < n; ++i) {
    long double r = 1.0L / x[i], q = 1.0L / std::sqrt((long double)x[i]);
    for (int j = 0; j < 3; ++j) e[j] = std::fmax(e[j], (double)std::fabs((o[6 * i + j] - r) / r));
    for (int j = 3; j < 6; ++j) e[j] = std::fmax(e[j], (double)std::fabs((o[6 * i + j] - q) / q));
  }
  std::printf("max rel err  rcp: hw %.3e  +1NR %.3e  +2NR %.3e\n", e[0], e[1], e[2]);
  std::printf("max rel err  rsq: hw %.3e  +1NR %.3e  +2NR %.3e\n", e[3], e[4], e[5]);
  return 0;
}
