// Microbenchmark: what caps lg_gram's fp64 MFMA rate on gfx950 -- waves per SIMD and the
// fp64 VALU multiplies that scale the A operand (4 v_mul_f64 per 16 MFMAs in lg_gram).
//   hipcc --offload-arch=gfx950 -O3 -o gram_rates tools/ubench/gram_rates.hip && ./gram_rates
#include <hip/hip_runtime.h>
#include <cstdio>
typedef double v4d __attribute__((ext_vector_type(4)));

// 16 accumulators (lg_gram's 4x4 tiles); NMUL fp64 multiplies per k-step produce the A
// operands (NMUL = 0: A fixed), as lg_gram's aw[u] = ta[u] * wt
template <int NMUL>
__global__ void __launch_bounds__(512) gram_loop(const double* in, double* out, int iters) {
  const int l = threadIdx.x & 63;
  double a[4], b[4];
  for (int u = 0; u < 4; ++u) {
    a[u] = in[l + 64 * u];
    b[u] = in[256 + l + 64 * u];
  }
  double w = in[512 + l];
  v4d acc[16];
  for (int i = 0; i < 16; ++i) acc[i] = (v4d){0, 0, 0, 0};
  for (int it = 0; it < iters; ++it) {
    double aw[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) aw[u] = (u < NMUL) ? a[u] * w : a[u];
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int v = 0; v < 4; ++v)
        acc[4 * u + v] = __builtin_amdgcn_mfma_f64_16x16x4f64(aw[u], b[v], acc[4 * u + v], 0, 0, 0);
    w = w * 0.9999999999;   // a new weight each k-step (keeps the multiplies in the loop)
  }
  double s = 0;
  for (int i = 0; i < 16; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <typename K>
void run(const char* name, K kern, int blocks, int threads, int iters, const double* din,
         double* dout) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipLaunchKernelGGL(kern, dim3(blocks), dim3(threads), 0, 0, din, dout, iters);
  hipDeviceSynchronize();
  hipEventRecord(e0);
  hipLaunchKernelGGL(kern, dim3(blocks), dim3(threads), 0, 0, din, dout, iters);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  const double waves = blocks * (threads / 64.0);
  const double tf = waves * iters * 16 * 2048.0 / (ms * 1e-3) / 1e12;
  std::printf("%-40s blocks=%5d thr=%4d (%.1f waves/SIMD)  %8.3f ms  %7.2f TFLOP/s\n", name,
              blocks, threads, waves / 1024.0, ms, tf);
}

int main() {
  double *din, *dout;
  hipMalloc(&din, 1024 * 8);
  hipMalloc(&dout, 1 << 24);
  double h[1024];
  for (int i = 0; i < 1024; ++i) h[i] = 1.0 + 1e-9 * i;
  hipMemcpy(din, h, sizeof h, hipMemcpyHostToDevice);
  const int it = 2048;
  for (int wps : {1, 2}) {
    // 256 CUs x 4 SIMDs: wps waves per SIMD as 256 x wps blocks of 256 threads
    run("16 acc, no multiply", gram_loop<0>, 256 * wps, 256, it, din, dout);
    run("16 acc, 4 fp64 mul per 16 MFMA", gram_loop<4>, 256 * wps, 256, it, din, dout);
    // lg_gram's shape: 512-thread workgroups (8 waves, 2 per SIMD)
    if (wps == 2) {
      run("16 acc, no multiply, 512 thr", gram_loop<0>, 256, 512, it, din, dout);
      run("16 acc, 4 mul, 512 thr", gram_loop<4>, 256, 512, it, din, dout);
    }
  }
  return 0;
}
