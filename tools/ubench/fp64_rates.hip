// Microbenchmark: fp64 MFMA (v_mfma_f64_16x16x4_f64) and VALU fp64 FMA throughput/latency
// on gfx950.  Prints TFLOP/s for full-chip grids and cycles per instruction for one wave.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef double v4d __attribute__((ext_vector_type(4)));

template <int NACC>
__global__ void mfma_loop(const double* in, double* out, int iters, long long* cyc) {
  const int l = threadIdx.x & 63;
  double a = in[l], b = in[64 + l];
  v4d acc[NACC];
  for (int i = 0; i < NACC; ++i) acc[i] = (v4d){0, 0, 0, 0};
  long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < NACC; ++i) acc[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[i], 0, 0, 0);
  }
  long long t1 = __builtin_amdgcn_s_memtime();
  double s = 0;
  for (int i = 0; i < NACC; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (threadIdx.x == 0 && blockIdx.x == 0) *cyc = t1 - t0;
}

template <int NACC>
__global__ void fma_loop(const double* in, double* out, int iters, long long* cyc) {
  const int l = threadIdx.x & 63;
  double a = in[l], b = in[64 + l];
  double acc[NACC];
  for (int i = 0; i < NACC; ++i) acc[i] = in[i];
  long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < NACC; ++i) acc[i] = fma(a, acc[i], b);
  }
  long long t1 = __builtin_amdgcn_s_memtime();
  double s = 0;
  for (int i = 0; i < NACC; ++i) s += acc[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (threadIdx.x == 0 && blockIdx.x == 0) *cyc = t1 - t0;
}

template <typename K>
void run(const char* name, K kern, int blocks, int threads, int iters, double flop_per_iter_wave,
         const double* din, double* dout, long long* dcyc) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipLaunchKernelGGL(kern, dim3(blocks), dim3(threads), 0, 0, din, dout, iters, dcyc);
  hipDeviceSynchronize();
  hipEventRecord(e0);
  hipLaunchKernelGGL(kern, dim3(blocks), dim3(threads), 0, 0, din, dout, iters, dcyc);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  long long cyc;
  hipMemcpy(&cyc, dcyc, 8, hipMemcpyDeviceToHost);
  const double waves = blocks * (threads / 64.0);
  const double tf = waves * iters * flop_per_iter_wave / (ms * 1e-3) / 1e12;
  std::printf("%-34s blocks=%5d thr=%4d  %8.3f ms  %8.2f TFLOP/s  wave0 cycles/iter %.1f\n", name,
              blocks, threads, ms, tf, (double)cyc / iters);
}

int main() {
  double *din, *dout;
  long long* dcyc;
  hipMalloc(&din, 1024 * 8);
  hipMalloc(&dout, 1 << 24);
  hipMalloc(&dcyc, 8);
  double h[1024];
  for (int i = 0; i < 1024; ++i) h[i] = 1.0 + 1e-9 * i;
  hipMemcpy(din, h, sizeof h, hipMemcpyHostToDevice);
  const int it = 4096;
  // one 16x16x4 f64 MFMA = 2048 flop per wave
  run("mfma f64 16x16x4, 1 acc, 1 wave", mfma_loop<1>, 1, 64, it, 2048.0 * 1, din, dout, dcyc);
  run("mfma f64 16x16x4, 4 acc, 1 wave", mfma_loop<4>, 1, 64, it, 2048.0 * 4, din, dout, dcyc);
  run("mfma f64 16x16x4, 8 acc, 1 wave", mfma_loop<8>, 1, 64, it, 2048.0 * 8, din, dout, dcyc);
  run("mfma f64 16x16x4, 8 acc, 1024 CU x4", mfma_loop<8>, 1024, 256, it, 2048.0 * 8, din, dout, dcyc);
  run("mfma f64 16x16x4, 8 acc, 2048x4", mfma_loop<8>, 2048, 256, it, 2048.0 * 8, din, dout, dcyc);
  // VALU fp64 FMA: 64 lanes x 2 flop per instruction
  run("valu fma f64, 1 chain, 1 wave", fma_loop<1>, 1, 64, it, 128.0 * 1, din, dout, dcyc);
  run("valu fma f64, 8 chains, 1 wave", fma_loop<8>, 1, 64, it, 128.0 * 8, din, dout, dcyc);
  run("valu fma f64, 16 chains, 1 wave", fma_loop<16>, 1, 64, it, 128.0 * 16, din, dout, dcyc);
  run("valu fma f64, 16 chains, 1024x4", fma_loop<16>, 1024, 256, it, 128.0 * 16, din, dout, dcyc);
  run("valu fma f64, 16 chains, 2048x4", fma_loop<16>, 2048, 256, it, 128.0 * 16, din, dout, dcyc);
  return 0;
}
