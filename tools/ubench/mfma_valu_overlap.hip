// Microbenchmark: do fp64 MFMA (v_mfma_f64_16x16x4_f64) and fp64 VALU FMA from two waves of
// one SIMD execute concurrently on gfx950?  And the latency of the cross-lane moves a
// blocked factorisation would use (ds_swizzle broadcast, ds_bpermute, LDS write -> read).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/ubench/mfma_valu_overlap.hip -o /tmp/ovl
#include <hip/hip_runtime.h>

#include <cstdio>
typedef double v4d __attribute__((ext_vector_type(4)));

// MODE 0: every wave MFMA; 1: every wave VALU; 2: waves 0-3 of the 8-wave block MFMA, 4-7 VALU
// (one of each per SIMD)
template <int MODE>
__global__ void __launch_bounds__(512) mixed(const double* in, double* out, int iters_m, int iters_v,
                                             long long* cyc) {
  const int l = threadIdx.x & 63, w = threadIdx.x >> 6;
  const bool do_m = MODE == 0 || (MODE == 2 && w < 4);
  double s = 0;
  const long long t0 = __builtin_amdgcn_s_memtime();
  if (do_m) {
    double a = in[l], b = in[64 + l];
    v4d acc[8];
    for (int i = 0; i < 8; ++i) acc[i] = (v4d){0, 0, 0, 0};
    for (int it = 0; it < iters_m; ++it) {
#pragma unroll
      for (int i = 0; i < 8; ++i) acc[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[i], 0, 0, 0);
    }
    for (int i = 0; i < 8; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  } else {
    double a = in[l], b = in[64 + l];
    double acc[16];
    for (int i = 0; i < 16; ++i) acc[i] = in[i];
    for (int it = 0; it < iters_v; ++it) {
#pragma unroll
      for (int i = 0; i < 16; ++i) acc[i] = fma(a, acc[i], b);
    }
    for (int i = 0; i < 16; ++i) s += acc[i];
  }
  const long long t1 = __builtin_amdgcn_s_memtime();
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (l == 0) cyc[blockIdx.x * 8 + w] = t1 - t0;
}

__device__ __forceinline__ double swz_bcast(double v, int) {
  // BitMode swizzle: lane' = (lane & 0x18) | 3 within each 32-lane half
  constexpr int OFF = (0x18) | (3 << 5) | (0 << 10);
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_ds_swizzle((int)(b & 0xffffffffll), OFF);
  const int hi = __builtin_amdgcn_ds_swizzle((int)(b >> 32), OFF);
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}
__device__ __forceinline__ double bperm(double v, int src) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_ds_bpermute(4 * src, (int)(b & 0xffffffffll));
  const int hi = __builtin_amdgcn_ds_bpermute(4 * src, (int)(b >> 32));
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}

// dependent chains: KIND 0 swizzle, 1 bpermute, 2 LDS store + load of another lane's word,
// 3 fp64 FMA (reference)
template <int KIND>
__global__ void lat(const double* in, double* out, int iters, int, long long* cyc) {
  __shared__ double buf[64];
  const int l = threadIdx.x & 63;
  double v = in[l];
  const long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
    if (KIND == 0) v = swz_bcast(v, 3) + 1.0;
    if (KIND == 1) v = bperm(v, (l * 8 + 3) & 63) + 1.0;
    if (KIND == 2) {
      buf[l] = v;
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
      __builtin_amdgcn_wave_barrier();
      v = buf[(l * 8 + 3) & 63] + 1.0;
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
      __builtin_amdgcn_wave_barrier();
    }
    if (KIND == 3) v = fma(v, 1.0000001, 1.0);
  }
  const long long t1 = __builtin_amdgcn_s_memtime();
  out[l] = v;
  if (l == 0) *cyc = t1 - t0;
}

template <typename K>
float timed(K kern, int blocks, int threads, const double* din, double* dout, int a, int b,
            long long* dcyc) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipLaunchKernelGGL(kern, dim3(blocks), dim3(threads), 0, 0, din, dout, a, b, dcyc);
  hipDeviceSynchronize();
  hipEventRecord(e0);
  hipLaunchKernelGGL(kern, dim3(blocks), dim3(threads), 0, 0, din, dout, a, b, dcyc);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  return ms;
}

int main() {
  double *din, *dout;
  long long* dcyc;
  hipMalloc(&din, 1024 * 8);
  hipMalloc(&dout, 1 << 26);
  hipMalloc(&dcyc, 1 << 20);
  double h[1024];
  for (int i = 0; i < 1024; ++i) h[i] = 1.0 + 1e-9 * i;
  hipMemcpy(din, h, sizeof h, hipMemcpyHostToDevice);
  const int im = 2048, iv = 2048 * 8 * 16 / 16;   // equal flops per wave: 8 MFMA (16384 flop) vs 16 FMA x 8 (16384)
  const int blocks = 256;                          // one 8-wave block per CU: 2 waves per SIMD
  const float tm = timed(mixed<0>, blocks, 512, din, dout, im, iv, dcyc);
  const float tv = timed(mixed<1>, blocks, 512, din, dout, im, iv, dcyc);
  const float tb = timed(mixed<2>, blocks, 512, din, dout, im, iv, dcyc);
  const double fw_m = 2048.0 * 8 * im, fw_v = 128.0 * 16 * iv;
  std::printf("2 waves/SIMD all MFMA : %8.3f ms %7.2f TF/s\n", tm, blocks * 8 * fw_m / (tm * 1e9));
  std::printf("2 waves/SIMD all VALU : %8.3f ms %7.2f TF/s\n", tv, blocks * 8 * fw_v / (tv * 1e9));
  std::printf("1 MFMA + 1 VALU wave  : %8.3f ms %7.2f TF/s (concurrent if ~half the sum %.3f)\n", tb,
              blocks * 4 * (fw_m + fw_v) / (tb * 1e9), tm + tv);
  const int it = 4096;
  const char* names[4] = {"ds_swizzle bcast (b64)", "ds_bpermute (b64)", "LDS store+load", "fp64 fma"};
  long long c;
  timed(lat<0>, 1, 64, din, dout, it, 0, dcyc);
  hipMemcpy(&c, dcyc, 8, hipMemcpyDeviceToHost);
  std::printf("%-24s %6.1f cycles per dependent step\n", names[0], (double)c / it);
  timed(lat<1>, 1, 64, din, dout, it, 0, dcyc);
  hipMemcpy(&c, dcyc, 8, hipMemcpyDeviceToHost);
  std::printf("%-24s %6.1f cycles per dependent step\n", names[1], (double)c / it);
  timed(lat<2>, 1, 64, din, dout, it, 0, dcyc);
  hipMemcpy(&c, dcyc, 8, hipMemcpyDeviceToHost);
  std::printf("%-24s %6.1f cycles per dependent step\n", names[2], (double)c / it);
  timed(lat<3>, 1, 64, din, dout, it, 0, dcyc);
  hipMemcpy(&c, dcyc, 8, hipMemcpyDeviceToHost);
  std::printf("%-24s %6.1f cycles per dependent step\n", names[3], (double)c / it);
  return 0;
}
