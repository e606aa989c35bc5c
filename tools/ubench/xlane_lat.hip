// Latency of the cross-lane hand-offs a column broadcast can use on gfx950 (one wave, a
// dependent chain of each, cycles per link from s_memtime):
//   lds    : ds_write_b64 by one lane group, ds_read_b64 by every lane (the elimination's
//            publish -> load today)
//   bperm  : ds_bpermute_b32 x 2 (one fp64 value from an arbitrary lane)
//   newbc  : DPP row_newbcast (lane n of each 16-lane row) x 2 halves + a select
//   rdlane : v_readlane_b32 x 2 -> SGPR -> VALU
// Build: hipcc --offload-arch=gfx950 -O3 tools/ubench/xlane_lat.hip -o tools/ubench/xlane_lat
#include <hip/hip_runtime.h>

#include <cstdio>

__device__ __forceinline__ double bperm(double v, int src) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_ds_bpermute(4 * src, (int)(b & 0xffffffffll));
  const int hi = __builtin_amdgcn_ds_bpermute(4 * src, (int)(b >> 32));
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}
template <int N>
__device__ __forceinline__ double newbc(double v) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_mov_dpp((int)(b & 0xffffffffll), 0x150 + N, 0xf, 0xf, false);
  const int hi = __builtin_amdgcn_mov_dpp((int)(b >> 32), 0x150 + N, 0xf, 0xf, false);
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}
__device__ __forceinline__ double rdlane(double v, int l) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readlane((int)(b & 0xffffffffll), l);
  const int hi = __builtin_amdgcn_readlane((int)(b >> 32), l);
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}
__device__ __forceinline__ void lds_order() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

__global__ void lat(const double* in, double* out, long long* cyc, int iters) {
  __shared__ double buf[64];
  const int lane = threadIdx.x;
  double v = in[lane];
  const int q = lane & 7, p = lane >> 3;
  long long t[5];
  t[0] = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < iters; ++i) {   // lds: owners q == 3 publish, all read row p's value
    if (q == 3) buf[p] = v;
    lds_order();
    v = fma(buf[p], 1.0000001, 1e-300);
    lds_order();
  }
  t[1] = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < iters; ++i) v = fma(bperm(v, 8 * p + 3), 1.0000001, 1e-300);
  t[2] = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < iters; ++i) {
    const double a = newbc<3>(v), b = newbc<11>(v);
    v = fma((p & 1) ? b : a, 1.0000001, 1e-300);
  }
  t[3] = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < iters; ++i) v = fma(rdlane(v, 3), 1.0000001, v);
  t[4] = __builtin_amdgcn_s_memtime();
  out[lane] = v;
  if (lane == 0)
    for (int k = 0; k < 4; ++k) cyc[k] = t[k + 1] - t[k];
}

int main() {
  double *din, *dout;
  long long* dc;
  (void)hipMalloc(&din, 64 * 8);
  (void)hipMalloc(&dout, 64 * 8);
  (void)hipMalloc(&dc, 4 * 8);
  double h[64];
  for (int i = 0; i < 64; ++i) h[i] = 1.0 + i;
  (void)hipMemcpy(din, h, sizeof h, hipMemcpyHostToDevice);
  const int iters = 1000;
  hipLaunchKernelGGL(lat, dim3(1), dim3(64), 0, 0, din, dout, dc, iters);
  hipLaunchKernelGGL(lat, dim3(1), dim3(64), 0, 0, din, dout, dc, iters);
  (void)hipDeviceSynchronize();
  long long c[4];
  (void)hipMemcpy(c, dc, sizeof c, hipMemcpyDeviceToHost);
  const char* nm[4] = {"lds write->read + fma", "ds_bpermute x2 + fma", "dpp row_newbcast x2 + sel + fma",
                       "readlane x2 + fma"};
  for (int k = 0; k < 4; ++k) std::printf("%-34s %6.1f cyc/link\n", nm[k], (double)c[k] / iters);
  return 0;
}
