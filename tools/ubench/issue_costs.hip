// Issue cost of the instructions of the register-resident LDL^T elimination on gfx950, at two
// waves per SIMD (the two-chains-per-SIMD build's occupancy): each wave runs 8 independent
// chains of one instruction kind for ITER iterations; the wave's s_memtime cycles over the
// loop divided by (ITER x 8) is the SIMD cycles per instruction of the pair (both waves issue
// the same stream).  Prints one line per kind.
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/issue_costs tools/ubench/issue_costs.hip
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr int ITER = 4096;

#define REP8(X) X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7)

template <int KIND>
__global__ void __launch_bounds__(256, 2) kern(double* out, unsigned long long* cyc, double s) {
  const int lane = threadIdx.x & 63;
  __shared__ double lds[1024];
  double a0 = lane * 1e-3 + 1.0, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4,
         a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  lds[threadIdx.x] = a0;
  lds[threadIdx.x + 256] = a1;
  __syncthreads();
  const double b = s, c = 1.0 - s;
  unsigned u0 = lane, u1 = lane + 1;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 1
  for (int it = 0; it < ITER; ++it) {
    if constexpr (KIND == 0) {   // v_fmac_f64 (independent)
#define F(i) asm volatile("v_fmac_f64 %0, %1, %2" : "+v"(a##i) : "v"(b), "v"(c));
      REP8(F)
#undef F
    } else if constexpr (KIND == 1) {   // v_mul_f64
#define F(i) asm volatile("v_mul_f64 %0, %0, %1" : "+v"(a##i) : "v"(b));
      REP8(F)
#undef F
    } else if constexpr (KIND == 2) {   // v_rcp_f64
#define F(i) asm volatile("v_rcp_f64 %0, %0" : "+v"(a##i));
      REP8(F)
#undef F
    } else if constexpr (KIND == 3) {   // v_readlane_b32 (into SGPRs), then nothing
      unsigned r;
#define F(i) asm volatile("v_readlane_b32 %0, %1, 5" : "=s"(r) : "v"(u0)); u1 += r;
      REP8(F)
#undef F
    } else if constexpr (KIND == 4) {   // v_cndmask_b32 (VCC)
#define F(i) asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(u0) : "v"(u1));
      REP8(F)
#undef F
    } else if constexpr (KIND == 5) {   // v_mov_b32
#define F(i) asm volatile("v_mov_b32 %0, %1" : "=v"(u0) : "v"(u1));
      REP8(F)
#undef F
    } else if constexpr (KIND == 6) {   // ds_read_b128, 8 distinct addresses per wave
      typedef double v2 __attribute__((ext_vector_type(2)));
      v2 r0, r1, r2, r3;
      const double* p = lds + 2 * ((lane >> 3) & 7);
      r0 = *(volatile v2*)(p);
      r1 = *(volatile v2*)(p + 16);
      r2 = *(volatile v2*)(p + 32);
      r3 = *(volatile v2*)(p + 48);
      r0 = *(volatile v2*)(p + 64);
      r1 = *(volatile v2*)(p + 80);
      r2 = *(volatile v2*)(p + 96);
      r3 = *(volatile v2*)(p + 112);
      a0 += r0[0] + r1[1] + r2[0] + r3[1];
    } else if constexpr (KIND == 7) {   // v_fma_f64 3-operand
#define F(i) asm volatile("v_fma_f64 %0, %1, %2, %0" : "+v"(a##i) : "v"(b), "v"(c));
      REP8(F)
#undef F
    }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if (lane == 0) cyc[blockIdx.x * 4 + (threadIdx.x >> 6)] = t1 - t0;
  out[blockIdx.x * 256 + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7 + u0 + u1;
}

template <int K>
void run(const char* name, int blocks) {
  double* out;
  unsigned long long* cyc;
  hipMalloc(&out, blocks * 256 * 8);
  hipMalloc(&cyc, blocks * 4 * 8);
  hipLaunchKernelGGL(kern<K>, dim3(blocks), dim3(256), 0, 0, out, cyc, 0.999);
  hipDeviceSynchronize();
  hipLaunchKernelGGL(kern<K>, dim3(blocks), dim3(256), 0, 0, out, cyc, 0.999);
  hipDeviceSynchronize();
  unsigned long long* h = new unsigned long long[blocks * 4];
  hipMemcpy(h, cyc, blocks * 4 * 8, hipMemcpyDeviceToHost);
  double s = 0;
  for (int i = 0; i < blocks * 4; ++i) s += h[i];
  s /= blocks * 4;
  printf("%-28s %6.2f cycles per instruction per wave (%d waves per SIMD)\n", name,
         s / (ITER * 8.0), blocks * 4 / 1024);
  delete[] h;
  hipFree(out);
  hipFree(cyc);
}

int main() {
  for (int blocks : {256, 512}) {
    run<0>("v_fmac_f64", blocks);
    run<7>("v_fma_f64", blocks);
    run<1>("v_mul_f64", blocks);
    run<2>("v_rcp_f64", blocks);
    run<3>("v_readlane_b32", blocks);
    run<4>("v_cndmask_b32", blocks);
    run<5>("v_mov_b32", blocks);
    run<6>("ds_read_b128 (8 addr)", blocks);
  }
  return 0;
}
