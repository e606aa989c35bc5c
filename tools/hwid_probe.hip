// Where do the waves of a workgroup land?  Each wave of a (G x 64*W) launch records its
// HW_ID register (SIMD, CU, shader engine) while every wave is resident (each spins ~50 us),
// then the host prints, per workgroup size, how many workgroups had two waves on one SIMD.
// Build: hipcc --offload-arch=gfx950 -O2 tools/hwid_probe.hip -o tools/hwid_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

__global__ void probe(unsigned* out) {
  const unsigned id = __builtin_amdgcn_s_getreg((31 << 11) | (0 << 6) | 4);  // HW_REG_HW_ID
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  while (__builtin_amdgcn_s_memtime() - t0 < 5000) __builtin_amdgcn_s_sleep(10);
  if ((threadIdx.x & 63) == 0) out[blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64] = id;
}

int main() {
  for (int W : {2, 4}) {
    for (int G : {256, 512, 1024}) {
      const int nw = G * W;
      unsigned* d = nullptr;
      if (hipMalloc(&d, nw * sizeof(unsigned)) != hipSuccess) return 1;
      hipLaunchKernelGGL(probe, dim3(G), dim3(64 * W), 0, 0, d);
      if (hipDeviceSynchronize() != hipSuccess) return 2;
      std::vector<unsigned> h(nw);
      (void)hipMemcpy(h.data(), d, nw * sizeof(unsigned), hipMemcpyDeviceToHost);
      (void)hipFree(d);
      int same = 0, cnt[4] = {0, 0, 0, 0};
      for (int g = 0; g < G; ++g) {
        bool clash = false;
        for (int a = 0; a < W; ++a) {
          const unsigned sa = (h[g * W + a] >> 4) & 3;
          cnt[sa]++;
          for (int b = a + 1; b < W; ++b) clash |= sa == ((h[g * W + b] >> 4) & 3);
        }
        same += clash;
      }
      std::printf("W=%d G=%d: workgroups with two waves on one SIMD: %d; waves per SIMD id: %d %d %d %d\n",
                  W, G, same, cnt[0], cnt[1], cnt[2], cnt[3]);
      for (int g = 0; g < 3; ++g) {
        std::printf("  wg %d:", g);
        for (int a = 0; a < W; ++a) {
          const unsigned v = h[g * W + a];
          std::printf(" [simd %u cu %u se %u]", (v >> 4) & 3, (v >> 8) & 15, (v >> 13) & 7);
        }
        std::printf("\n");
      }
    }
  }
  return 0;
}
