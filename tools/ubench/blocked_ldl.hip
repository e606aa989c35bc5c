// Microbenchmark: blocked LDL^T of a 64x64 SPD matrix held by ONE wavefront in fp64 MFMA
// C layout (10 lower 16x16 tiles, lane l / reg g = row (l>>4) + 4g, col l & 15), panels of
// 4 columns factored row-per-lane on the VALU, trailing rank-4 updates as
// v_mfma_f64_16x16x4_f64.  The candidate replacement of the hyper block's 8x8-cyclic
// register elimination (gst_kernel.hpp chol_range: ~16.5k cycles per 61-column
// factorisation at one wave per SIMD, tools/stage_profile.py).
//
// Prints cycles per factorisation (s_memtime, one wave and two waves per SIMD) and the
// pivots' / quadratic form's error against a host LDL^T.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/ubench/blocked_ldl.hip -o /tmp/blocked_ldl
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <random>
#include <vector>

typedef double v4d __attribute__((ext_vector_type(4)));

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
__device__ __forceinline__ double rcp_nr(double a) {
  double y = __builtin_amdgcn_rcp(a);
  double e = fma(-a, y, 1.0);
  y = fma(y, e, y);
  e = fma(-a, y, 1.0);
  return fma(y, e, y);
}
constexpr int TI(int I, int J) { return I * (I + 1) / 2 + J; }

// LA = 0: panel after panel; LA = 1: VALU look-ahead (the next panel is extracted before
// this panel's trailing MFMAs and updated by this panel on the VALU, so its factorisation
// does not wait for the matrix pipe)
template <int WPB, int NP, int AUG, int LA>
__global__ void __launch_bounds__(64 * WPB) ldl_blocked(const double* A, double* piv,
                                                        double* quad, long long* cyc, int reps) {
  __shared__ double P[WPB][4][64];
  __shared__ double Vb[WPB][64][4];
  __shared__ double Lb[WPB][64][4];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int mat = blockIdx.x * WPB + w;
  const double* Am = A + (size_t)(mat % 64) * 4096;
  const int col = lane & 15, rg = lane >> 4;
  long long tot = 0;
  for (int rep = 0; rep < reps; ++rep) {
    v4d acc[10];
#pragma unroll
    for (int I = 0; I < 4; ++I)
#pragma unroll
      for (int J = 0; J <= I; ++J)
#pragma unroll
        for (int g = 0; g < 4; ++g) acc[TI(I, J)][g] = Am[(16 * I + rg + 4 * g) * 64 + 16 * J + col];
    const long long t0 = __builtin_amdgcn_s_memtime();
    double dmine = 1.0, q = 0.0;
    double v[4], nx[4];
    // extract panel p (rows c0.., the 4 columns) into row-per-lane registers
    auto extract = [&](int p, double (&dst)[4]) __attribute__((always_inline)) {
      const int J = p >> 2, cb = 4 * (p & 3);
      const int pc = col - cb;
#pragma unroll
      for (int I = 0; I < 4; ++I) {
        if (I < J) continue;
#pragma unroll
        for (int g = 0; g < 4; ++g)
          if (pc >= 0 && pc < 4) P[w][pc][16 * I + rg + 4 * g] = acc[TI(I, J)][g];
      }
      lds_order();
#pragma unroll
      for (int j = 0; j < 4; ++j) dst[j] = P[w][j][lane];
      lds_order();
    };
    if (LA) extract(0, v);
#pragma unroll
    for (int p = 0; p < NP; ++p) {
      const int J = p >> 2, c0 = 4 * p;
      if (!LA) extract(p, v);
      double l[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int pr = c0 + j;
        const double d = rdlane(v[j], pr);
        const double y = rcp_nr(d);
        const bool below = lane > pr;
        l[j] = below ? v[j] * y : 0.0;
        dmine = lane == pr ? d : dmine;
#pragma unroll
        for (int jj = j + 1; jj < 4; ++jj) {
          const double u = rdlane(v[jj], pr);
          v[jj] = below ? fma(-l[j], u, v[jj]) : v[jj];
        }
        v[j] = below ? v[j] : 0.0;
      }
      if (lane == AUG && c0 < AUG) q = fma(v[3], l[3], fma(v[2], l[2], fma(v[1], l[1], fma(v[0], l[0], q))));
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        Vb[w][lane][j] = v[j];
        Lb[w][lane][j] = l[j];
      }
      lds_order();
      double a[4], b[4];
#pragma unroll
      for (int T = 0; T < 4; ++T) {
        const int r = 16 * T + col;
        const bool ok = T >= J && r >= c0 + 4;
        a[T] = ok ? -Vb[w][r][rg] : 0.0;
        b[T] = ok ? Lb[w][r][rg] : 0.0;
      }
      if (LA && p + 1 < NP) {
        // next panel: its columns as they stand (updated by panels < p), then panel p's
        // rank-4 update applied here on the VALU: nx_j -= sum_k v_k * l_{c1+j, k}
        extract(p + 1, nx);
        const int c1 = c0 + 4;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          double s = nx[j];
#pragma unroll
          for (int k = 0; k < 4; ++k) s = fma(-v[k], rdlane(l[k], c1 + j), s);
          nx[j] = s;
        }
      }
      lds_order();
      // trailing update; with look-ahead the next panel's columns are masked out of it
      // (they were updated on the VALU) -- except that the MFMA still writes them, which
      // is harmless: the next extraction reads nx from registers, and later panels live in
      // other columns
#pragma unroll
      for (int I = 0; I < 4; ++I)
#pragma unroll
        for (int JJ = 0; JJ <= I; ++JJ)
          if (JJ >= J)
            acc[TI(I, JJ)] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[I], b[JJ], acc[TI(I, JJ)], 0, 0, 0);
      if (LA) {
#pragma unroll
        for (int j = 0; j < 4; ++j) v[j] = nx[j];
      }
    }
    const long long t1 = __builtin_amdgcn_s_memtime();
    tot += t1 - t0;
    if (rep == 0) {
      piv[mat * 64 + lane] = dmine;
      if (lane == AUG) quad[mat] = q;
    }
  }
  if (lane == 0) cyc[mat] = tot / reps;
}

template <int LA>
void run(const std::vector<double>& hA, int grid, const char* label) {
  constexpr int WPB = 4, NP = 15, AUG = 60;
  const int nmat = grid * WPB;
  double *dA, *dpiv, *dq;
  long long* dcyc;
  (void)hipMalloc(&dA, hA.size() * 8);
  (void)hipMemcpy(dA, hA.data(), hA.size() * 8, hipMemcpyHostToDevice);
  (void)hipMalloc(&dpiv, nmat * 64 * 8);
  (void)hipMalloc(&dq, nmat * 8);
  (void)hipMalloc(&dcyc, nmat * 8);
  hipLaunchKernelGGL((ldl_blocked<WPB, NP, AUG, LA>), dim3(grid), dim3(64 * WPB), 0, 0, dA, dpiv, dq, dcyc, 20);
  (void)hipDeviceSynchronize();
  std::vector<double> piv(nmat * 64), qq(nmat);
  std::vector<long long> cyc(nmat);
  (void)hipMemcpy(piv.data(), dpiv, piv.size() * 8, hipMemcpyDeviceToHost);
  (void)hipMemcpy(qq.data(), dq, qq.size() * 8, hipMemcpyDeviceToHost);
  (void)hipMemcpy(cyc.data(), dcyc, cyc.size() * 8, hipMemcpyDeviceToHost);
  // host LDL^T of matrix 0..63
  double maxe = 0.0, qe = 0.0;
  for (int mt = 0; mt < 64 && mt < nmat; ++mt) {
    std::vector<double> a(hA.begin() + mt * 4096, hA.begin() + (mt + 1) * 4096);
    double qh = 0.0;
    for (int k = 0; k < NP * 4; ++k) {
      const double d = a[k * 64 + k];
      maxe = std::fmax(maxe, std::fabs(piv[mt * 64 + k] - d) / std::fabs(d));
      qh += a[AUG * 64 + k] * a[AUG * 64 + k] / d;
      for (int i = k + 1; i < 64; ++i)
        for (int j = k + 1; j < 64; ++j) a[i * 64 + j] -= a[i * 64 + k] * a[k * 64 + j] / d;
    }
    qe = std::fmax(qe, std::fabs(qq[mt] - qh) / std::fabs(qh));
  }
  std::vector<long long> s(cyc);
  std::sort(s.begin(), s.end());
  std::printf("%-28s grid %4d (%d waves/SIMD): median %lld cyc/factorisation (min %lld max %lld); "
              "pivot rel err %.2e, quad rel err %.2e\n",
              label, grid, grid * WPB / 1024, s[s.size() / 2], s.front(), s.back(), maxe, qe);
  (void)hipFree(dA);
  (void)hipFree(dpiv);
  (void)hipFree(dq);
  (void)hipFree(dcyc);
}

int main() {
  std::mt19937_64 rng(7);
  std::normal_distribution<double> nd;
  std::vector<double> hA(64 * 4096);
  for (int mt = 0; mt < 64; ++mt) {
    std::vector<double> B(64 * 64);
    for (auto& x : B) x = nd(rng);
    for (int i = 0; i < 64; ++i)
      for (int j = 0; j < 64; ++j) {
        double s = (i == j) ? 4.0 : 0.0;
        for (int k = 0; k < 64; ++k) s += B[i * 64 + k] * B[j * 64 + k] / 64.0;
        hA[mt * 4096 + i * 64 + j] = s;
      }
  }
  for (int grid : {256, 512}) {
    run<0>(hA, grid, "blocked, no look-ahead");
    run<1>(hA, grid, "blocked, VALU look-ahead");
  }
  return 0;
}
