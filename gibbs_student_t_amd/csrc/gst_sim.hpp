// Batched synthetic-pulsar generator: the simulate_data.py:10-39 recipe for D datasets at
// once, one workgroup per dataset, Philox variates keyed by (seed, dataset id).
//
//   err_t   = 10^(-7 + 0.2 xi_t)                 simulate_data.py:15 (or given error bars)
//   red     = F (sqrt(phi(A, gamma)) * xi_red)   simulate_data.py:21 (or a given realisation,
//                                                 e.g. red.txt)
//   z_t     ~ Bernoulli(theta)                   simulate_data.py:24
//   r_t     = red_t + ((1 - z_t) err_t + z_t sigma_out) xi_t          simulate_data.py:26
//             (xi_t ~ N(0,1), or Student-t(dof): the BASELINE config-4 grid)
//   r       = r - U (U^T r)                      the timing-model refit (tempo2's fit, run
//                                                 by libstempo when the tim is re-read)
//   clean   : the no_outlier twin (simulate_data.py:35-37): the outlier TOAs deleted and the
//             timing model refit on the kept TOAs, r2 = r_k - U_k (U_k^T U_k)^-1 U_k^T r_k
//
// The CPU restatement that pins it is oracle/sim_oracle.py (same Philox stream).
#pragma once
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "gst_kernel.hpp"
#include "philox.hpp"

namespace gst {

enum : uint32_t {
  TAG_SIM_RED = 8u << 24,   // red-noise Fourier coefficient k
  TAG_SIM_ERR = 9u << 24,   // error-bar normal of TOA t
  TAG_SIM_Z = 10u << 24,    // outlier uniform of TOA t
  TAG_SIM_XI = 11u << 24,   // white-noise normal of TOA t
  TAG_SIM_T = 12u << 24,    // Student-t gamma of TOA t (gamma_mt attempts in the low bits)
};
constexpr uint32_t SIM_SWEEP = 0xFFFFFFFFu;   // counter word 2 of every generator draw
constexpr int SIM_BLOCK = 256;
constexpr int SIM_MAX_NF = 512, SIM_MAX_TM_CLEAN = 64;

struct SimArgs {
  int n, nf, ntm, D;
  const double* F;        // [n][nf] Fourier basis (unused when red is given)
  const double* lf;       // [nf] log f_k
  const double* ldf;      // [nf] log df_k
  double log_fyr, log_12pi2;
  const double* U;        // [n][ntm] orthonormal timing-model basis
  const double* red;      // [n] fixed red-noise realisation, or null (power-law draw)
  const double* err_in;   // [n] fixed error bars, or null (log-normal draw)
  const double *theta, *sigma_out, *log10_A, *gamma, *dof;   // [D]; dof <= 0: Gaussian
  uint32_t k0, k1;
  long long ds0;
  double *r, *err, *z, *r_clean;   // [D][n]; r_clean may be null
};

// block-wide sum of one value per thread (SIM_BLOCK threads); every thread gets the sum
__device__ __forceinline__ double sim_block_sum(double v, double* red4) {
  v = wave_sum(v);
  const int w = threadIdx.x >> 6;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red4[w] = v;
  __syncthreads();
  return (red4[0] + red4[1]) + (red4[2] + red4[3]);
}

__global__ void __launch_bounds__(SIM_BLOCK) gst_simulate_kernel(SimArgs a) {
  __shared__ double coef[SIM_MAX_NF];
  __shared__ double red4[4];
  __shared__ double G[SIM_MAX_TM_CLEAN * SIM_MAX_TM_CLEAN];
  __shared__ double cv[SIM_MAX_TM_CLEAN];
  const int d = blockIdx.x;
  const int tid = threadIdx.x;
  const int n = a.n;
  Rng rng;
  rng.k0 = a.k0;
  rng.k1 = a.k1;
  rng.chain = (uint32_t)(a.ds0 + d);
  rng.sweep = SIM_SWEEP;
  double* r = a.r + (size_t)d * n;
  double* err = a.err + (size_t)d * n;
  double* zo = a.z + (size_t)d * n;

  // red-noise coefficients sqrt(phi_k) xi_k (log phi_k as the sampler's prior, model.powerlaw)
  if (!a.red) {
    const double lA = a.log10_A[d], g = a.gamma[d];
    const double lc = 2.0 * lA * 2.302585092994045684 - a.log_12pi2 + (g - 3.0) * a.log_fyr;
    for (int k = tid; k < a.nf; k += SIM_BLOCK)
      coef[k] = sqrt(exp(lc - g * a.lf[k] + a.ldf[k])) * normal_from(rng, (uint32_t)k, TAG_SIM_RED);
  }
  __syncthreads();
  const double th = a.theta[d], so = a.sigma_out[d], dof = a.dof[d];
  for (int t = tid; t < n; t += SIM_BLOCK) {
    const double e = a.err_in ? a.err_in[t]
                              : pow(10.0, -7.0 + normal_from(rng, (uint32_t)t, TAG_SIM_ERR) * 0.2);
    double uz, unused;
    rng.uniform2((uint32_t)t, TAG_SIM_Z, uz, unused);
    const double zz = uz < th ? 1.0 : 0.0;
    double xi = normal_from(rng, (uint32_t)t, TAG_SIM_XI);
    if (dof > 0.0) {   // numpy standard_t: sqrt(df / 2) * N / sqrt(Gamma(df / 2))
      const double gg = gamma_mt(0.5 * dof, rng, (uint32_t)t, TAG_SIM_T);
      xi = sqrt(0.5 * dof) * xi / sqrt(gg);
    }
    double rt;
    if (a.red) {
      rt = a.red[t];
    } else {
      rt = 0.0;
      const double* Ft = a.F + (size_t)t * a.nf;
      for (int k = 0; k < a.nf; ++k) rt = fma(Ft[k], coef[k], rt);
    }
    r[t] = rt + ((1.0 - zz) * e + zz * so) * xi;
    err[t] = e;
    zo[t] = zz;
  }
  __syncthreads();
  // refit: r -= U (U^T r), one block reduction per timing-model column
  for (int j = 0; j < a.ntm; ++j) {
    double s = 0.0;
    for (int t = tid; t < n; t += SIM_BLOCK) s = fma(a.U[(size_t)t * a.ntm + j], r[t], s);
    s = sim_block_sum(s, red4);
    if (tid == 0) coef[j % SIM_MAX_NF] = s;   // coef is free again: c_j (ntm <= SIM_MAX_NF)
  }
  __syncthreads();
  for (int t = tid; t < n; t += SIM_BLOCK) {
    double p = 0.0;
    for (int j = 0; j < a.ntm; ++j) p = fma(a.U[(size_t)t * a.ntm + j], coef[j], p);
    r[t] -= p;
  }
  if (!a.r_clean) return;
  __syncthreads();
  // the no_outlier twin: normal equations of the kept TOAs' refit, G beta = U_k^T r_k
  const int m = a.ntm;
  for (int ij = tid; ij < m * m; ij += SIM_BLOCK) {
    const int i = ij / m, j = ij % m;
    double s = 0.0;
    if (j <= i)
      for (int t = 0; t < n; ++t)
        s = zo[t] != 0.0 ? s : fma(a.U[(size_t)t * m + i], a.U[(size_t)t * m + j], s);
    G[ij] = s;
  }
  for (int j = tid; j < m; j += SIM_BLOCK) {
    double s = 0.0;
    for (int t = 0; t < n; ++t) s = zo[t] != 0.0 ? s : fma(a.U[(size_t)t * m + j], r[t], s);
    cv[j] = s;
  }
  __syncthreads();
  if (tid == 0) {   // Cholesky G = L L^T in place (lower), then L L^T beta = c (m <= 64)
    for (int k = 0; k < m; ++k) {
      double dkk = G[k * m + k];
      for (int p = 0; p < k; ++p) dkk -= G[k * m + p] * G[k * m + p];
      dkk = sqrt(dkk);
      G[k * m + k] = dkk;
      for (int i = k + 1; i < m; ++i) {
        double v = G[i * m + k];
        for (int p = 0; p < k; ++p) v -= G[i * m + p] * G[k * m + p];
        G[i * m + k] = v / dkk;
      }
    }
    for (int i = 0; i < m; ++i) {   // forward: L y = c
      double v = cv[i];
      for (int p = 0; p < i; ++p) v -= G[i * m + p] * cv[p];
      cv[i] = v / G[i * m + i];
    }
    for (int i = m - 1; i >= 0; --i) {   // back: L^T beta = y
      double v = cv[i];
      for (int p = i + 1; p < m; ++p) v -= G[p * m + i] * cv[p];
      cv[i] = v / G[i * m + i];
    }
  }
  __syncthreads();
  double* r2 = a.r_clean + (size_t)d * n;
  for (int t = tid; t < n; t += SIM_BLOCK) {
    double p = 0.0;
    for (int j = 0; j < m; ++j) p = fma(a.U[(size_t)t * m + j], cv[j], p);
    r2[t] = zo[t] != 0.0 ? 0.0 : r[t] - p;
  }
}

}  // namespace gst
