// Large-model path (BASELINE config 5: n ~ 1e5 TOAs, m ~ 420 basis columns) for gfx950.
//
// The register-resident persistent kernel (gst_kernel.hpp) holds a whole chain in one
// wavefront; that stops at m ~ 80 and n ~ 256.  Here one sweep of every chain is a short
// pipeline of launches on one stream, each kernel shaped for its own roofline:
//
//   record   state -> chain records (gibbs.py:355-361)                       HBM copy
//   white    21 white-noise likelihoods + MH (gibbs.py:114-143, 262-284),
//            then N^-1, sum log N, r^T N^-1 r at the final white x            HBM/VALU
//   gram     G_c = [T|r]^T diag(N_c^-1) [T|r] for every chain c               fp64 MFMA
//            (gibbs.py:302-304): T HBM-resident and shared by all chains; one
//            workgroup = 8 chains x one 64x64 super-tile, full TOA range
//   tmelim   timing-model columns eliminated once per sweep (blocked right-    fp64 MFMA
//            looking LDL^T, 16-column panels in LDS, MFMA trailing update)
//            -> Schur complement S0 of the Fourier block + augmented row
//   hyper    10 red-noise MH steps (gibbs.py:80-111, 288-329): S0 + diag(phi^-1)
//            factored in LDS per proposal; b draw's Fourier part (gibbs.py:145-182)
//   btm      b draw's timing-model part (back substitution through G)
//   tb       y = r - T b for all chains as one MFMA GEMM (T streamed once)    fp64 MFMA
//   toa      theta, z, alpha, nu (gibbs.py:185-259)                           HBM/VALU
//
// Variates use the same Philox counters as the persistent kernel (stage tags, step and
// TOA indices), so both paths draw identical numbers for the same (seed, chain, sweep).
// Internal column order as in gst_kernel.hpp, [TM | pad | Fourier | r | pad], with the
// TM block padded to a multiple of 16 (one MFMA tile) and the dimension mp to 16.
#pragma once
#include <hip/hip_runtime.h>

#include "gst_kernel.hpp"

namespace gst {

constexpr int LBLK = 256;      // threads of the per-chain kernels (4 waves)
// threads per chain of the per-TOA passes (lg_white, lg_toa): 16 waves per chain for the
// 100k-TOA datasets; 4 for datasets of up to TBLK_SMALL_NPAD TOAs, where a pass is a few
// TOAs per thread and a 16-wave chain spent it in barriers and reductions with one chain per
// CU.  The block size sets the reduction order, so it is chosen PER DATASET (kernel classes
// below), never from the launch's other datasets or its chain count: a dataset's chains are
// the same launched alone, batched with any others, or split over launches and ranks.
constexpr int TBLK = 1024;
constexpr int TBLK_SMALL = 256;
constexpr int TBLK_SMALL_NPAD = 32768;
// lg_white only: one wave per chain up to 8k TOAs (its 21 likelihood passes are then a few
// loads and one wave reduction each, with no workgroup barrier)
constexpr int TBLK_WAVE = 64;
constexpr int TBLK_WAVE_NPAD = 8192;
// Kernel classes of a dataset (the host launches one kernel per class present in a batch;
// a chain whose dataset is of another class returns at once):
//   lg_white: 0 = one wave (npad <= TBLK_WAVE_NPAD), 1 = TBLK_SMALL, 2 = TBLK threads;
//   lg_toa:   0 = TBLK_SMALL, 1 = TBLK threads;
//   hyper:    8 / 16 = lg_hyper_reg<8 / 16> (hyper block of <= 62 / 126 columns), 0 = lg_hyper
//             (LDS-resident block, <= HYPER_LDS_MAX columns), 1 = lg_hyper<1> (larger blocks:
//             blocked elimination in global memory), 2 = lg_hyper<2> (larger blocks made of
//             ECORR epochs -- hundreds of them -- around a small timing-model + Fourier block:
//             the epochs eliminated first, see lg_hyper).
__host__ __device__ constexpr int white_class(int npad) {
  return npad <= TBLK_WAVE_NPAD ? 0 : (npad <= TBLK_SMALL_NPAD ? 1 : 2);
}
__host__ __device__ constexpr int toa_class(int npad) { return npad <= TBLK_SMALL_NPAD ? 0 : 1; }
// hyper class from the dataset's own hyper block nf + nec: lg_hyper_reg<MT> takes up to
// HR<MT>::RA = 8 MT - 2 columns (62 / 126)
constexpr int HYPER_LDS_MAX = 138;   // lg_hyper's LDS block: (ms (ms + 1) + 3 ms) doubles < 160 KB
// lg_hyper<2>: the timing-model + Fourier + augmented-row block X it factors per likelihood
// (qx = ntm + nfourier + 1 rows) is at most EC_QX_MAX (its lower 16x16 tiles, at most
// EC_TPW per wave, accumulate in MFMA registers); the epochs' couplings stream through LDS
// EC_ECH epochs at a time
constexpr int EC_QX_MAX = 76;
constexpr int EC_TPW = 4;
constexpr int EC_ECH = 32;
static_assert(((EC_QX_MAX + 15) / 16) * ((EC_QX_MAX + 15) / 16 + 1) / 2 <= EC_TPW * (LBLK / 64),
              "lg_hyper<2> tiles per wave");
// (force_lds: GST_DEBUG_LARGE_HYPER, the generic kernels: class 0, or 1 past HYPER_LDS_MAX)
// Class 2 (epochs first) for every block past HYPER_LDS_MAX it can take, and for blocks past
// lg_hyper_reg<8>'s 62 columns whose ECORR epochs outnumber X's rows (measured: mb, 20
// Fourier + 60 epochs, 1.8-2.1x over lg_hyper_reg<16>; ecb, 20 + 24, 0.54-0.85x of
// lg_hyper_reg<8>)
// Class 2 needs disjoint epochs (each TOA in at most one ECORR column: the ECORR block of
// T^T N^-1 T is then diagonal, which its elimination assumes); gst_model_set checks the basis
// (DevModel::ec_disjoint) and other ECORR bases take class 1 / the register kernels.
__host__ __device__ constexpr int hyper_class(int hcols, int force_lds, int nec, int qx,
                                              int disjoint = 1) {
  return (nec > 0 && disjoint && qx <= EC_QX_MAX && !force_lds &&
          (hcols > HYPER_LDS_MAX || (hcols > 8 * 8 - 2 && nec >= qx)))
             ? 2
         : hcols > HYPER_LDS_MAX ? 1
                                 : (force_lds ? 0 : (hcols <= 8 * 8 - 2 ? 8 : (hcols <= 8 * 16 - 2 ? 16 : 0)));
}
__host__ __device__ inline int hyper_class_of(const DevModel& md, int force_lds) {
  return hyper_class(md.nf + md.nec, force_lds, md.nec, md.ntm + md.nf + 1, md.ec_disjoint);
}
// Epochs-first chains (class 2) whose timing model has <= 16 columns and whose Fourier block
// fits the register layout run lg_hyper_ecr<MT, RA> (one wave per chain, MT = 6 / 8: Fourier
// blocks of <= 30 / 46 columns) instead of lg_hyper<2>; 0: lg_hyper<2> (also under
// GST_DEBUG_EPOCHS_LDS or GST_DEBUG_LARGE_HYPER)
// (instance id: 1 = <6, 46>, 2 = <8, 62>: (MT, augmented row); an instance <6, 38> for
// Fourier blocks of <= 22 columns, cutting eight pad steps, spilled 148 B/lane and measured
// no faster on ebig / mb)
// (and at most EC_REG_MAX epochs: their pivots and augmented-row entries live in registers)
constexpr int EC_REG_MAX = 192;
__host__ __device__ constexpr int ec_reg_mt(int hclass, int ntm, int nf, int nec, int debug) {
  return (hclass != 2 || ntm > 16 || nec > EC_REG_MAX || (debug & DEBUG_EPOCHS_LDS)) ? 0
         : (16 + nf <= 46 ? 1 : (16 + nf <= 62 ? 2 : 0));
}
__host__ __device__ inline int ec_reg_mt_of(const DevModel& md, int force_lds, int debug) {
  return ec_reg_mt(hyper_class_of(md, force_lds), md.ntm, md.nf, md.nec, debug);
}
// Chains whose dataset has disjoint ECORR epochs and runs them epochs first (class 2) take the
// structured Gram lg_gram_ec (DevModel::gx_nt > 0), which computes only the blocks class 2 reads:
// G_xx (X = timing model, Fourier, r), the epochs' diagonal and their couplings to X.  The
// dense Grams (lg_gram, lg_gram_small) skip these chains.  GST_DEBUG_LARGE_GRAM: dense.
__host__ __device__ inline bool gram_ec_of(const DevModel& md, int force_lds, int debug) {
  return md.gx_nt > 0 && !(debug & DEBUG_LARGE_GRAM) && hyper_class_of(md, force_lds) == 2;
}
constexpr int GRAM_WAVES = 8;  // chains per gram workgroup
#ifndef GST_TM_PW
#define GST_TM_PW 16   // A/B builds override it (32: config-5 tmelim 1.75 -> 2.95 ms, ebig -20%)
#endif
constexpr int TM_PW = GST_TM_PW;   // panel width of the blocked eliminations (panel_ldl)
#ifndef GST_TM_TILES
#define GST_TM_TILES 4   // (8: measured no faster on config 5, round 6)
#endif
constexpr int TM_TILES = GST_TM_TILES;   // trailing-update tiles per wave per round (panel_ldl)

struct LScratch {
  double* G;   // [C][mp*mp] Gram (row-major, lower triangle); kept for the floor pass
  double* G2;  // [C][mp*mp] lg_tmelim's output: timing-model factor + Schur complement S0
  double* y;   // [C][npad]  r - T b
  double* w;   // [C][npad]  1/N (white scratch: y^2/a during the white block)
  double* sc;  // [C][16]    per-chain scalars (SC_*)
  double* v;   // [C][mp]    b-draw solution (internal order)
  double* G3;  // [C][mp*mp] lg_hyper<1>'s factor of the hyper block (null unless needed)
};
enum : int {
  SC_LOGDETN = 0,
  SC_RNR = 1,
  SC_LDTM = 2,
  SC_QUADTM = 3,
  SC_FAILTM = 4,
  SC_XLAST = 5,
  SC_REDRAW = 6,
  SC_FB = 7,
  SC_TMPMIN = 8,   // smallest / largest pivot of the real timing-model columns
  SC_TMPMAX = 9,
  SC_FLOOR = 10,   // the b draw's SVD noise floor f (floor_shift), 0: the exact draw
};

struct LArgs {
  DevState st;
  DevRec rec;
  DevTape tape;
  LScratch s;
  int ys;  // row stride of the per-TOA scratch y, w: the batch's largest npad
  int C, nsweeps, it, record_every;
  unsigned mask;
  unsigned long long seed;
  long long sweep0, chain0;
  int eval_only;
  double *out_w, *out_h;
  int floor_pass;  // 1: the b draw's floor pass (lg_tmelim + hyper on chains with SC_FLOOR > 0)
  int kclass;      // the launched kernel's class (white_class / toa_class / hyper_class)
  int hyper_lds;   // GST_DEBUG_LARGE_HYPER: every dataset takes lg_hyper (class 0)
};

// Dataset of chain c (dataset batches: one DevModel per dataset).  Chains of one 16-chain
// group must share their dataset (the Gram workgroups and the T b GEMM stage one dataset's
// T for the whole group; NativeSampler.alloc checks this).  An index out of range reads
// dataset 0 and is flagged by lg_white (status bit 4).
constexpr int LGROUP = 16;
__device__ __forceinline__ int ds_of(const LArgs& a, int c) {
  const int d = a.st.dataset ? __builtin_amdgcn_readfirstlane(a.st.dataset[c]) : 0;
  return (unsigned)d < (unsigned)a.st.nd ? d : 0;
}

__device__ __forceinline__ Rng make_rng(const LArgs& a, int c) {
  Rng r;
  r.k0 = (uint32_t)(a.seed & 0xffffffffull);
  r.k1 = (uint32_t)(a.seed >> 32);
  r.chain = (uint32_t)(a.chain0 + c);
  r.sweep = (uint32_t)(a.sweep0 + a.it);
  return r;
}

__device__ __forceinline__ const double* tape_row(const LArgs& a, int c) {
  return a.tape.data ? a.tape.data + ((size_t)c * a.nsweeps + a.it) * a.tape.stride : nullptr;
}

// Deterministic block sum (NW waves): every thread gets the bitwise-identical value.
template <int NW = 4>
__device__ __forceinline__ double block_sum(double v, double* red) {
  if constexpr (NW == 1) {   // one wave: no barrier
    (void)red;
    return wave_sum(v);
  }
  v = wave_sum(v);
  const int wv = threadIdx.x >> 6;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[wv] = v;
  __syncthreads();
  double s = 0.0;
#pragma unroll
  for (int h = 0; h < NW; h += 4) s += (red[h] + red[h + 1]) + (red[h + 2] + red[h + 3]);
  return s;
}

// Three deterministic block sums (NW = 4 waves) behind one pair of barriers; red3: [3][4]
__device__ __forceinline__ void block_sum3(double& a, double& b, double& c, double* red3) {
  a = wave_sum(a);
  b = wave_sum(b);
  c = wave_sum(c);
  const int wv = threadIdx.x >> 6;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) {
    red3[wv] = a;
    red3[4 + wv] = b;
    red3[8 + wv] = c;
  }
  __syncthreads();
  a = (red3[0] + red3[1]) + (red3[2] + red3[3]);
  b = (red3[4] + red3[5]) + (red3[6] + red3[7]);
  c = (red3[8] + red3[9]) + (red3[10] + red3[11]);
}

// K deterministic block sums behind one pair of barriers, each bitwise block_sum<NW>'s;
// red: [K][NW]
template <int NW, int K>
__device__ __forceinline__ void block_sum_k(double (&v)[K], double* red) {
#pragma unroll
  for (int j = 0; j < K; ++j) v[j] = wave_sum(v[j]);
  if constexpr (NW == 1) {
    (void)red;
    return;
  }
  const int wv = threadIdx.x >> 6;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) {
#pragma unroll
    for (int j = 0; j < K; ++j) red[j * NW + wv] = v[j];
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < K; ++j) {
    const double* r = red + j * NW;
    double sum = 0.0;
#pragma unroll
    for (int h = 0; h < NW; h += 4) sum += (r[h] + r[h + 1]) + (r[h + 2] + r[h + 3]);
    v[j] = sum;
  }
}

// MH variates of global step gs (0..19 white, 20..29 hyper) exactly as the persistent
// kernel draws them (gst_kernel.hpp mh_variates): parameter, jump, log(u_acc), 10^(2 jump).
__device__ __forceinline__ void mh_variate(const DevModel& md, const Rng& rng, const double* tp,
                                           int gs, double* out4) {
  const bool white = gs < NWHITE;
  const int step = white ? gs : gs - NWHITE;
  double us, par, xi, la;
  if (tp) {
    const double* e = tp + (white ? TP_WHITE : TP_HYPER) + 4 * step;
    us = e[0];
    par = e[1];
    xi = e[2];
    la = log(e[3]);
  } else {
    const uint32_t tag = white ? TAG_WHITE : TAG_HYPER;
    double ua, ub, uidx, unused;
    rng.uniform2(0u, tag | (uint32_t)(3 * step), ua, ub);
    us = ua;
    la = log(ub);
    xi = normal_from(rng, 0u, tag | (uint32_t)(3 * step + 1));
    const int nind = white ? md.nw : md.nh;
    rng.uniform2(0u, tag | (uint32_t)(3 * step + 2), uidx, unused);
    int k = (int)(uidx * nind);
    k = k < nind - 1 ? k : nind - 1;
    const int* ind = white ? md.wind : md.hind;
    int pk = ind[0];
#pragma unroll
    for (int j = 1; j < PMAX; ++j) pk = (k == j) ? ind[j] : pk;
    par = (double)pk;
  }
  int cnt = 0;
#pragma unroll
  for (int i = 0; i < 5; ++i) cnt += (md.mh_cdf[i] <= us) ? 1 : 0;
  cnt = cnt < 4 ? cnt : 4;
  const double scale = md.mh_size[0] * (cnt == 0) + md.mh_size[1] * (cnt == 1) +
                       md.mh_size[2] * (cnt == 2) + md.mh_size[3] * (cnt == 3) +
                       md.mh_size[4] * (cnt == 4);
  const double delta = mh_step(xi, white ? md.sig_w : md.sig_h, scale);
  out4[0] = par;
  out4[1] = delta;
  out4[2] = la;
  out4[3] = exp(2.0 * delta * 2.302585092994045684);
}

typedef double XVec[PMAX];   // a chain's parameter vector (x, or an MH proposal)

__device__ __forceinline__ double lnpriorP(const DevModel& md, const XVec& xq) {
  bool in = true;
#pragma unroll
  for (int j = 0; j < PMAX; ++j)
    if (j < md.P) in = in && (xq[j] >= md.pmin[j]) && (xq[j] <= md.pmax[j]);
  return in ? md.lp_sum : -INFINITY;
}

// x[i] for a wave-uniform or per-thread runtime index (a select chain: no scratch array)
// (the empty asm keeps r in a register between the selects: without it the compiler turns the
// chain back into an indexed load, which puts the whole of x in scratch memory)
__device__ __forceinline__ double xget(const XVec& x, int i) {
  double r = x[0];
#pragma unroll
  for (int j = 1; j < PMAX; ++j) {
    r = (i == j) ? x[j] : r;
    asm volatile("" : "+v"(r));
  }
  return r;
}

__device__ __forceinline__ void load_x(const DevModel& md, const DevState& st, int c,
                                       XVec& x) {
#pragma unroll
  for (int j = 0; j < PMAX; ++j) x[j] = j < md.P ? st.x[(size_t)c * md.P + j] : 0.0;
}

// White-noise variances N0_t = efac_b^2 sigma_t^2 + 10^(2 equad_b) of backend b = bk[t]
// (enterprise MeasurementNoise + EquadNoise, per selection; gibbs.py:154,268,297).  With one
// backend this is exactly the classic model's expression.
// The dataset's sigma^2 / backend pointers and nb are copied in (registers): read through
// md inside a per-TOA loop they were re-loaded every iteration (no machine LICM in this
// build), each behind a full memory wait.
struct WhiteNoise {
  double ef2[NBMAX], Q[NBMAX];
  const double* s2;   // md.sig2
  const int* bk;      // md.bk (nb > 1)
  int nb;
  __device__ __forceinline__ double n0(int t) const {
    if (nb <= 1) return ef2[0] * s2[t] + Q[0];
    return n0v(bk[t], s2[t]);
  }
  // N0 of a TOA of backend b (0 with one backend) and sigma^2 sv
  __device__ __forceinline__ double n0v(int b, double sv) const {
    if (nb <= 1) return ef2[0] * sv + Q[0];
    double e = ef2[0], q = Q[0];
#pragma unroll
    for (int j = 1; j < NBMAX; ++j) {
      e = (b == j) ? ef2[j] : e;
      q = (b == j) ? Q[j] : q;
    }
    return e * sv + q;
  }
};

__device__ __forceinline__ WhiteNoise white_noise(const DevModel& md, const XVec& x) {
  WhiteNoise w;
  w.s2 = md.sig2;
  w.bk = md.bk;
  w.nb = md.nb;
#pragma unroll
  for (int b = 0; b < NBMAX; ++b) {
    if (b < md.nb) {
      // (value selects, not a pointer select between x and md: that made the compiler load
      // through a flat pointer into the private x array)
      const int ei = md.efac_b[b];
      const double xe = xget(x, ei >= 0 ? ei : 0);
      const double ef = ei >= 0 ? xe : md.efac_const;
      w.ef2[b] = ef * ef;
      w.Q[b] = exp(2.0 * xget(x, md.equad_b[b]) * 2.302585092994045684);
    } else {
      w.ef2[b] = 0.0;
      w.Q[b] = 0.0;
    }
  }
  return w;
}

// ------------------------------------------------------------------------------------
// record: the state at the start of the sweep (gibbs.py:355-361)
// ------------------------------------------------------------------------------------
__global__ void __launch_bounds__(LBLK) lg_record(const DevModel* __restrict__ mds, LArgs a) {
  const int c = blockIdx.x;
  const DevModel& md = mds[ds_of(a, c)];
  const int ri = a.it / a.record_every;
  if (ri >= a.rec.nrec) return;
  const size_t base = (size_t)c * a.rec.nrec + ri;
  const int n = md.n, m = md.m, nst = a.st.nst;
  for (int j = threadIdx.x; j < md.P; j += LBLK)
    if (a.rec.x) a.rec.x[base * md.P + j] = a.st.x[(size_t)c * md.P + j];
  for (int j = threadIdx.x; j < m; j += LBLK)
    if (a.rec.b) a.rec.b[base * m + j] = a.st.b[(size_t)c * m + j];
  for (int t = threadIdx.x; t < n; t += LBLK) {
    if (a.rec.z) a.rec.z[base * nst + t] = a.st.z[(size_t)c * nst + t];
    if (a.rec.alpha) a.rec.alpha[base * nst + t] = a.st.alpha[(size_t)c * nst + t];
    if (a.rec.pout) a.rec.pout[base * nst + t] = a.st.pout[(size_t)c * nst + t];
  }
  if (threadIdx.x == 0) {
    if (a.rec.theta) a.rec.theta[base] = a.st.theta[c];
    if (a.rec.nu) a.rec.nu[base] = a.st.nu[c];
  }
}

// ------------------------------------------------------------------------------------
// white: MH over the white-noise parameters, then N^-1 for the Gram
// ------------------------------------------------------------------------------------
template <int TB>
__global__ void __launch_bounds__(TB) lg_white(const DevModel* __restrict__ mds, LArgs a) {
  const int c = blockIdx.x;
  const DevModel& md = mds[ds_of(a, c)];
  if (threadIdx.x == 0 && a.st.dataset && a.st.status &&
      (unsigned)a.st.dataset[c] >= (unsigned)a.st.nd)
    a.st.status[c] |= 4;                          // bad dataset index (ran on dataset 0)
  if (white_class(md.npad) != a.kclass) return;   // another class's launch runs this chain
  __shared__ double red[TB / 64];
  __shared__ double redk[7 * (TB / 64)];   // lnlk: [2 K + 1][waves]
  __shared__ double wtab[3][2][NBMAX];     // the pass's candidates: efac_b^2, Q_b
  __shared__ double mhv[NWHITE][4];
  constexpr int WU = TB == 64 ? 8 : 4;   // TOAs per thread per round of the per-TOA loops
  const int n = md.n, nst = a.st.nst, npad = md.npad;
  const double* zc = a.st.z + (size_t)c * nst;
  const double* alc = a.st.alpha + (size_t)c * nst;
  const double* yc = a.s.y + (size_t)c * a.ys;
  double* wc = a.s.w + (size_t)c * a.ys;
  double* sc = a.s.sc + (size_t)c * 16;
  XVec xv;
  load_x(md, a.st, c, xv);
  if (threadIdx.x == 0) sc[SC_XLAST] = xget(xv, md.P - 1);   // chain[ii, -1] (gibbs.py:373)
  const Rng rng = make_rng(a, c);
  const double* tp = tape_row(a, c);
  const bool do_white = (a.mask & 1u) || a.eval_only;

  if (do_white) {
    if (!a.eval_only && threadIdx.x < NWHITE) mh_variate(md, rng, tp, threadIdx.x, mhv[threadIdx.x]);
    __syncthreads();
    // a proposal's variances come from its parameters, except that Q of a one-backend model
    // moves by 10^(2 delta) with its equad (the MH variate's 4th entry), as the persistent
    // kernel carries it.
    // K likelihoods per pass over the TOAs (the pass streams the chain's y^2 / a row from
    // HBM, 800 KB at 100k TOAs; K = 3 costs VALU work, not bytes).  The block's first pass
    // (FIRST) reads z, alpha and y instead and leaves y_t^2 / a_t (a_t = alpha_t^z_t) in the
    // w row for the later passes, with sum log a_t.  Per TOA and likelihood: N0 (one FMA),
    // its reciprocal (estimate + one Newton step, ~2e-15 relative) times y^2 / a into the sum,
    // and N0 into a product of U factors (N0 ~ 1e-22 .. 1e-6 s^2: no under/overflow in 4)
    // that enters the mantissa / exponent accumulation once per round.
    double la = 0.0;
    auto lnlk = [&](auto kc, auto first_c, auto& out) __attribute__((always_inline)) {
      constexpr int K = decltype(kc)::value;
      constexpr bool FIRST = decltype(first_c)::value;
      double sq[K], lsv[2 * K + 1];
      LogProd lp[K];
      double lat = 0.0;   // FIRST: this thread's sum log a_t
#pragma unroll
      for (int j = 0; j < K; ++j) sq[j] = 0.0;
      // one backend: WU TOAs' loads in flight per round (the passes were latency-bound at one
      // load and one full wait per TOA)
      if (md.nb <= 1) {
        double e[K], q[K];
#pragma unroll
        for (int j = 0; j < K; ++j) {
          e[j] = wtab[j][0][0];
          q[j] = wtab[j][1][0];
        }
        const GDouble* s2 = (const GDouble*)md.sig2;
        const GDouble* w2 = (const GDouble*)wc;
        // WU TOAs per thread per round, all loads issued first (the first pass's four loads
        // per TOA: four TOAs per round); full rounds run unmasked, the last partial round is
        // masked (its TOAs past n read TOA threadIdx.x and contribute factor 1 / term 0)
        constexpr int U = FIRST ? 4 : WU;
        auto round = [&](int t0, auto masked_c) __attribute__((always_inline)) {
          constexpr bool M = decltype(masked_c)::value;
          double sv[U], wv[U], zv[U], av[U];
#pragma unroll
          for (int k = 0; k < U; ++k) {
            const int t = !M || t0 + k * TB < n ? t0 + k * TB : min((int)threadIdx.x, n - 1);
            sv[k] = s2[t];
            if constexpr (FIRST) {
              zv[k] = zc[t];
              av[k] = alc[t];
              wv[k] = yc[t];
            } else {
              wv[k] = w2[t];
            }
          }
#pragma unroll
          for (int k = 0; k < U; ++k) {
            const bool in = !M || t0 + k * TB < n;
            if constexpr (FIRST) {
              // w_t = y_t^2 / a_t, a_t = alpha_t^z_t; log 1 = 0 exactly, so only outliers add
              // to sum log a_t
              const bool zt = in && zv[k] != 0.0;
              const double at = zt ? av[k] : 1.0;
              lat += log(at);
              const double w = wv[k] * wv[k] / at;
              if (in) wc[t0 + k * TB] = w;
              wv[k] = w;
            }
            if constexpr (M) wv[k] = in ? wv[k] : 0.0;
          }
#pragma unroll
          for (int j = 0; j < K; ++j) {
            double pr = 1.0;
#pragma unroll
            for (int k = 0; k < U; ++k) {
              double N0 = e[j] * sv[k] + q[j];
              if constexpr (M) N0 = t0 + k * TB < n ? N0 : 1.0;
              pr *= N0;
              sq[j] = fma(wv[k], rcp_nr1(N0), sq[j]);
            }
            lp[j].mul(pr);
          }
        };
        int t0 = threadIdx.x;
        for (; t0 + (U - 1) * TB < n; t0 += U * TB) round(t0, std::false_type{});
        if (t0 < n) round(t0, std::true_type{});
      } else {
        for (int t = threadIdx.x; t < n; t += TB) {
          const double sv = md.sig2[t];
          const int b = md.bk[t];
          double wt;
          if constexpr (FIRST) {
            const double at = zc[t] != 0.0 ? alc[t] : 1.0;
            const double yt = yc[t];
            lat += log(at);
            wt = yt * yt / at;
            wc[t] = wt;
          } else {
            wt = wc[t];
          }
#pragma unroll
          for (int j = 0; j < K; ++j) {
            const double N0 = wtab[j][0][b] * sv + wtab[j][1][b];
            lp[j].mul(N0);
            sq[j] = fma(wt, rcp_nr1(N0), sq[j]);
          }
        }
      }
#pragma unroll
      for (int j = 0; j < K; ++j) {
        lsv[2 * j] = lp[j].log_sum();
        lsv[2 * j + 1] = sq[j];
      }
      lsv[2 * K] = lat;
      block_sum_k<TB / 64, 2 * K + 1>(lsv, redk);
      if constexpr (FIRST) la = lsv[2 * K];
#pragma unroll
      for (int j = 0; j < K; ++j) out[j] = -0.5 * ((la + lsv[2 * j]) + lsv[2 * j + 1]);
    };
    // The candidates' variances wait in LDS (wtab[j]: efac_b^2 and Q_b of every backend, one
    // thread per backend), so that only the chain's own x lives in registers across a pass
    // (three proposals' parameter vectors and variance sets held there cost ~190 registers
    // and spilled).  A proposal is (x0, Q0) moved by its step's jump; Q of a one-backend
    // model is carried multiplicatively (Q0 10^(2 delta) when the step moves equad).
    constexpr double LN10 = 2.302585092994045684;
    auto propose = [&](int step, const XVec& x0, double Q0, XVec& qv, double& Qq)
        __attribute__((always_inline)) {
      const int par = (int)mhv[step][0];
#pragma unroll
      for (int j = 0; j < PMAX; ++j) qv[j] = (j == par) ? x0[j] + mhv[step][1] : x0[j];
      Qq = (par == md.idx_equad) ? Q0 * mhv[step][3] : Q0;
    };
    auto stage = [&](int j, const XVec& qv, double Qq) __attribute__((always_inline)) {
      const int b = threadIdx.x;
      if (b < md.nb) {
        const int ei = md.efac_b[b];
        const double xe = xget(qv, ei >= 0 ? ei : 0);
        const double ef = ei >= 0 ? xe : md.efac_const;
        wtab[j][0][b] = ef * ef;
        wtab[j][1][b] = md.nb <= 1 ? Qq : exp(2.0 * xget(qv, md.equad_b[b]) * LN10);
      }
    };
    double Qx = exp(2.0 * xget(xv, md.equad_b[0]) * LN10);   // (one backend: the carried Q)
    double l0, p0 = lnpriorP(md, xv);
    stage(0, xv, Qx);
    if (a.eval_only) {
      __syncthreads();
      double l1v[1];
      lnlk(std::integral_constant<int, 1>{}, std::true_type{}, l1v);
      l0 = l1v[0];
      if (threadIdx.x == 0) a.out_w[c] = l0;
    } else {
      // MH steps two per pass (gibbs.py:114-143 runs them one at a time): a pass evaluates
      // step s's proposal from the current state and both possible proposals of step s + 1
      // (from the state step s rejects to, and from the one it accepts to), so the 21
      // likelihoods of the block take 11 passes over the TOAs.  Decisions, proposals and
      // values are exactly the sequential loop's (a proposal outside the prior is evaluated
      // and ignored, where the loop skips it); proposals are recomputed, not kept, after a
      // pass.
      auto settle = [&](int step, const XVec& x0, double Q0, double l1)
          __attribute__((always_inline)) -> bool {
        XVec qv;
        double Qq;
        propose(step, x0, Q0, qv, Qq);
        const double p1 = lnpriorP(md, qv);
        const bool acc = p1 != -INFINITY && (l1 + p1) - (l0 + p0) > mhv[step][2];
        if (acc) {
#pragma unroll
          for (int j = 0; j < PMAX; ++j) xv[j] = qv[j];
          l0 = l1;
          p0 = p1;
          Qx = Qq;
        }
        return acc;
      };
      {  // pass 0: the current state and step 0's proposal
        {
          XVec q0;
          double Q0;
          propose(0, xv, Qx, q0, Q0);
          stage(1, q0, Q0);
        }
        __syncthreads();
        double lv[2];
        lnlk(std::integral_constant<int, 2>{}, std::true_type{}, lv);
        l0 = lv[0];
        settle(0, xv, Qx, lv[1]);
      }
      for (int step = 1; step < NWHITE; step += 2) {
        const bool two = step + 1 < NWHITE;
        {
          XVec qs, qo;
          double Qs, Qo;
          propose(step, xv, Qx, qs, Qs);
          stage(0, qs, Qs);
          if (two) {
            propose(step + 1, xv, Qx, qo, Qo);     // step s rejected
            stage(1, qo, Qo);
            propose(step + 1, qs, Qs, qo, Qo);     // step s accepted
            stage(2, qo, Qo);
          }
        }
        __syncthreads();
        double lv[3];
        if (two) {
          lnlk(std::integral_constant<int, 3>{}, std::false_type{}, lv);
        } else {
          double l1v[1];
          lnlk(std::integral_constant<int, 1>{}, std::false_type{}, l1v);
          lv[0] = l1v[0];
        }
        const bool acc = settle(step, xv, Qx, lv[0]);
        // step s + 1 from the state step s left (xv, Qx are already that state)
        if (two) settle(step + 1, xv, Qx, acc ? lv[2] : lv[1]);
      }
      if (threadIdx.x < md.P) a.st.x[(size_t)c * md.P + threadIdx.x] = xget(xv, threadIdx.x);
    }
  }
  __syncthreads();
  // N^-1, sum log N, r^T N^-1 r at the final white parameters (gibbs.py:297,309-312)
  const WhiteNoise wf = white_noise(md, xv);
  double sr = 0.0;
  LogProd lp;
  for (int t0 = threadIdx.x; t0 < npad; t0 += WU * TB) {
    double zv[WU], av[WU], sv[WU], rv[WU];
    int bv[WU];
#pragma unroll
    for (int k = 0; k < WU; ++k) {
      const int t = t0 + k * TB < n ? t0 + k * TB : min((int)threadIdx.x, n - 1);  // in-bounds, masked below
      zv[k] = zc[t];
      av[k] = alc[t];
      sv[k] = wf.s2[t];
      rv[k] = md.resid[t];
      bv[k] = wf.nb > 1 ? wf.bk[t] : 0;
    }
#pragma unroll
    for (int k = 0; k < WU; ++k) {
      const int t = t0 + k * TB;
      if (t >= npad) continue;
      double wt = 0.0;
      if (t < n) {
        const double N = (zv[k] != 0.0 ? av[k] : 1.0) * wf.n0v(bv[k], sv[k]);
        lp.mul(N);
        sr += rv[k] * rv[k] / N;
        wt = 1.0 / N;
      }
      wc[t] = wt;
    }
  }
  const double sl = block_sum<TB / 64>(lp.log_sum(), red);
  sr = block_sum<TB / 64>(sr, red);
  if (threadIdx.x == 0) {
    sc[SC_LOGDETN] = sl;
    sc[SC_RNR] = sr;
  }
}

// ------------------------------------------------------------------------------------
// gram: G_c = T_aug^T diag(w_c) T_aug, lower 16x16 tiles, fp64 MFMA 16x16x4
// ------------------------------------------------------------------------------------
// Workgroup = 8 waves = 8 chains sharing one 64x64 super-tile (I, J) of the Gram.  The T
// operands (8 column tiles x 16 k-steps = 64 TOAs = 64 KB) are staged cooperatively in LDS,
// double-buffered: chunk i+1 is fetched into registers while chunk i feeds the MFMAs, so
// every T element is read from L2/HBM once per workgroup and the MFMAs never wait on a
// global load.  Each wave scales its A operand by its own chain's weights (LDS too).
constexpr int GRAM_KC = 16;                       // k-steps (of 4 TOAs) per chunk
constexpr int GRAM_LDS = 2 * GRAM_KC * 8 * 64 + 2 * GRAM_WAVES * 64;   // doubles

// Inner loop + store of one super-tile; the valid tile pattern (NU rows of tiles, diagonal
// or not) is a template parameter, so the 16 MFMAs of a k-step are straight-line code (with
// the pattern as runtime conditions every MFMA sat behind its own scalar branch).
template <int NU, bool DIAG>
__device__ __forceinline__ void gram_tile(const DevModel& md, const LArgs& a, double* Tl,
                                          double* Wl, int I, int J, int c, bool live) {
  constexpr int NV = DIAG ? NU : 4;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int NT = md.mp / 16;
  const int nch = md.npad / (4 * GRAM_KC);
  const double* wc = a.s.w + (size_t)c * a.ys;
  const int tl = lane >> 4;

  // staging map: 512 threads x 8 double2 = 8 tiles x 16 k-steps x 32 double2
  int gcol[8];
#pragma unroll
  for (int u = 0; u < 8; ++u) gcol[u] = min(u < 4 ? 4 * I + u : 4 * J + u - 4, NT - 1);
  typedef double v2d __attribute__((ext_vector_type(2)));
  v2d stg[8];
  double wstg;
  auto fetch = [&](int ch) __attribute__((always_inline)) {
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      const int e = tid + 512 * r;
      const int q = e & 31, u = (e >> 5) & 7, k = e >> 8;
      const size_t ks = (size_t)ch * GRAM_KC + k;
      stg[r] = *(const v2d*)(md.Tmf + (ks * NT + gcol[u]) * 64 + 2 * q);
    }
    wstg = wc[(size_t)ch * 64 + lane];
  };
  auto stash = [&](int buf) __attribute__((always_inline)) {
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      const int e = tid + 512 * r;
      const int q = e & 31, u = (e >> 5) & 7, k = e >> 8;
      *(v2d*)(Tl + ((buf * GRAM_KC + k) * 8 + u) * 64 + 2 * q) = stg[r];
    }
    Wl[(buf * GRAM_WAVES + wv) * 64 + lane] = wstg;
  };

  v4d acc[4][4];
#pragma unroll
  for (int u = 0; u < 4; ++u)
#pragma unroll
    for (int v = 0; v < 4; ++v) acc[u][v] = (v4d){0.0, 0.0, 0.0, 0.0};
  fetch(0);
  stash(0);
  __syncthreads();
#pragma unroll 1
  for (int ch = 0; ch < nch; ++ch) {
    const int buf = ch & 1;
    if (ch + 1 < nch) fetch(ch + 1);
    const double* Tb = Tl + buf * GRAM_KC * 8 * 64 + lane;
    const double* Wb = Wl + (buf * GRAM_WAVES + wv) * 64 + tl;
    // operands of k-step k+1 are read from LDS before k's MFMAs are issued, so the
    // lgkmcnt wait is covered by the k-step's MFMAs instead of stalling the wave
    double ta[4], tb[4], wt = Wb[0];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      ta[u] = u < NU ? Tb[u * 64] : 0.0;
      tb[u] = u < NV ? Tb[(4 + u) * 64] : 0.0;
    }
#pragma unroll
    for (int k = 0; k < GRAM_KC; ++k) {
      double na[4], nb[4], nw = 0.0;
      if (k + 1 < GRAM_KC) {
        nw = Wb[4 * (k + 1)];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          na[u] = u < NU ? Tb[((k + 1) * 8 + u) * 64] : 0.0;
          nb[u] = u < NV ? Tb[((k + 1) * 8 + 4 + u) * 64] : 0.0;
        }
      }
      double aw[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) aw[u] = ta[u] * wt;
#pragma unroll
      for (int u = 0; u < NU; ++u)
#pragma unroll
        for (int v = 0; v < NV; ++v)
          if (!DIAG || v <= u)
            acc[u][v] = __builtin_amdgcn_mfma_f64_16x16x4f64(aw[u], tb[v], acc[u][v], 0, 0, 0);
      if (k + 1 < GRAM_KC) {
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          ta[u] = na[u];
          tb[u] = nb[u];
        }
        wt = nw;
      }
      // the other buffer is free since the last barrier: stash the prefetched chunk mid-way
      // so the wait for its global loads overlaps the second half of this chunk's MFMAs
      if (k == GRAM_KC / 2 - 1 && ch + 1 < nch) stash(buf ^ 1);
    }
    __syncthreads();
  }
  if (!live) return;
  double* Gc = a.s.G + (size_t)c * md.mp * md.mp;
#pragma unroll
  for (int u = 0; u < NU; ++u)
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      if (DIAG && v > u) continue;
      const int X = 4 * I + u, Y = 4 * J + v;
#pragma unroll
      for (int g = 0; g < 4; ++g)
        Gc[(size_t)(16 * X + tl + 4 * g) * md.mp + 16 * Y + (lane & 15)] = acc[u][v][g];
    }
}

__global__ void __launch_bounds__(64 * GRAM_WAVES) lg_gram(const DevModel* __restrict__ mds,
                                                           LArgs a, int nsb, int npairs) {
  extern __shared__ double lsm[];
  double* Tl = lsm;                               // [2][KC][8 tiles][64]
  double* Wl = lsm + 2 * GRAM_KC * 8 * 64;        // [2][8 waves][64]
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  // block order: pair-major (the chain groups of one super-tile run together and share its
  // T columns in L2), off-diagonal super-tiles first, the shorter diagonal ones last
  const int ngroups = (a.C + GRAM_WAVES - 1) / GRAM_WAVES;
  const int prank = blockIdx.x / ngroups;
  const int cg = (blockIdx.x % ngroups) * GRAM_WAVES + wv;
  const bool live = cg < a.C;
  const int c = live ? cg : a.C - 1;              // dead waves still stage and sync
  // the group's dataset (its first chain's): every wave stages that dataset's T
  const int dsg = ds_of(a, (blockIdx.x % ngroups) * GRAM_WAVES);
  const DevModel& md = mds[dsg];
  if (gram_ec_of(md, a.hyper_lds, a.st.debug)) return;   // the group's Gram is lg_gram_ec's
  if (live && prank == 0 && ds_of(a, c) != dsg && (threadIdx.x & 63) == 0 && a.st.status)
    a.st.status[c] |= 8;                          // batch layout violated: flag, never silent
  const int noff = npairs - nsb;
  int I, J;
  if (prank < noff) {                              // (I, J), I > J, row-major
    I = 1;
    while (I * (I + 1) / 2 <= prank) ++I;
    J = prank - I * (I - 1) / 2;
  } else {
    I = J = prank - noff;
  }
  const int NT = md.mp / 16;
  const int nu = min(4, NT - 4 * I);              // valid tile rows (columns: 4 off-diagonal)
  // wave-uniform dispatch on the tile pattern
  if (I != J) {
    switch (nu) {
      case 4: gram_tile<4, false>(md, a, Tl, Wl, I, J, c, live); break;
      case 3: gram_tile<3, false>(md, a, Tl, Wl, I, J, c, live); break;
      case 2: gram_tile<2, false>(md, a, Tl, Wl, I, J, c, live); break;
      default: gram_tile<1, false>(md, a, Tl, Wl, I, J, c, live); break;
    }
  } else {
    switch (nu) {
      case 4: gram_tile<4, true>(md, a, Tl, Wl, I, J, c, live); break;
      case 3: gram_tile<3, true>(md, a, Tl, Wl, I, J, c, live); break;
      case 2: gram_tile<2, true>(md, a, Tl, Wl, I, J, c, live); break;
      default: gram_tile<1, true>(md, a, Tl, Wl, I, J, c, live); break;
    }
  }
}

// ------------------------------------------------------------------------------------
// gram, small models (mp <= 16 GS_NTMAX): one wave per chain computes every lower tile of its
// Gram, T streamed from L2 with two k-steps of operands in flight (the persistent kernel's
// Gram loop, weights from the white pass's w row).  With a few 16-column tiles the 64x64
// super-tiles of lg_gram split the lower triangle unevenly between their workgroups (m ~ 75:
// 10 / 4 / 1 tiles), and the diagonal one set the time.  Every tile receives the same MFMA
// sequence as in lg_gram (k-steps in order, A = T w, B = T), so G is bitwise lg_gram's.
// ------------------------------------------------------------------------------------
constexpr int GS_NTMAX = 6;
constexpr int GS_WPB = 4;
constexpr int GS_DEPTH = 4;
template <int NT>
__global__ void __launch_bounds__(64 * GS_WPB) lg_gram_small(const DevModel* __restrict__ mds,
                                                               LArgs a) {
  constexpr int NTT = NT * (NT + 1) / 2;
  const int lane = threadIdx.x & 63;
  const int c = blockIdx.x * GS_WPB + (int)__builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  if (c >= a.C) return;
  const DevModel& md = mds[ds_of(a, c)];
  if (gram_ec_of(md, a.hyper_lds, a.st.debug)) return;   // lg_gram_ec's chain
  const int tl = lane >> 4, nks = md.npad / 4, mp = md.mp;
  const GDouble* wc = (const GDouble*)(a.s.w + (size_t)c * a.ys);
  const GDouble* Tm = (const GDouble*)md.Tmf;
  v4d acc[NTT];
#pragma unroll
  for (int i = 0; i < NTT; ++i) acc[i] = (v4d){0.0, 0.0, 0.0, 0.0};
  // GS_DEPTH k-steps of operands in flight: a set is reloaded right after its MFMAs issue, so
  // its loads have GS_DEPTH - 1 k-steps of MFMAs (T misses L2 beyond ~4k TOAs) to arrive
  constexpr int D = GS_DEPTH;
  double t[D][NT], w[D];
  auto tload = [&](double (&tt)[NT], double& ww, int ks) __attribute__((always_inline)) {
#pragma unroll
    for (int X = 0; X < NT; ++X) tt[X] = Tm[((size_t)ks * NT + X) * 64 + lane];
    ww = wc[4 * ks + tl];
  };
  auto kstep = [&](const double (&t)[NT], const double wt) __attribute__((always_inline)) {
#pragma unroll
    for (int I = 0; I < NT; ++I) {
      const double av = t[I] * wt;
#pragma unroll
      for (int J = 0; J <= I; ++J)
        acc[I * (I + 1) / 2 + J] =
            __builtin_amdgcn_mfma_f64_16x16x4f64(av, t[J], acc[I * (I + 1) / 2 + J], 0, 0, 0);
    }
  };
  // nks = npad / 4 is a multiple of 16: the main loop has no conditional load, so the
  // compiler's wait counts keep the later sets' loads in flight (a branch in the body made
  // it wait for every load at the top of each iteration)
  static_assert(16 % D == 0, "k-step count is a multiple of 16");
#pragma unroll
  for (int d = 0; d < D; ++d) {
    tload(t[d], w[d], d);
    __builtin_amdgcn_sched_barrier(0);
  }
  int ks = 0;
  for (; ks + D < nks; ks += D) {
#pragma unroll
    for (int d = 0; d < D; ++d) {
      kstep(t[d], w[d]);
      tload(t[d], w[d], ks + d + D);
      // keep the k-steps in program order: the scheduler otherwise hoists all four sets'
      // weight multiplies to the top of the body, i.e. waits for every load there
      __builtin_amdgcn_sched_barrier(0);
    }
  }
#pragma unroll
  for (int d = 0; d < D; ++d) kstep(t[d], w[d]);
  double* Gc = a.s.G + (size_t)c * mp * mp;
#pragma unroll
  for (int I = 0; I < NT; ++I)
#pragma unroll
    for (int J = 0; J <= I; ++J)
#pragma unroll
      for (int g = 0; g < 4; ++g)
        Gc[(size_t)(16 * I + tl + 4 * g) * mp + 16 * J + (lane & 15)] = acc[I * (I + 1) / 2 + J][g];
}

// ------------------------------------------------------------------------------------
// gram, disjoint ECORR epochs (hyper class 2): only the blocks the epochs-first elimination
// reads.  With X = [timing model | Fourier] (internal columns 0 .. Q-1), r and the epoch
// columns E (each TOA in at most one epoch, value u_t):
//   G_xx = [X|r]^T W [X|r]       one wave's MFMA tiles over the compact packed [X | r | 1]
//   G_ee = sum_{t in e} w_t u_t^2,   G_ex = sum_{t in e} w_t u_t [X|r]_t
// the second pair as MFMAs too: per block of 16 epochs, A = the 16 x 4 indicator of which
// epoch each of 4 consecutive (epoch-ordered) TOAs belongs to, B = their w u [X | r | u] rows,
// accumulating the block's 16 rows of [G_ex | G_er | G_ee].  O(n (Q + 2)^2 / 2) MFMA work per
// chain instead of the dense Gram's O(n mp^2 / 2) (gibbs.py:302-304; the E-E off-diagonal
// blocks are exactly zero and never read).  Two waves per chain: G_xx and the epochs' blocks
// (their MFMAs share the SIMD's pipe; the second wave hides the first's load latency).
// ------------------------------------------------------------------------------------
constexpr int GEC_CPB = GS_WPB / 2;   // chains per lg_gram_ec workgroup
template <int NX>
__global__ void __launch_bounds__(64 * GS_WPB) lg_gram_ec(const DevModel* __restrict__ mds,
                                                            LArgs a) {
  constexpr int NXT = NX * (NX + 1) / 2;
  const int lane = threadIdx.x & 63;
  const int wv = (int)__builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int c = blockIdx.x * GEC_CPB + (wv >> 1), role = wv & 1;
  if (c >= a.C) return;
  const DevModel& md = mds[ds_of(a, c)];
  if (!gram_ec_of(md, a.hyper_lds, a.st.debug) || md.gx_nt != NX) return;
  const int tl = lane >> 4, mp = md.mp, Q = md.ntm_pad + md.nf, raug = md.raug;
  const int ec0 = md.ntm_pad + md.nf;   // internal column of epoch 0
  const GDouble* wc = (const GDouble*)(a.s.w + (size_t)c * a.ys);
  double* Gc = a.s.G + (size_t)c * mp * mp;
  constexpr int D = GS_DEPTH;
  // ---- G_xx: lg_gram_small's loop over the compact columns
  if (role == 0) {
    const GDouble* Tm = (const GDouble*)md.Tx;
    const int nks = md.npad / 4;
    v4d acc[NXT];
#pragma unroll
    for (int i = 0; i < NXT; ++i) acc[i] = (v4d){0.0, 0.0, 0.0, 0.0};
    double t[D][NX], w[D];
    auto tload = [&](double (&tt)[NX], double& ww, int ks) __attribute__((always_inline)) {
#pragma unroll
      for (int X = 0; X < NX; ++X) tt[X] = Tm[((size_t)ks * NX + X) * 64 + lane];
      ww = wc[4 * ks + tl];
    };
    auto kstep = [&](const double (&tt)[NX], const double wt) __attribute__((always_inline)) {
#pragma unroll
      for (int I = 0; I < NX; ++I) {
        const double av = tt[I] * wt;
#pragma unroll
        for (int J = 0; J <= I; ++J)
          acc[I * (I + 1) / 2 + J] =
              __builtin_amdgcn_mfma_f64_16x16x4f64(av, tt[J], acc[I * (I + 1) / 2 + J], 0, 0, 0);
      }
    };
    static_assert(16 % D == 0, "k-step count is a multiple of 16");
#pragma unroll
    for (int d = 0; d < D; ++d) {
      tload(t[d], w[d], d);
      __builtin_amdgcn_sched_barrier(0);
    }
    int ks = 0;
    for (; ks + D < nks; ks += D) {
#pragma unroll
      for (int d = 0; d < D; ++d) {
        kstep(t[d], w[d]);
        tload(t[d], w[d], ks + d + D);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
#pragma unroll
    for (int d = 0; d < D; ++d) kstep(t[d], w[d]);
    // compact column q -> internal: q < Q itself, Q the residual row, Q + 1 (ones) unused
#pragma unroll
    for (int I = 0; I < NX; ++I)
#pragma unroll
      for (int J = 0; J <= I; ++J)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int qa = 16 * I + tl + 4 * g, qb = 16 * J + (lane & 15);
          if (qa >= qb && qa <= Q && qb <= Q) {
            const int gi = qa < Q ? qa : raug, gj = qb < Q ? qb : raug;
            Gc[(size_t)gi * mp + gj] = acc[I * (I + 1) / 2 + J][g];
          }
        }
  }
  // ---- epochs: blocks of 16, A = indicator (lane: row = lane & 15, k = lane >> 4),
  // B = w_t u_t [X | r | u]_t (lane: k = lane >> 4, column = lane & 15)
  if (role == 1) {
    const GDouble* Xe = (const GDouble*)md.Xe;
    const int* ekl = md.ekl;
    const int nks = md.nkse;
    v4d acc[NX];
#pragma unroll
    for (int v = 0; v < NX; ++v) acc[v] = (v4d){0.0, 0.0, 0.0, 0.0};
    double xb[D][NX], ind[D];
    auto eload = [&](int d, int ks) __attribute__((always_inline)) {
      const int p = 4 * ks + tl;
      const int tt = ekl[2 * p], el = ekl[2 * p + 1];
      const double wt = tt >= 0 ? (double)wc[tt] : 0.0;
      ind[d] = el == (lane & 15) ? 1.0 : 0.0;
#pragma unroll
      for (int v = 0; v < NX; ++v) xb[d][v] = Xe[((size_t)ks * NX + v) * 64 + lane] * wt;
    };
    auto flush = [&](int blk) __attribute__((always_inline)) {
#pragma unroll
      for (int v = 0; v < NX; ++v) {
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int e = 16 * blk + tl + 4 * g, q = 16 * v + (lane & 15);
          if (e < md.nec) {
            const int ge = ec0 + e;
            if (q < Q)
              Gc[(size_t)ge * mp + q] = acc[v][g];
            else if (q == Q)
              Gc[(size_t)raug * mp + ge] = acc[v][g];
            else if (q == Q + 1)
              Gc[(size_t)ge * mp + ge] = acc[v][g];
          }
        }
        acc[v] = (v4d){0.0, 0.0, 0.0, 0.0};
      }
    };
    static_assert(16 % D == 0, "k-step count is a multiple of 16");
#pragma unroll
    for (int d = 0; d < D; ++d) {
      eload(d, d);
      __builtin_amdgcn_sched_barrier(0);
    }
    int blk = 0, kend = md.eblk[1];
    int ks = 0;
    auto estep = [&](int d, int k) __attribute__((always_inline)) {
      while (k == kend) {              // (wave-uniform) the block's k-steps are done
        if (blk < md.neblk) flush(blk);
        ++blk;
        kend = blk < md.neblk ? md.eblk[blk + 1] : 0x7fffffff;
      }
#pragma unroll
      for (int v = 0; v < NX; ++v)
        acc[v] = __builtin_amdgcn_mfma_f64_16x16x4f64(ind[d], xb[d][v], acc[v], 0, 0, 0);
    };
    for (; ks + D < nks; ks += D) {
#pragma unroll
      for (int d = 0; d < D; ++d) {
        estep(d, ks + d);
        eload(d, ks + d + D);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
#pragma unroll
    for (int d = 0; d < D; ++d) estep(d, ks + d);
    if (blk < md.neblk) flush(blk);
  }
}

// ------------------------------------------------------------------------------------
// tmelim: eliminate the timing-model columns [0, K0) of G (LDL^T-scaled, raw columns)
// ------------------------------------------------------------------------------------
// Panels of 16 columns: the panel (rows k0..mp) is factored in LDS, written back, then the
// trailing lower triangle is updated by MFMA: G_ij -= sum_kk P_i,kk P_j,kk / a_kk.
// Blocked right-looking LDL^T (raw columns) of columns [k_lo, k_hi) of a symmetric mp x mp
// matrix (row-major, lower triangle): panels of TM_PW columns factored in LDS (P, [mp][TM_PW+1]),
// each panel written back raw to Gout, the trailing lower triangle (rows / columns past the
// panel, up to mp) updated by MFMA tiles.  The first panel and its trailing tiles are read from
// Gin, every later read is of Gout (Gin stays intact).  diag(gk, v) gives diagonal element gk
// as its panel is loaded (priors are added there: a trailing update never reads a diagonal
// before its own panel).  Thread 0 accumulates sum log a_kk, sum a_{zrow,k}^2 / a_kk, the
// smallest / largest pivot of the columns real(gk) selects and the failure flag.  k_lo and mp
// are multiples of 16; the last panel may be partial (its columns past k_hi are updated, not
// eliminated).  trail_all: also update the trailing triangle after the last panel (the
// timing-model elimination leaves the Schur complement S0 there).
template <class DiagF, class RealF>
__device__ void panel_ldl(const double* Gin, double* Gout, int mp, int k_lo, int k_hi, int zrow,
                          bool trail_all, DiagF diag, RealF real, double* P, double* ainv,
                          double& ld, double& quad, double& pmin, double& pmax, int& fail) {
  constexpr int PS = TM_PW + 1;        // panel row stride
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  for (int k0 = k_lo; k0 < k_hi; k0 += TM_PW) {
    const int R = mp - k0;
    const int pw = k_hi - k0 < TM_PW ? k_hi - k0 : TM_PW;
    const double* Gsrc = k0 == k_lo ? Gin : Gout;
    // load the panel
    for (int e = tid; e < R * TM_PW; e += LBLK) {
      const int i = e / TM_PW, kk = e % TM_PW;
      const int gi = k0 + i, gk = k0 + kk;
      double v = (gi >= gk) ? Gsrc[(size_t)gi * mp + gk] : 0.0;
      if (gi == gk && kk < pw) v = diag(gk, v);
      P[i * PS + kk] = v;
    }
    __syncthreads();
    // factor the panel (columns kk < pw, rows kk..R)
    for (int kk = 0; kk < pw; ++kk) {
      const double akk = P[kk * PS + kk];
      const double r = 1.0 / akk;
      for (int e = tid; e < (R - kk - 1) * (TM_PW - kk - 1); e += LBLK) {
        const int i = kk + 1 + e / (TM_PW - kk - 1);
        const int j = kk + 1 + e % (TM_PW - kk - 1);
        if (j <= i) P[i * PS + j] -= P[i * PS + kk] * (P[j * PS + kk] * r);
      }
      if (tid == 0) {
        fail |= !(akk > 0.0) ? 1 : 0;
        if (real(k0 + kk)) {
          pmin = fmin(pmin, akk);
          pmax = fmax(pmax, akk);
        }
        ld += log(akk);
        const double zr = P[(zrow - k0) * PS + kk];
        quad += zr * zr * r;
        ainv[kk] = r;
      }
      __syncthreads();
    }
    if (pw < TM_PW) {   // columns past k_hi: no update from them
      if (tid < TM_PW && tid >= pw) ainv[tid] = 0.0;
      __syncthreads();
    }
    // write the raw panel back (columns k0..k0+16, rows >= column)
    for (int e = tid; e < R * TM_PW; e += LBLK) {
      const int i = e / TM_PW, kk = e % TM_PW;
      if (i >= kk) Gout[(size_t)(k0 + i) * mp + k0 + kk] = P[i * PS + kk];
    }
    // trailing update of rows/cols >= k1 by MFMA tiles (wave-strided over lower tiles)
    const int k1 = k0 + TM_PW;
    if (k1 < k_hi || trail_all) {
      const int TR = (mp - k1) / 16;
      const int ntile = TR * (TR + 1) / 2;
      // TM_TILES tiles per wave per round, their loads issued first (the rounds were bound by
      // one global load round trip per tile); tiles past ntile in the last round are masked
      constexpr int NW = LBLK / 64;
      for (int e0 = wv; e0 < ntile; e0 += TM_TILES * NW) {
        int r0[TM_TILES], c0[TM_TILES];
        bool in[TM_TILES];
        v4d acc[TM_TILES];
#pragma unroll
        for (int h = 0; h < TM_TILES; ++h) {
          const int e = e0 + h * NW;
          in[h] = e < ntile;
          const int ee = in[h] ? e : e0;
          int X = 0;
          while ((X + 1) * (X + 2) / 2 <= ee) ++X;
          const int Y = ee - X * (X + 1) / 2;
          r0[h] = k1 + 16 * X;
          c0[h] = k1 + 16 * Y;
#pragma unroll
          for (int g = 0; g < 4; ++g)
            acc[h][g] = Gsrc[(size_t)(r0[h] + (lane >> 4) + 4 * g) * mp + c0[h] + (lane & 15)];
        }
#pragma unroll
        for (int h = 0; h < TM_TILES; ++h) {
#pragma unroll
          for (int k4 = 0; k4 < TM_PW / 4; ++k4) {
            const int kk = 4 * k4 + (lane >> 4);
            const double av = -P[(r0[h] - k0 + (lane & 15)) * PS + kk];
            const double bv = P[(c0[h] - k0 + (lane & 15)) * PS + kk] * ainv[kk];
            acc[h] = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, acc[h], 0, 0, 0);
          }
          if (in[h]) {
#pragma unroll
            for (int g = 0; g < 4; ++g)
              Gout[(size_t)(r0[h] + (lane >> 4) + 4 * g) * mp + c0[h] + (lane & 15)] = acc[h][g];
          }
        }
      }
    }
    __syncthreads();
  }
}

__global__ void __launch_bounds__(LBLK) lg_tmelim(const DevModel* __restrict__ mds, LArgs a) {
  const int c = blockIdx.x;
  const DevModel& md = mds[ds_of(a, c)];
  double* sc = a.s.sc + (size_t)c * 16;
  // floor pass: only the chains whose b draw runs at the SVD noise floor, with Sigma + f I
  const double fsh = a.floor_pass ? sc[SC_FLOOR] : 0.0;
  if (a.floor_pass && !(fsh > 0.0)) return;
  if (hyper_class_of(md, a.hyper_lds) == 2) return;   // lg_hyper<2> factors the timing model
  extern __shared__ double lsm[];
  double* P = lsm;                     // [mp][TM_PW + 1]
  __shared__ double ainv[TM_PW];
  const int mp = md.mp, K0 = md.ntm_pad;
  // G stays the Gram (the floor pass re-eliminates it); the factor and S0 go to G2
  const double* Gg = a.s.G + (size_t)c * mp * mp;
  double* Gc = a.s.G2 + (size_t)c * mp * mp;
  double ld = 0.0, quad = 0.0, pmin = INFINITY, pmax = 0.0;
  int fail = 0;
  // timing-model prior 1/tm_weight on its diagonal, unit pivots on the pad columns
  const int ntm = md.ntm;
  const double tmp = md.tm_phiinv;
  panel_ldl(Gg, Gc, mp, 0, K0, md.raug, true,
            [&](int gk, double v) { return (gk < ntm) ? (v + tmp) + fsh : 1.0; },
            [&](int gk) { return gk < ntm; }, P, ainv, ld, quad, pmin, pmax, fail);
  if (threadIdx.x == 0) {
    sc[SC_LDTM] = ld;
    sc[SC_QUADTM] = quad;
    sc[SC_FAILTM] = (double)fail;
    sc[SC_TMPMIN] = pmin;
    sc[SC_TMPMAX] = pmax;
  }
}

// ------------------------------------------------------------------------------------
// hyper: red-noise MH on S0 + diag(phi^-1) in LDS; b draw's Fourier block
// ------------------------------------------------------------------------------------
struct HyperLds {
  double* S;    // [ms][SS] working factor (raw columns), row-major lower
  int SS;
};

// MODE 1 (BIG, hyper class 1: blocks past HYPER_LDS_MAX columns): the same MH, likelihood
// and b draw with the block factored by panel_ldl into the chain's G3 instead of in LDS (S is
// then G3's hyper block, row stride mp).
//
// MODE 2 (EC, hyper class 2: such blocks made of ECORR epochs around a timing-model + Fourier
// block of at most EC_QX_MAX rows -- NANOGrav-style pulsars, one ECORR column per observing
// epoch): Sigma is eliminated epochs first, in the order [ECORR | TM | Fourier], from the raw
// Gram G.  Epochs share no TOA, so the ECORR block of T^T N^-1 T is diagonal and eliminating it
// costs no fill: pivots a_e = G_ee + phi_e^-1, and the rest becomes
//   X = G_xx + diag(phi_x^-1) - sum_e G_xe G_ex / a_e      (x: TM, Fourier, augmented row)
// factored densely in LDS.  Per likelihood that is O(nec qx^2) + O(qx^3) work instead of the
// (nf + nec)^3 of MODE 1; lg_tmelim does nothing for these chains (the timing model is part
// of X, so its prior enters per likelihood) and this kernel draws all of b (lg_btm skips
// them).  Same variates (Philox by internal column), MH decisions and outputs otherwise.
template <int MODE>
__global__ void __launch_bounds__(LBLK) lg_hyper(const DevModel* __restrict__ mds, LArgs a) {
  constexpr bool BIG = MODE == 1, EC = MODE == 2;
  const int c = blockIdx.x;
  const DevModel& md = mds[ds_of(a, c)];
  if (hyper_class_of(md, a.hyper_lds) != MODE) return;   // another class's chain
  if (EC && ec_reg_mt_of(md, a.hyper_lds, a.st.debug)) return;   // lg_hyper_ecr's chain
  extern __shared__ double lsm[];
  // the hyper-dependent columns: Fourier (power law) then ECORR epochs (10^(2 ecorr_b))
  const int nf = md.nf + md.nec, K0 = md.ntm_pad, mp = md.mp;
  const int nfr = md.nf, nec = md.nec, ntm = md.ntm;
  const int ms = nf + 1;               // Fourier + ECORR block + augmented row
  // EC: X's rows: ntm timing-model columns, nfr Fourier columns, the augmented row (nxd = qx-1)
  const int qx = ntm + nfr + 1, nxd = qx - 1, qxp = (qx + 15) & ~15;
  const int SS = BIG ? mp : (EC ? qx + 1 : ms + 1);
  // LDS: S [ms][SS] (BIG: the panel [mp][TM_PW + 1] and 1 / a_kk [TM_PW] instead; EC: X
  // [qx][SS] and its epochs-eliminated base XB [qx][SS], then the vectors below sized mp, the
  // pivots a_e, one chunk of couplings [EC_ECH][qxp])
  double* P = lsm;
  double* S = BIG ? a.s.G3 + (size_t)blockIdx.x * mp * mp + (size_t)K0 * mp + K0 : lsm;
  double* ainv = lsm + mp * (TM_PW + 1);
  double* XB = S + qx * SS;            // EC: G_xx - sum_e G_xe G_ex / a_e (no priors)
  double* ph = BIG ? ainv + TM_PW : S + (EC ? 2 * qx : ms) * SS;   // [nf] phi^-1
  const int vlen = EC ? mp : ms;
  double* vv = ph + nf;                // [vlen] back-substitution accumulators / Delta
  double* wv_ = vv + vlen;             // [vlen] rhs
  double* aE = wv_ + vlen;             // EC: [nec] epoch pivots a_e
  double* Ech = aE + nec;              // EC: [2][EC_ECH][qxp] couplings G_ex, two chunks of epochs
  double* einv = Ech + 2 * EC_ECH * qxp;   // EC: [2][EC_ECH] their 1 / a_e
  double* dl = einv + 2 * EC_ECH;      // EC: [mp] Delta (tape mode), internal order
  double* vfull = dl + mp;             // EC: [mp] the b draw, internal order
  const double* Gg = a.s.G + (size_t)c * mp * mp;   // EC: the raw Gram (lower triangle)
  // EC: internal column of X's row i, and G at (r, q) from the lower triangle
  auto gx = [&](int i) { return i < ntm ? i : (i < nxd ? K0 + (i - ntm) : md.raug); };
  auto Gl = [&](int r, int q) { return r >= q ? Gg[(size_t)r * mp + q] : Gg[(size_t)q * mp + r]; };
  // EC: this wave's lower 16x16 tiles of X (tile t = wave + 4 h, rows r0_, columns c0_)
  int r0_[EC ? EC_TPW : 1], c0_[EC ? EC_TPW : 1];
  bool tin_[EC ? EC_TPW : 1];
  if constexpr (EC) {
    const int TR = qxp / 16, ntile = TR * (TR + 1) / 2;
#pragma unroll
    for (int h = 0; h < EC_TPW; ++h) {
      const int t = (threadIdx.x >> 6) + (LBLK / 64) * h;
      tin_[h] = t < ntile;
      int X = 0;
      while ((X + 1) * (X + 2) / 2 <= t) ++X;
      r0_[h] = 16 * X;
      c0_[h] = 16 * (t - X * (X + 1) / 2);
    }
  }
  // EC: the ECORR parameters XB, a_e and the epochs' likelihood terms (ecs) were made for
  __shared__ double eck[NBMAX];
  __shared__ double ecs[3];
  __shared__ double red3[EC ? 12 : 1];
  __shared__ int ecvalid;
  if (EC && threadIdx.x == 0) ecvalid = 0;
  __shared__ double red[4];
  __shared__ double mhv[NHYPER][4];
  __shared__ double bc[4];
  __shared__ double hst[3];            // BIG: the factorisation's sum log a_kk, quad, failure
  const int tid = threadIdx.x;
  double* sc = a.s.sc + (size_t)c * 16;
  // floor pass: only the chains whose b draw runs at the SVD noise floor (SC_FLOOR > 0)
  const double fsh = a.floor_pass ? sc[SC_FLOOR] : 0.0;
  if (a.floor_pass && !(fsh > 0.0)) return;
  const double* Gc = (K0 > 0 ? a.s.G2 : a.s.G) + (size_t)c * mp * mp;
  const Rng rng = make_rng(a, c);
  const double* tp = tape_row(a, c);
  XVec xv;
  load_x(md, a.st, c, xv);
  const double logdetN = sc[SC_LOGDETN], rNr = sc[SC_RNR];
  // (EC: the timing model is factored with the rest, lg_tmelim left these untouched)
  const double ld_tm = EC ? 0.0 : sc[SC_LDTM], quad_tm = EC ? 0.0 : sc[SC_QUADTM];
  const int fail_tm = EC ? 0 : sc[SC_FAILTM] != 0.0;
  const double x_last0 = sc[SC_XLAST];
  int status = fail_tm ? 1 : 0;
  if (!a.eval_only && !a.floor_pass && tid < NHYPER) mh_variate(md, rng, tp, NWHITE + tid, mhv[tid]);

  // factor S0 + diag(phi^-1(q)) in LDS (+ f I in the floor pass); returns the b-marginalised
  // lnL (gibbs.py:288-329)
  auto lnl = [&](const XVec& q, int& failed) -> double {
    const double lA = xget(q, md.idx_logA);
    const double g = xget(q, md.idx_gamma);
    const double lc = 2.0 * lA * 2.302585092994045684 - md.log_12pi2 + (g - 3.0) * md.log_fyr;
    for (int f = tid; f < nf; f += LBLK) {
      if (f < nfr) {
        ph[f] = exp(-(lc - g * md.lfreq[f] + md.ldf[f])) + fsh;
      } else {
        const int b = md.ecb[f - nfr];
        int pi = md.ecorr_b[0];
#pragma unroll
        for (int j = 1; j < NBMAX; ++j) pi = (b == j) ? md.ecorr_b[j] : pi;
        ph[f] = exp(-2.0 * xget(q, pi) * 2.302585092994045684) + fsh;
      }
    }
    double logdet_phi = ((double)nfr * lc - g * md.sum_lfreq + md.sum_ldf) + md.logdet_phi_tm;
    for (int b = 0; b < md.nb; ++b)   // log 10^(2 ecorr_b) per ECORR column of backend b
      if (md.ec_count[b] > 0.0)
        logdet_phi += md.ec_count[b] * (2.0 * xget(q, md.ecorr_b[b]) * 2.302585092994045684);
    __syncthreads();
    double ld = 0.0, quad = 0.0;
    int fl = 0;
    if constexpr (EC) {
      // dense LDL^T of columns [k0, k1) of A, two columns per barrier: the trailing block
      // (rows i, cols j <= i past k + 1: 32 row groups x 8 col groups) takes columns k and
      // k + 1 at once, each thread forming column k + 1's updated entries c_i = A_i,k+1 -
      // A_ik A_k+1,k / a_kk itself; column k + 1 itself is written back in the next round (no
      // thread reads it there).  The trailing block covers every row and column past k1.
      auto wback = [&](double* A, int kd) {   // column kd's update by column kd - 1
        const double s10r = A[kd * SS + kd - 1] * (1.0 / A[(kd - 1) * SS + kd - 1]);
        for (int i = kd + tid; i < qx; i += LBLK) A[i * SS + kd] -= A[i * SS + kd - 1] * s10r;
      };
      auto elim = [&](double* A, int k0, int k1) {
        int kd = -1;
        for (int k = k0; k < k1; k += 2) {
          if (kd >= 0) wback(A, kd);
          if (k + 1 < k1) {
            const double r0 = 1.0 / A[k * SS + k];
            const double s10r = A[(k + 1) * SS + k] * r0;
            const double r1 = 1.0 / (A[(k + 1) * SS + k + 1] - A[(k + 1) * SS + k] * s10r);
            const int i0 = k + 2 + (tid >> 3), j0 = k + 2 + (tid & 7);
            for (int i = i0; i < qx; i += 32) {
              const double sik = A[i * SS + k];
              const double li0 = sik * r0, li1 = (A[i * SS + k + 1] - sik * s10r) * r1;
              for (int j = j0; j <= i; j += 8) {
                const double sjk = A[j * SS + k];
                A[i * SS + j] -= li0 * sjk + li1 * (A[j * SS + k + 1] - sjk * s10r);
              }
            }
            kd = k + 1;
          } else {
            const double r = 1.0 / A[k * SS + k];
            const int i0 = k + 1 + (tid >> 3), j0 = k + 1 + (tid & 7);
            for (int i = i0; i < qx; i += 32) {
              const double lik = A[i * SS + k] * r;
              for (int j = j0; j <= i; j += 8) A[i * SS + j] -= lik * A[j * SS + k];
            }
            kd = -1;
          }
          __syncthreads();
        }
        if (kd >= 0) {
          wback(A, kd);
          __syncthreads();
        }
      };
      // per-thread partial sums of log a_kk, z_k^2 / a_kk and failed pivots over [k0, k1)
      // (a pivot and its augmented-row entry are final once their column is eliminated)
      auto colsums = [&](const double* A, int k0, int k1, double& l, double& qd, double& f) {
        for (int k = k0 + tid; k < k1; k += LBLK) {
          const double akk = A[k * SS + k], zr = A[nxd * SS + k];
          f += !(akk > 0.0) ? 1.0 : 0.0;
          l += log(akk);
          qd += zr * zr * (1.0 / akk);
        }
      };
      // XB = G_xx - sum_e G_xe G_ex / a_e + the timing-model prior, its timing-model columns
      // eliminated: depends on the ECORR parameters only, so it is recomputed only when one
      // changed since the last factorisation (a proposal of log10_A or gamma reuses it and
      // factors the Fourier block alone)
      bool same = ecvalid != 0;
      for (int b = 0; b < md.nb; ++b) same = same && xget(q, md.ecorr_b[b]) == eck[b];
      if (!same) {
        // chunks of EC_ECH epochs: A = (G_ex / a_e)^T, B = G_ex on the MFMA, k = epochs
        const int lane = tid & 63;
        v4d acc[EC_TPW];
#pragma unroll
        for (int h = 0; h < EC_TPW; ++h) acc[h] = v4d{0.0, 0.0, 0.0, 0.0};
        // (two chunk buffers: chunk ch + 1 loads while chunk ch's MFMAs run, one barrier each)
        auto load_chunk = [&](int e0, int bsel) {
          const int ne = nec - e0 < EC_ECH ? nec - e0 : EC_ECH;
          double* E = Ech + bsel * EC_ECH * qxp;
          for (int t = tid; t < EC_ECH * qxp; t += LBLK) {
            const int ee = t / qxp, i = t - ee * qxp;
            E[t] = (ee < ne && i < qx) ? Gl(K0 + nfr + e0 + ee, gx(i)) : 0.0;
          }
          if (tid < EC_ECH) {
            double r = 0.0;
            if (tid < ne) {
              const int ge = K0 + nfr + e0 + tid;
              const double ae = Gg[(size_t)ge * mp + ge] + ph[nfr + e0 + tid];
              aE[e0 + tid] = ae;
              r = 1.0 / ae;
            }
            einv[bsel * EC_ECH + tid] = r;
          }
        };
        const int nch = (nec + EC_ECH - 1) / EC_ECH;
        load_chunk(0, 0);
        __syncthreads();
        for (int ch = 0; ch < nch; ++ch) {
          if (ch + 1 < nch) load_chunk((ch + 1) * EC_ECH, (ch + 1) & 1);
          const double* E = Ech + (ch & 1) * EC_ECH * qxp;
          const double* ei = einv + (ch & 1) * EC_ECH;
#pragma unroll
          for (int h = 0; h < EC_TPW; ++h) {
            if (!tin_[h]) continue;
#pragma unroll
            for (int k4 = 0; k4 < EC_ECH / 4; ++k4) {
              const int kk = 4 * k4 + (lane >> 4);
              const double av = E[kk * qxp + r0_[h] + (lane & 15)] * ei[kk];
              const double bv = E[kk * qxp + c0_[h] + (lane & 15)];
              acc[h] = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, acc[h], 0, 0, 0);
            }
          }
          __syncthreads();
        }
#pragma unroll
        for (int h = 0; h < EC_TPW; ++h) {
          if (!tin_[h]) continue;
#pragma unroll
          for (int g = 0; g < 4; ++g) {
            const int i = r0_[h] + (lane >> 4) + 4 * g, j = c0_[h] + (lane & 15);
            if (i < qx && j <= i) {
              double v = Gg[(size_t)gx(i) * mp + gx(j)] - acc[h][g];
              if (i == j && i < ntm) v = (v + md.tm_phiinv) + fsh;
              XB[i * SS + j] = v;
            }
          }
        }
        __syncthreads();
        elim(XB, 0, ntm);
        // the epochs' and the timing model's pivots and augmented-row terms
        double lde = 0.0, qde = 0.0, fle = 0.0;
        for (int e = tid; e < nec; e += LBLK) {
          const double ae = aE[e];
          const double zr = Gg[(size_t)md.raug * mp + K0 + nfr + e];
          fle += !(ae > 0.0) ? 1.0 : 0.0;
          lde += log(ae);
          qde += zr * zr * (1.0 / ae);
        }
        colsums(XB, 0, ntm, lde, qde, fle);
        block_sum3(lde, qde, fle, red3);
        if (tid == 0) {
          ecs[0] = lde;
          ecs[1] = qde;
          ecs[2] = fle;
          for (int b = 0; b < md.nb; ++b) eck[b] = xget(q, md.ecorr_b[b]);
          ecvalid = 1;
        }
        __syncthreads();
      }
      // X = XB + the Fourier priors; its Fourier block (+ augmented row) factored per likelihood
      for (int t = tid; t < qx * qx; t += LBLK) {
        const int i = t / qx, j = t - i * qx;
        if (j > i) continue;
        double v = XB[i * SS + j];
        if (i == j && i >= ntm && i < nxd) v += ph[i - ntm];
        S[i * SS + j] = v;
      }
      const double lde = ecs[0], qde = ecs[1], fle = ecs[2];
      __syncthreads();
      elim(S, ntm, nxd);
      double ldx = 0.0, qdx = 0.0, flx = 0.0;
      colsums(S, ntm, nxd, ldx, qdx, flx);
      block_sum3(ldx, qdx, flx, red3);
      ld = ldx + lde;
      quad = qdx + qde;
      fl = (flx != 0.0 || fle != 0.0) ? 1 : 0;
    } else if constexpr (BIG) {
      // blocked elimination of the hyper block (+ its augmented row) of S0 + diag(phi^-1):
      // G2 -> G3 (the block and the augmented row are contiguous there, raug = K0 + nf)
      double pmn = INFINITY, pmx = 0.0;
      panel_ldl(Gc, S - ((size_t)K0 * mp + K0), mp, K0, K0 + nf, md.raug, false,
                [&](int gk, double v) { return v + ph[gk - K0]; }, [](int) { return true; }, P,
                ainv, ld, quad, pmn, pmx, fl);
      if (tid == 0) {
        hst[0] = ld;
        hst[1] = quad;
        hst[2] = (double)fl;
      }
      __syncthreads();
      ld = hst[0];
      quad = hst[1];
      fl = hst[2] != 0.0;
      __syncthreads();
    } else {
    for (int e = tid; e < ms * ms; e += LBLK) {
      const int i = e / ms, j = e % ms;
      if (j > i) continue;
      const int gi = (i < nf) ? K0 + i : md.raug, gj = K0 + j;
      double v = Gc[(size_t)gi * mp + gj];
      if (i == j && i < nf) v += ph[i];
      S[i * SS + j] = v;
    }
    __syncthreads();
    for (int k = 0; k < nf; ++k) {
      const double akk = S[k * SS + k];
      const double r = 1.0 / akk;
      const double zr = S[nf * SS + k];
      fl |= !(akk > 0.0) ? 1 : 0;
      ld += log(akk);
      quad += zr * zr * r;
      // rows i in (k, nf], cols j in (k, i]: 32 row groups x 8 column groups
      const int i0 = k + 1 + (tid >> 3), j0 = k + 1 + (tid & 7);
      for (int i = i0; i < ms; i += 32) {
        const double lik = S[i * SS + k] * r;
        for (int j = j0; j <= i; j += 8) S[i * SS + j] -= lik * S[j * SS + k];
      }
      __syncthreads();
    }
    }
    failed = fl | fail_tm;
    if (failed) return -INFINITY;
    double ll = -0.5 * (logdetN + rNr);
    ll += 0.5 * ((quad_tm + quad) - (ld_tm + ld) - logdet_phi);
    return ll;
  };

  const bool run = (a.mask & 6u) || a.eval_only;
  bool redraw = false, Lvalid = false;
  int fb = 0;
  if (run) {
    __syncthreads();
    double l0 = 0.0, p0 = 0.0;
    // the floor pass refactors the final x only (its MH decisions stand)
    const int first = ((a.mask & 2u) || a.eval_only) && !a.floor_pass ? -1 : NHYPER;
    for (int step = first; step <= NHYPER; ++step) {
      XVec q;
      double luacc = 0.0;
      if (step == NHYPER) {
        if (a.eval_only || !(a.mask & 4u)) break;
        redraw = true;
#pragma unroll
        for (int j = 0; j < PMAX; ++j)
          if (j < md.P) redraw = redraw && (xv[j] != x_last0);   // gibbs.py:373
        if (a.mask & 128u) redraw = true;
        if (!redraw || Lvalid) break;
      }
      if (step < 0 || step == NHYPER) {
#pragma unroll
        for (int j = 0; j < PMAX; ++j) q[j] = xv[j];
      } else {
        const int par = (int)mhv[step][0];
#pragma unroll
        for (int j = 0; j < PMAX; ++j) q[j] = (j == par) ? xv[j] + mhv[step][1] : xv[j];
        luacc = mhv[step][2];
      }
      const double p1 = lnpriorP(md, q);
      if (step >= 0 && step < NHYPER && p1 == -INFINITY) continue;
      int f1 = 0;
      const double l1 = lnl(q, f1);
      if (step == NHYPER) {
        fb = f1;
        break;
      }
      if (f1) status |= 1;
      if (step < 0) {
        l0 = l1;
        p0 = p1;
        // a failed initial factorisation is no factor to draw b from: if every proposal
        // is then skipped, step NHYPER refactors (and flags status 2) instead
        Lvalid = !f1;
        if (a.eval_only) {
          if (tid == 0) a.out_h[c] = l1;
          break;
        }
        continue;
      }
      if ((l1 + p1) - (l0 + p0) > luacc) {
#pragma unroll
        for (int j = 0; j < PMAX; ++j) xv[j] = q[j];
        l0 = l1;
        p0 = p1;
        Lvalid = true;
      } else {
        Lvalid = false;
      }
    }
  }
  if (a.eval_only) return;
  // the SVD noise floor (floor_shift): pivots of the real columns, timing model and hyper block
  double fs = 0.0;
  if (!a.floor_pass && redraw && !fb && !(a.st.debug & DEBUG_EXACT_BDRAW)) {
    double mn = INFINITY, mx = 0.0;
    if constexpr (EC) {   // the epochs' pivots, then X's (timing model and Fourier)
      for (int e = tid; e < nec; e += LBLK) {
        mn = fmin(mn, aE[e]);
        mx = fmax(mx, aE[e]);
      }
      for (int k = tid; k < nxd; k += LBLK) {
        mn = fmin(mn, S[k * SS + k]);
        mx = fmax(mx, S[k * SS + k]);
      }
    } else {
      for (int k = tid; k < nf; k += LBLK) {
        mn = fmin(mn, S[k * SS + k]);
        mx = fmax(mx, S[k * SS + k]);
      }
    }
    mx = wave_max(mx);
    mn = -wave_max(-mn);
    if ((tid & 63) == 0) {
      red[tid >> 6] = mx;
      bc[tid >> 6] = mn;
    }
    __syncthreads();
    mx = fmax(fmax(red[0], red[1]), fmax(red[2], red[3]));
    mn = fmin(fmin(bc[0], bc[1]), fmin(bc[2], bc[3]));
    if constexpr (!EC) {   // (the timing model's, from lg_tmelim)
      mx = fmax(mx, sc[SC_TMPMAX]);
      mn = fmin(mn, sc[SC_TMPMIN]);
    }
    fs = floor_of(mn, mx);
    __syncthreads();
  }
  if (tid < md.P) a.st.x[(size_t)c * md.P + tid] = xget(xv, tid);
  if (tid == 0) {
    sc[SC_REDRAW] = redraw ? 1.0 : 0.0;
    sc[SC_FB] = (double)fb;
    if (!a.floor_pass) sc[SC_FLOOR] = fs;
    if (a.st.status)
      a.st.status[c] = (a.st.status[c] | status | ((redraw && fb) ? 2 : 0) |
                        (fs > 0.0 ? STATUS_FLOOR : 0)) +
                       ((fs > 0.0 && !a.floor_pass) ? STATUS_FLOOR_COUNT : 0);
  }
  if (!redraw || fb || fs > 0.0) return;   // fs > 0: the floor pass draws b
  if constexpr (EC) {
    // b draw, all of it: X's columns by back substitution through X's factor, then each
    // epoch e from its pivot and its couplings to X: v_e = (w_e - y_e sum_x G_xe v_x) y_e,
    // w = zraw y + eta as below (Philox normals by internal column)
    if (tp) {
      for (int i = tid; i < mp; i += LBLK) dl[i] = 0.0;
      __syncthreads();
      for (int j = tid; j < md.m; j += LBLK) dl[md.ref2int[j]] = tp[TP_DELTA + j];
      __syncthreads();
    }
    for (int k = tid; k < nxd; k += LBLK) {
      const double yk = rsqrt_nr(S[k * SS + k]);
      if (tp) {
        double s = 0.0;
        for (int i = k; i < nxd; ++i) s += S[i * SS + k] * dl[gx(i)];
        wv_[k] = (S[nxd * SS + k] + s) * yk;
      } else {
        wv_[k] = S[nxd * SS + k] * yk + normal_k(rng, (uint32_t)gx(k), TAG_BDRAW);
      }
      vv[k] = 0.0;
    }
    __syncthreads();
    for (int i = nxd - 1; i >= 0; --i) {
      if (tid == 0) {
        const double yi = rsqrt_nr(S[i * SS + i]);
        bc[0] = (wv_[i] - yi * vv[i]) * yi;
      }
      __syncthreads();
      const double vi = bc[0];
      if (tid == 0) vfull[gx(i)] = vi;
      for (int k = tid; k < i; k += LBLK) vv[k] += S[i * SS + k] * vi;
      __syncthreads();
    }
    for (int e = tid; e < nec; e += LBLK) {
      const int ge = K0 + nfr + e;
      const double ae = aE[e], ye = rsqrt_nr(ae);
      double sx = 0.0;
      for (int i = 0; i < nxd; ++i) sx += Gl(gx(i), ge) * vfull[gx(i)];
      const double zr = Gg[(size_t)md.raug * mp + ge];
      double we;
      if (tp) {
        double s = ae * dl[ge];
        for (int i = 0; i < nxd; ++i) s += Gl(gx(i), ge) * dl[gx(i)];
        we = (zr + s) * ye;
      } else {
        we = zr * ye + normal_k(rng, (uint32_t)ge, TAG_BDRAW);
      }
      vfull[ge] = (we - ye * sx) * ye;
    }
    __syncthreads();
    for (int j = tid; j < md.m; j += LBLK)
      a.st.b[(size_t)c * md.m + j] = vfull[md.ref2int[j]];
    return;
  }
  // b draw, Fourier block: w_k = zraw_k y_k + eta_k, then L^T v = w (raw columns, pivots on
  // the diagonal, y_k = 1/sqrt(a_kk)); back substitution in axpy form over rows of S
  double* vF = a.s.v + (size_t)c * mp + K0;
  if (tp) {
    for (int i = tid; i < nf; i += LBLK) vv[i] = 0.0;
    __syncthreads();
    for (int j = tid; j < md.m; j += LBLK) {
      const int ii = md.ref2int[j] - K0;
      if (ii >= 0 && ii < nf) vv[ii] = tp[TP_DELTA + j];
    }
    __syncthreads();
    // eta_k = y_k sum_{i >= k} a_ik Delta_i (so that L^-T eta = Delta)
    for (int k = tid; k < nf; k += LBLK) {
      double s = 0.0;
      for (int i = k; i < nf; ++i) s += S[i * SS + k] * vv[i];
      const double yk = rsqrt_nr(S[k * SS + k]);
      wv_[k] = (S[nf * SS + k] + s) * yk;
    }
  } else {
    for (int k = tid; k < nf; k += LBLK)
      wv_[k] = S[nf * SS + k] * rsqrt_nr(S[k * SS + k]) +
               normal_k(rng, (uint32_t)(K0 + k), TAG_BDRAW);
  }
  __syncthreads();
  for (int k = tid; k < nf; k += LBLK) vv[k] = 0.0;   // acc_k = sum_{i>k} a_ik v_i
  __syncthreads();
  for (int i = nf - 1; i >= 0; --i) {
    if (tid == 0) {
      const double yi = rsqrt_nr(S[i * SS + i]);
      bc[0] = (wv_[i] - yi * vv[i]) * yi;
    }
    __syncthreads();
    const double vi = bc[0];
    if (tid == 0) vF[i] = vi;
    for (int k = tid; k < i; k += LBLK) vv[k] += S[i * SS + k] * vi;
    __syncthreads();
  }
  (void)red;
}

// ------------------------------------------------------------------------------------
// hyper, register-resident (hyper blocks of at most 62 / 126 columns, MT = 8 / 16): one wave
// per chain runs lg_hyper's MH with the persistent kernel's elimination (gst_kernel.hpp
// chol_range: 8x8-cyclic register layout, one published column per LDS hand-off) instead of
// an LDS factorisation with a workgroup barrier per column.  Internal order: the nf hyper
// columns, unit-prior dummies up to RA (exact no-ops: zero coupling, pivot 1), the augmented
// row at RA, one zero pad row.  Same variates, MH decisions and outputs (x, status, v's
// Fourier block, the redraw flags) as lg_hyper; the likelihood sums run in the persistent
// kernel's order.  MT = 16 (config 5's 121-row block, the 80-column ECORR models): 272
// registers of factor per lane, so no paired tail (its second column view would spill) and
// two chains per workgroup (S0 is 68 KB of LDS per chain).
// ------------------------------------------------------------------------------------
template <int MT>
struct HR {
  static constexpr int RA = 8 * MT - 2;        // augmented row (the paired tail covers an
                                               // even number of columns from slot KP)
  static constexpr int WPB = MT <= 8 ? 4 : 2;  // chains (waves) per workgroup
  static constexpr int KP = MT <= 8 ? kp_for(1) : MT;
  static constexpr int NCS = (8 * MT + 63) / 64;   // hyper columns per lane (64 sl + lane)
  static constexpr int S0 = 64 * SL(MT, 0);        // S0 [slot][lane]
  static constexpr int LDS = S0 + 8 * MT /*colq*/ + 8 * MT /*junk*/ + 8 * pair_pw(MT) /*colq2*/ +
                             64 * NCS /*phi^-1*/ + 4 * NHYPER /*mhv*/ + 64 * NCS /*rhs*/;
};
constexpr int HR_COLS = HR<8>::RA;        // hyper columns (nf + nec) lg_hyper_reg<8> takes
constexpr int HR_COLS_WIDE = HR<16>::RA;  // ... and lg_hyper_reg<16>
static_assert(HR_COLS == 8 * 8 - 2 && HR_COLS_WIDE == 8 * 16 - 2, "hyper_class thresholds");

template <int MT>
__global__ void __launch_bounds__(64 * HR<MT>::WPB) lg_hyper_reg(const DevModel* __restrict__ mds,
                                                                   LArgs a) {
  using H = HR<MT>;
  constexpr int RA = H::RA, NSL = SL(MT, 0), NCS = H::NCS, WPB = H::WPB;
  __shared__ double smem[WPB][H::LDS];
  const int lane = threadIdx.x & 63;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int c = blockIdx.x * WPB + wv;
  if (c >= a.C) return;
  const DevModel& md = mds[ds_of(a, c)];
  if (hyper_class_of(md, a.hyper_lds) != MT) return;  // another class's chain
  double* S0R = smem[wv];
  double* colq = S0R + H::S0;
  double* junk = colq + 8 * MT;
  double* colq2 = junk + 8 * MT;
  double* ph = colq2 + 8 * pair_pw(MT);
  double* mhv = ph + 64 * NCS;
  double* rhs = mhv + 4 * NHYPER;
  const int p = lane >> 3, q = lane & 7;
  const int nf = md.nf + md.nec, nfr = md.nf, K0 = md.ntm_pad, mp = md.mp;
  double* sc = a.s.sc + (size_t)c * 16;
  // floor pass: only the chains whose b draw runs at the SVD noise floor (SC_FLOOR > 0)
  const double fsh = a.floor_pass ? sc[SC_FLOOR] : 0.0;
  if (a.floor_pass && !(fsh > 0.0)) return;
  const double* Gc = (K0 > 0 ? a.s.G2 : a.s.G) + (size_t)c * mp * mp;
  const Rng rng = make_rng(a, c);
  const double* tp = tape_row(a, c);
  XVec xv;
  load_x(md, a.st, c, xv);
  const double logdetN = sc[SC_LOGDETN], rNr = sc[SC_RNR];
  const double ld_tm = sc[SC_LDTM], quad_tm = sc[SC_QUADTM];
  const int fail_tm = sc[SC_FAILTM] != 0.0;
  const double x_last0 = sc[SC_XLAST];
  int status = fail_tm ? 1 : 0;
  if (!a.eval_only && !a.floor_pass && lane < NHYPER)
    mh_variate(md, rng, tp, NWHITE + lane, mhv + 4 * lane);
  // S0 from the Gram's trailing block (lg_tmelim left the Schur complement there), in the
  // cyclic layout: slot (r, s), lane (p, q) = internal (8r+p, 8s+q); diagonal slots hold the
  // full symmetric 8x8 block
  auto gidx = [&](int i) __attribute__((always_inline)) { return i < nf ? K0 + i : (i == RA ? md.raug : -1); };
#pragma unroll
  for (int r = 0; r < MT; ++r)
#pragma unroll
    for (int s2 = 0; s2 <= r; ++s2) {
      int i = 8 * r + p, j = 8 * s2 + q;
      if (j > i) { const int t = i; i = j; j = t; }
      const int gi = gidx(i), gj = gidx(j);
      double v = (i == j) ? 1.0 : 0.0;
      if (gi >= 0 && gj >= 0) v = Gc[(size_t)gi * mp + gj];
      S0R[64 * SL(r, s2) + lane] = v;
    }
  double L[NSL];
  double apr[2] = {1.0, 1.0}, zr[2] = {0.0, 0.0};
  // factor S0 + diag(phi^-1(q)) in registers; the b-marginalised lnL (gibbs.py:288-329)
  auto lnl = [&](const XVec& xq, int& failed) __attribute__((always_inline)) -> double {
    const double lA = xget(xq, md.idx_logA);
    const double g = xget(xq, md.idx_gamma);
    const double lc = 2.0 * lA * 2.302585092994045684 - md.log_12pi2 + (g - 3.0) * md.log_fyr;
#pragma unroll
    for (int cs = 0; cs < NCS; ++cs) {
      const int jc = 64 * cs + lane;
      double pv = 0.0;                  // phi^-1 of internal column jc (0: none)
      if (jc < nfr) {
        pv = exp(-(lc - g * md.lfreq[jc] + md.ldf[jc])) + fsh;
      } else if (jc < nf) {
        const int b = md.ecb[jc - nfr];
        int pi = md.ecorr_b[0];
#pragma unroll
        for (int j = 1; j < NBMAX; ++j) pi = (b == j) ? md.ecorr_b[j] : pi;
        pv = exp(-2.0 * xget(xq, pi) * 2.302585092994045684) + fsh;
      }
      ph[jc] = pv;
    }
    double logdet_phi = ((double)nfr * lc - g * md.sum_lfreq + md.sum_ldf) + md.logdet_phi_tm;
    for (int b = 0; b < md.nb; ++b)
      if (md.ec_count[b] > 0.0)
        logdet_phi += md.ec_count[b] * (2.0 * xget(xq, md.ecorr_b[b]) * 2.302585092994045684);
    lds_order();
#pragma unroll
    for (int r = 0; r < MT; ++r)
#pragma unroll
      for (int s2 = 0; s2 <= r; ++s2) {
        double v = S0R[64 * SL(r, s2) + lane];
        if (r == s2 && p == q) v += ph[8 * r + p];
        L[SL(r, s2)] = v;
      }
    CholCtx cc{colq, junk, colq2, lane, p, q, RA, 1.0, 0.0, 0, 0, {1.0, 1.0}, {0.0, 0.0}};
    chol_range<MT, 0, RA, H::KP>(L, cc);
    chol_harvest<MT, 0, RA, RA>(L, cc);
    chol_stats<0, RA>(cc);
#pragma unroll
    for (int cs = 0; cs < NCS; ++cs) {
      apr[cs] = cc.apr[cs];
      zr[cs] = cc.zr[cs];
    }
    failed = cc.fail | fail_tm;
    if (failed) return -INFINITY;
    const double ld = log(cc.mant) + (double)cc.expo * 0.693147180559945309417;
    double ll = -0.5 * (logdetN + rNr);
    ll += 0.5 * ((quad_tm + cc.quad) - (ld_tm + ld) - logdet_phi);
    return ll;
  };

  const bool run = (a.mask & 6u) || a.eval_only;
  bool redraw = false, Lvalid = false;
  int fb = 0;
  lds_order();
  if (run) {
    double l0 = 0.0, p0 = 0.0;
    // the floor pass refactors the final x only (its MH decisions stand)
    const int first = ((a.mask & 2u) || a.eval_only) && !a.floor_pass ? -1 : NHYPER;
    for (int step = first; step <= NHYPER; ++step) {
      XVec xq;
      double luacc = 0.0;
      if (step == NHYPER) {
        if (a.eval_only || !(a.mask & 4u)) break;
        redraw = true;
#pragma unroll
        for (int j = 0; j < PMAX; ++j)
          if (j < md.P) redraw = redraw && (xv[j] != x_last0);   // gibbs.py:373
        if (a.mask & 128u) redraw = true;
        if (!redraw || Lvalid) break;
      }
      if (step < 0 || step == NHYPER) {
#pragma unroll
        for (int j = 0; j < PMAX; ++j) xq[j] = xv[j];
      } else {
        const int par = (int)mhv[4 * step + 0];
        const double delta = mhv[4 * step + 1];
#pragma unroll
        for (int j = 0; j < PMAX; ++j) xq[j] = (j == par) ? xv[j] + delta : xv[j];
        luacc = mhv[4 * step + 2];
      }
      const double p1 = lnpriorP(md, xq);
      if (step >= 0 && step < NHYPER && p1 == -INFINITY) continue;
      int f1 = 0;
      const double l1 = lnl(xq, f1);
      if (step == NHYPER) {
        fb = f1;
        break;
      }
      if (f1) status |= 1;
      if (step < 0) {
        l0 = l1;
        p0 = p1;
        Lvalid = !f1;   // see lg_hyper
        if (a.eval_only) {
          if (lane == 0) a.out_h[c] = l1;
          break;
        }
        continue;
      }
      if ((l1 + p1) - (l0 + p0) > luacc) {
#pragma unroll
        for (int j = 0; j < PMAX; ++j) xv[j] = xq[j];
        l0 = l1;
        p0 = p1;
        Lvalid = true;
      } else {
        Lvalid = false;
      }
    }
  }
  if (a.eval_only) return;
  // the SVD noise floor (floor_shift): pivots of the real columns, timing model and hyper block
  double fs = 0.0;
  if (!a.floor_pass && redraw && !fb && !(a.st.debug & DEBUG_EXACT_BDRAW)) {
    double mn, mx;
    const double ap[2] = {apr[0], NCS > 1 ? apr[1] : 1.0};
    pivot_range(ap, lane, 0, 0, nf, mn, mx);
    fs = floor_of(fmin(mn, sc[SC_TMPMIN]), fmax(mx, sc[SC_TMPMAX]));
  }
  if (lane < md.P) a.st.x[(size_t)c * md.P + lane] = xget(xv, lane);
  if (lane == 0) {
    sc[SC_REDRAW] = redraw ? 1.0 : 0.0;
    sc[SC_FB] = (double)fb;
    if (!a.floor_pass) sc[SC_FLOOR] = fs;
    if (a.st.status)
      a.st.status[c] = (a.st.status[c] | status | ((redraw && fb) ? 2 : 0) |
                        (fs > 0.0 ? STATUS_FLOOR : 0)) +
                       ((fs > 0.0 && !a.floor_pass) ? STATUS_FLOOR_COUNT : 0);
  }
  if (!redraw || fb || fs > 0.0) return;   // fs > 0: the floor pass draws b
  // b draw, hyper block (lg_hyper's back substitution): the raw factor goes to the S0 region
  // ([slot][lane]: a_ik at 64 SL(i/8, k/8) + 8 (i%8) + k%8); lane owns columns lane + 64 cs
#pragma unroll
  for (int sl = 0; sl < NSL; ++sl) S0R[64 * sl + lane] = L[sl];
  lds_order();
  auto aik = [&](int i, int k) __attribute__((always_inline)) { return S0R[64 * SL(i >> 3, k >> 3) + 8 * (i & 7) + (k & 7)]; };
  double yk[NCS], w[NCS], acc[NCS];       // acc_k = sum_{i > k} a_ik v_i
#pragma unroll
  for (int cs = 0; cs < NCS; ++cs) {
    const int k = 64 * cs + lane;
    yk[cs] = k < nf ? rsqrt_nr(apr[cs]) : 0.0;   // apr: pivot of column k (chol_harvest)
    w[cs] = 0.0;
    acc[cs] = 0.0;
  }
  if (tp) {
#pragma unroll
    for (int cs = 0; cs < NCS; ++cs) rhs[64 * cs + lane] = 0.0;
    lds_order();
    for (int j = lane; j < md.m; j += 64) {
      const int ii = md.ref2int[j] - K0;
      if (ii >= 0 && ii < nf) rhs[ii] = tp[TP_DELTA + j];
    }
    lds_order();
    // eta_k = y_k sum_{i >= k} a_ik Delta_i (so that L^-T eta = Delta)
#pragma unroll
    for (int cs = 0; cs < NCS; ++cs) {
      const int k = 64 * cs + lane;
      double sacc = 0.0;
      if (k < nf)
        for (int i = k; i < nf; ++i) sacc += aik(i, k) * rhs[i];
      w[cs] = (zr[cs] + sacc) * yk[cs];
    }
  } else {
#pragma unroll
    for (int cs = 0; cs < NCS; ++cs) {
      const int k = 64 * cs + lane;
      if (k < nf) w[cs] = zr[cs] * yk[cs] + normal_k(rng, (uint32_t)(K0 + k), TAG_BDRAW);
    }
  }
  double* vF = a.s.v + (size_t)c * mp + K0;
  for (int i = nf - 1; i >= 0; --i) {
    double ys = yk[0], ws = w[0], as = acc[0];
    if (NCS > 1 && i >= 64) {
      ys = yk[NCS - 1];
      ws = w[NCS - 1];
      as = acc[NCS - 1];
    }
    const double yi = rdlane(ys, i & 63), wi = rdlane(ws, i & 63), ai = rdlane(as, i & 63);
    const double vi = (wi - yi * ai) * yi;
    if (lane == 0) vF[i] = vi;
#pragma unroll
    for (int cs = 0; cs < NCS; ++cs) {
      const int k = 64 * cs + lane;
      if (k < i) acc[cs] += aik(i, k) * vi;
    }
  }
}

// ------------------------------------------------------------------------------------
// hyper class 2, register-resident (lg_hyper_ecr<MT, RA>): the epochs-first elimination of
// lg_hyper<2> (ECORR epochs, then the timing model, then the Fourier block) run by ONE wave
// per chain with the persistent kernel's 8x8-cyclic register elimination, where lg_hyper<2>
// spends a 256-thread workgroup and ~20 barriers per likelihood on a ~35-row block (round 5:
// 72% of an ebig sweep).  X's rows in the register layout (X index = internal column):
//   [TM (ntm) | unit-prior pads to 16 | Fourier (nf) | pads | augmented row at RA | pad]
// Per distinct ECORR value (a proposal of a log10_ecorr, or the first likelihood):
//   L = G_xx (+ the timing-model prior) - sum_e g_e g_e^T / a_e,  a_e = G_ee + phi_e^-1,
// one rank-1 downdate per epoch on the VALU (g_e = G_xe staged through LDS, the lane's rows
// 8r+p and columns 8s+q read as 128-bit loads), then the timing-model columns eliminated and
// the whole factor kept in LDS (F); per likelihood the Fourier block's Schur complement is
// reloaded, phi^-1 added and its columns eliminated (chol_range, paired tail).  log|Sigma| =
// sum log a_e + log|X's pivots|, d^T Sigma^-1 d likewise.  The b draw back-substitutes X's
// factor and then each epoch from its pivot and couplings, with lg_hyper<2>'s Philox normals
// (by internal column): the same elimination order, so the same draws to rounding.
// The kernel is latency-bound, not issue-bound: everything it reads more than once from the
// Gram is fetched once into LDS (each epoch's G_ee, its augmented-row entry and backend:
// nec <= EC_REG_MAX), the coupling rows stream two groups ahead, and the per-lane model data
// every likelihood reads are copied into registers once.
// ------------------------------------------------------------------------------------
constexpr int EC_NEB = 3;                   // 64-epoch blocks (EC_REG_MAX = 64 EC_NEB)
template <int MT, int RA_>
struct HE {
  static constexpr int RA = RA_;                 // augmented row (<= 8 MT - 2)
  static constexpr int ID = MT == 8 ? 2 : 1;     // ec_reg_mt's instance id
  static constexpr int KT = 2;                   // timing-model slot columns (ntm <= 16)
  static constexpr int WPB = MT <= 6 ? 4 : 2;    // chains (waves) per workgroup (he_wpb)
  static constexpr int KP = kp_for(1);
  static constexpr int NSL = SL(MT, 0);
  static constexpr int EG = 4;                   // epochs per staged group
  // F [NSL][64] the factor (TM slots) + the Fourier block's Schur complement / final factor;
  // colq, junk, colq2 (chol_range); gq [EG][8][MT] staged coupling rows; ph [64]; mhv
  // [4 NHYPER]; dx [64] tape Delta by X row; vx [64] the b draw's X solution; the chain's x
  // and the MH proposal [PMAX] each; the cached ECORR values' phi^-1 [NBMAX]; each epoch's
  // G_ee, augmented-row entry and backend [EC_REG_MAX] each (wave-uniform and per-epoch
  // values kept in LDS: in registers they cost the 256-register budget of two chains per
  // SIMD; 20 KB per chain, two 4-chain workgroups per CU)
  static constexpr int LDS = 64 * NSL + 8 * MT + 8 * MT + 8 * pair_pw(MT) + EG * 8 * MT + 64 +
                             4 * NHYPER + 64 + 64 + 2 * PMAX + NBMAX + 3 * 64 * EC_NEB;
};

__host__ __device__ constexpr int he_wpb(int MT) { return MT <= 6 ? 4 : 2; }
template <int MT, int RA_>
__global__ void __launch_bounds__(64 * he_wpb(MT), 2) lg_hyper_ecr(const DevModel* __restrict__ mds,
                                                                      LArgs a) {
  using H = HE<MT, RA_>;
  constexpr int RA = H::RA, NSL = H::NSL, KT = H::KT, WPB = H::WPB, EG = H::EG;
  static_assert(MT % 2 == 0 && 8 * MT <= 64 && RA % 2 == 0 && RA <= 8 * MT - 2,
                "one X row per lane");
  __shared__ double smem[WPB][H::LDS];
  const int lane = threadIdx.x & 63;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int c = blockIdx.x * WPB + wv;
  if (c >= a.C) return;
  const DevModel& md = mds[ds_of(a, c)];
  if (ec_reg_mt_of(md, a.hyper_lds, a.st.debug) != H::ID) return;   // another kernel's chain
  double* F = smem[wv];
  double* colq = F + 64 * NSL;
  double* junk = colq + 8 * MT;
  double* colq2 = junk + 8 * MT;
  double* gq = colq2 + 8 * pair_pw(MT);
  double* ph = gq + EG * 8 * MT;
  double* mhv = ph + 64;
  double* dx = mhv + 4 * NHYPER;
  double* vx = dx + 64;
  double* xs = vx + 64;        // [PMAX] x
  double* xqs = xs + PMAX;     // [PMAX] the proposal being evaluated
  double* phb = xqs + PMAX;    // [NBMAX] phi^-1 (+ f) per backend of the cached elimination
  double* ege = phb + NBMAX;   // [EC_REG_MAX] G_ee of epoch e
  double* ezr = ege + 64 * EC_NEB;   // [EC_REG_MAX] z_e = G_{r,e}
  double* ebd = ezr + 64 * EC_NEB;   // [EC_REG_MAX] the epoch's backend
  const int p = lane >> 3, q = lane & 7;
  const int nfr = md.nf, nec = md.nec, ntm = md.ntm, K0 = md.ntm_pad, mp = md.mp, P = md.P;
  double* sc = a.s.sc + (size_t)c * 16;
  const double fsh = a.floor_pass ? sc[SC_FLOOR] : 0.0;
  if (a.floor_pass && !(fsh > 0.0)) return;
  const GDouble* Gg = (const GDouble*)(a.s.G + (size_t)c * mp * mp);   // the raw Gram
  const Rng rng = make_rng(a, c);
  const double* tp = tape_row(a, c);
  if (lane < PMAX) xs[lane] = lane < P ? a.st.x[(size_t)c * P + lane] : 0.0;
  const double logdetN = sc[SC_LOGDETN], rNr = sc[SC_RNR];
  const double x_last0 = sc[SC_XLAST];
  int status = 0;
  if (!a.eval_only && !a.floor_pass && lane < NHYPER)
    mh_variate(md, rng, tp, NWHITE + lane, mhv + 4 * lane);
  // internal column of X row i (-1: a unit-prior pad); X rows are internal columns (K0 = 16)
  auto gxi = [&](int i) __attribute__((always_inline)) {
    return (i < ntm || (i >= 16 && i < 16 + nfr)) ? i : (i == RA ? md.raug : -1);
  };
  const int gl = gxi(lane);   // this lane's X row (epoch downdates, b draw)
  const int raug = md.raug, nb = md.nb;
  // per-lane copies of what every likelihood reads (a global load inside the MH loop is a full
  // memory latency per likelihood, and the scalar ones share lgkmcnt with the LDS traffic):
  // lane 16 + f: log f, log df of Fourier column f; lane b < nb: backend b's ecorr index and
  // epoch count, and the ECORR value of the cached elimination
  const int fl_ = lane - 16;
  const double lf_l = (fl_ >= 0 && fl_ < nfr) ? md.lfreq[fl_] : 0.0;
  const double ldf_l = (fl_ >= 0 && fl_ < nfr) ? md.ldf[fl_] : 0.0;
  const int pib = lane < nb ? md.ecorr_b[lane] : -1;
  const double ecc = lane < nb ? md.ec_count[lane] : 0.0;
  const int iA = md.idx_logA, iG = md.idx_gamma;
  // epochs e: G_ee, the augmented-row entry z_e = G_{r,e} and the backend
#pragma unroll
  for (int k = 0; k < EC_NEB; ++k) {
    const int e = 64 * k + lane, ge = K0 + nfr + e;
    const bool v = e < nec;
    ege[e] = v ? Gg[(size_t)ge * mp + ge] : 1.0;
    ezr[e] = v ? Gg[(size_t)raug * mp + ge] : 0.0;
    ebd[e] = v ? (double)md.ecb[e] : 0.0;
  }
  double L[NSL];
  // cache of the last ECORR values' elimination (wave-uniform) and the TM columns' harvest
  bool ecvalid = false;
  double lde = 0.0, qde = 0.0, aemin = INFINITY, aemax = 0.0, tm_ld = 0.0, tm_quad = 0.0;
  int fle = 0, tm_fail = 0;
  double tm_apr = 1.0, tm_zr = 0.0, f_apr = 1.0, f_zr = 0.0;   // lane k: column k's pivot, aug
  double eck_l = 0.0;
  lds_order();

  // the b-marginalised lnL (gibbs.py:288-329) at the proposal in xqs
  auto lnl = [&](int& failed) __attribute__((always_inline)) -> double {
    const double lA = xqs[iA];
    const double g = xqs[iG];
    const double lc = 2.0 * lA * 2.302585092994045684 - md.log_12pi2 + (g - 3.0) * md.log_fyr;
    ph[lane] = (fl_ >= 0 && fl_ < nfr) ? exp(-(lc - g * lf_l + ldf_l)) + fsh : 0.0;
    double logdet_phi = ((double)nfr * lc - g * md.sum_lfreq + md.sum_ldf) + md.logdet_phi_tm;
    const double xb = pib >= 0 ? xqs[pib] : 0.0;   // lane b: backend b's log10_ecorr
    const double tb_ = ecc > 0.0 ? ecc * (2.0 * xb * 2.302585092994045684) : 0.0;
#pragma unroll
    for (int b = 0; b < NBMAX; ++b)   // backend by backend, as lg_hyper<2>
      if (b < nb) logdet_phi += rdlane(tb_, b);
    const bool same = ecvalid && __ballot(pib >= 0 && xb != eck_l) == 0ull;
    CholCtx cc{colq, junk, colq2, lane, p, q, RA, 1.0, 0.0, 0, 0, {1.0, 1.0}, {0.0, 0.0}};
    if (!same) {
      if (lane < NBMAX) phb[lane] = pib >= 0 ? exp(-2.0 * xb * 2.302585092994045684) + fsh : 0.0;
      eck_l = xb;
      // the epochs' coupling rows g_e (lane = X row), two groups of EG in flight
      const int rr = lane >> 3, pp = lane & 7;   // this lane's X row 8 rr + pp
      const int e_end = K0 + nfr + nec;
      auto gload = [&](int ge) __attribute__((always_inline)) -> double {
        if (ge >= e_end || gl < 0) return 0.0;
        return gl == raug ? Gg[(size_t)raug * mp + ge] : Gg[(size_t)ge * mp + gl];
      };
      double gn[EG], gn2[EG];
#pragma unroll
      for (int u = 0; u < EG; ++u) {
        gn[u] = gload(K0 + nfr + u);
        gn2[u] = gload(K0 + nfr + EG + u);
      }
      lds_order();
      // a_e = G_ee + phi^-1 of its backend, 1 / a_e, and the epochs' likelihood terms
      double yek[EC_NEB];
      {
        double l_ = 0.0, q_ = 0.0, mn = INFINITY, mx = 0.0;
        int f_ = 0;
#pragma unroll
        for (int k = 0; k < EC_NEB; ++k) {
          const int e = 64 * k + lane;
          const bool v = e < nec;
          const double ae = ege[e] + phb[(int)ebd[e]];
          yek[k] = v ? 1.0 / ae : 0.0;
          if (v) {
            const double zr = ezr[e];
            f_ |= !(ae > 0.0) ? 1 : 0;
            l_ += log(ae);
            q_ += zr * zr * (1.0 / ae);
            mn = fmin(mn, ae);
            mx = fmax(mx, ae);
          }
        }
        lde = wave_sum(l_);
        qde = wave_sum(q_);
        fle = __ballot(f_) != 0ull ? 1 : 0;
        aemin = -wave_max(-mn);
        aemax = wave_max(mx);
      }
      // L = -sum_e g_e g_e^T / a_e: 64 epochs per block (1 / a_e by readlane), EG per group,
      // g_e staged in LDS as [p][r] (the lane's rows 8r+p and columns 8s+q contiguous)
#pragma unroll
      for (int sl = 0; sl < NSL; ++sl) L[sl] = 0.0;
#pragma unroll
      for (int k = 0; k < EC_NEB; ++k) {
        const int eb = 64 * k;
        if (eb >= nec) break;
        const int ne = nec - eb < 64 ? nec - eb : 64;
#pragma unroll 1
        for (int u0 = 0; u0 < ne; u0 += EG) {
          double gcur[EG];
#pragma unroll
          for (int u = 0; u < EG; ++u) {
            gcur[u] = gn[u];
            gn[u] = gn2[u];
          }
          const int gnext = K0 + nfr + eb + u0 + 2 * EG;   // (rows past this block: the next)
#pragma unroll
          for (int u = 0; u < EG; ++u) gn2[u] = gload(gnext + u);
          lds_order();   // the previous group's reads precede these stores
#pragma unroll
          for (int u = 0; u < EG; ++u)
            if (rr < MT) gq[u * 8 * MT + pp * MT + rr] = gcur[u];
          lds_order();
#pragma unroll
          for (int u = 0; u < EG; ++u) {
            if (u0 + u >= ne) break;
            typedef double v2_t __attribute__((ext_vector_type(2)));
            double gr[MT], gc[MT];
            const double* bp = gq + u * 8 * MT + p * MT;
            const double* bq = gq + u * 8 * MT + q * MT;
#pragma unroll
            for (int r = 0; r < MT; r += 2) {
              const v2_t x0 = *(const v2_t*)(bp + r), x1 = *(const v2_t*)(bq + r);
              gr[r] = x0[0];
              gr[r + 1] = x0[1];
              gc[r] = x1[0];
              gc[r + 1] = x1[1];
            }
            const double ye = rdlane(yek[k], u0 + u);
#pragma unroll
            for (int r = 0; r < MT; ++r) {
              const double t = gr[r] * ye;
#pragma unroll
              for (int s2 = 0; s2 <= r; ++s2) L[SL(r, s2)] = fma(-t, gc[s2], L[SL(r, s2)]);
            }
          }
        }
      }
      // + G_xx at the lane's slots and the timing-model prior (unit pads)
#pragma unroll
      for (int r = 0; r < MT; ++r)
#pragma unroll
        for (int s2 = 0; s2 <= r; ++s2) {
          int i = 8 * r + p, j = 8 * s2 + q;
          if (j > i) { const int t = i; i = j; j = t; }
          const int gi = gxi(i), gj = gxi(j);
          double v = (gi >= 0 && gj >= 0) ? Gg[(size_t)gi * mp + gj] : (i == j ? 1.0 : 0.0);
          if (i == j && i < ntm) v = (v + md.tm_phiinv) + fsh;
          L[SL(r, s2)] = v + L[SL(r, s2)];
        }
      // the timing-model columns, kept with the epochs' elimination
      chol_range<MT, 0, 16, H::KP>(L, cc);
      chol_harvest<MT, 0, 16, RA>(L, cc);
      chol_stats<0, 16>(cc);
      tm_ld = log(cc.mant) + (double)cc.expo * 0.693147180559945309417;
      tm_quad = cc.quad;
      tm_fail = cc.fail;
      tm_apr = cc.apr[0];
      tm_zr = cc.zr[0];
#pragma unroll
      for (int sl = 0; sl < NSL; ++sl) F[64 * sl + lane] = L[sl];
      ecvalid = true;
      cc = CholCtx{colq, junk, colq2, lane, p, q, RA, 1.0, 0.0, 0, 0, {1.0, 1.0}, {0.0, 0.0}};
    } else {
#pragma unroll
      for (int r = KT; r < MT; ++r)
#pragma unroll
        for (int s2 = KT; s2 <= r; ++s2) L[SL(r, s2)] = F[64 * SL(r, s2) + lane];
    }
    lds_order();
    // + the Fourier priors on the diagonal, then the Fourier block's columns
#pragma unroll
    for (int r = KT; r < MT; ++r)
      if (p == q) L[SL(r, r)] += ph[8 * r + p];
    chol_range<MT, KT, RA, H::KP>(L, cc);
    chol_harvest<MT, 16, RA, RA>(L, cc);
    chol_stats<16, RA>(cc);
    f_apr = cc.apr[0];
    f_zr = cc.zr[0];
    failed = (cc.fail | tm_fail | fle) != 0;
    if (failed) return -INFINITY;
    const double ld = log(cc.mant) + (double)cc.expo * 0.693147180559945309417;
    double ll = -0.5 * (logdetN + rNr);
    ll += 0.5 * ((tm_quad + qde + cc.quad) - (tm_ld + lde + ld) - logdet_phi);
    return ll;
  };
  // the proposal in xqs within the prior box (lnprior, gibbs.py:337-339)
  const double pmin_l = lane < P ? md.pmin[lane] : 0.0, pmax_l = lane < P ? md.pmax[lane] : 0.0;
  auto in_prior = [&]() __attribute__((always_inline)) {
    const bool out = lane < P && !(xqs[lane] >= pmin_l && xqs[lane] <= pmax_l);
    return __ballot(out) == 0ull;
  };

  const bool run = (a.mask & 6u) || a.eval_only;
  bool redraw = false, Lvalid = false;
  int fb = 0;
  if (run) {
    double l0 = 0.0, p0 = 0.0;
    // the floor pass refactors the final x only (its MH decisions stand)
    const int first = ((a.mask & 2u) || a.eval_only) && !a.floor_pass ? -1 : NHYPER;
    for (int step = first; step <= NHYPER; ++step) {
      double luacc = 0.0;
      if (step == NHYPER) {
        if (a.eval_only || !(a.mask & 4u)) break;
        // gibbs.py:373: every element of x differs from the sweep's starting last parameter
        redraw = __ballot(lane < P && xs[lane] == x_last0) == 0ull;
        if (a.mask & 128u) redraw = true;
        if (!redraw || Lvalid) break;
      }
      lds_order();
      if (step < 0 || step == NHYPER) {
        if (lane < PMAX) xqs[lane] = xs[lane];
      } else {
        const int par = (int)mhv[4 * step + 0];
        const double delta = mhv[4 * step + 1];
        if (lane < PMAX) xqs[lane] = (lane == par) ? xs[lane] + delta : xs[lane];
        luacc = mhv[4 * step + 2];
      }
      lds_order();
      const double p1 = in_prior() ? md.lp_sum : -INFINITY;
      if (step >= 0 && step < NHYPER && p1 == -INFINITY) continue;
      int f1 = 0;
      const double l1 = lnl(f1);
      if (step == NHYPER) {
        fb = f1;
        break;
      }
      if (f1) status |= 1;
      if (step < 0) {
        l0 = l1;
        p0 = p1;
        Lvalid = !f1;   // see lg_hyper
        if (a.eval_only) {
          if (lane == 0) a.out_h[c] = l1;
          break;
        }
        continue;
      }
      if ((l1 + p1) - (l0 + p0) > luacc) {
        if (lane < PMAX) xs[lane] = xqs[lane];
        l0 = l1;
        p0 = p1;
        Lvalid = true;
      } else {
        Lvalid = false;
      }
    }
  }
  if (a.eval_only) return;
  lds_order();
  // the SVD noise floor (floor_shift): the epochs' pivots, then X's real columns (timing
  // model, Fourier), as lg_hyper<2>
  double fs = 0.0;
  const double apx = lane < 16 ? tm_apr : f_apr;   // pivot of X column `lane`
  const double zrx = lane < 16 ? tm_zr : f_zr;
  if (!a.floor_pass && redraw && !fb && !(a.st.debug & DEBUG_EXACT_BDRAW)) {
    double mn, mx;
    const double ap[2] = {apx, 1.0};
    pivot_range(ap, lane, ntm, 16, 16 + nfr, mn, mx);
    fs = floor_of(fmin(mn, aemin), fmax(mx, aemax));
  }
  if (lane < P) a.st.x[(size_t)c * P + lane] = xs[lane];
  if (lane == 0) {
    sc[SC_REDRAW] = redraw ? 1.0 : 0.0;
    sc[SC_FB] = (double)fb;
    if (!a.floor_pass) sc[SC_FLOOR] = fs;
    if (a.st.status)
      a.st.status[c] = (a.st.status[c] | status | ((redraw && fb) ? 2 : 0) |
                        (fs > 0.0 ? STATUS_FLOOR : 0)) +
                       ((fs > 0.0 && !a.floor_pass) ? STATUS_FLOOR_COUNT : 0);
  }
  if (!redraw || fb || fs > 0.0) return;   // fs > 0: the floor pass draws b
  // b draw: X's factor -- the timing-model slots in F since the last ECORR elimination (the
  // ECORR values of x), the Fourier block's from the registers -- then the epochs.  Reference
  // order [Fourier | TM | ECORR]: X row i < ntm is b[nf + i], row 16 + f is b[f].
#pragma unroll
  for (int r = KT; r < MT; ++r)
#pragma unroll
    for (int s2 = KT; s2 <= r; ++s2) F[64 * SL(r, s2) + lane] = L[SL(r, s2)];
  const int refx = lane < ntm ? nfr + lane : ((lane >= 16 && lane < 16 + nfr) ? lane - 16 : -1);
  if (tp) dx[lane] = refx >= 0 ? tp[TP_DELTA + refx] : 0.0;
  lds_order();
  auto aik = [&](int i, int k) __attribute__((always_inline)) {
    return F[64 * SL(i >> 3, k >> 3) + 8 * (i & 7) + (k & 7)];
  };
  const bool real = refx >= 0;
  const double yk = real ? rsqrt_nr(apx) : 0.0;
  double w = 0.0;
  if (real) {
    if (tp) {
      // eta_k = y_k sum_{i >= k} a_ik Delta_i (so that L^-T eta = Delta)
      double s = 0.0;
      for (int i = lane; i < RA; ++i) s += aik(i, lane) * dx[i];
      w = (zrx + s) * yk;
    } else {
      w = zrx * yk + normal_k(rng, (uint32_t)lane, TAG_BDRAW);   // X row = internal column
    }
  }
  double acc = 0.0;   // acc_k = sum_{i > k} a_ik v_i
  double* brow = a.st.b + (size_t)c * md.m;
  for (int i = RA - 1; i >= 0; --i) {
    const double yi = rdlane(yk, i), wi = rdlane(w, i), ai = rdlane(acc, i);
    const double vi = (wi - yi * ai) * yi;
    if (lane == 0) vx[i] = vi;
    if (lane < i) acc += aik(i, lane) * vi;
  }
  lds_order();
  if (refx >= 0) brow[refx] = vx[lane];
  // the epochs: v_e = (w_e - y_e sum_x G_xe v_x) y_e, w_e = z_e y_e + eta_e.  A lane's epoch
  // row G_e,[0, RA) is read with every load issued before the first use (a loop of dependent
  // load -> FMA steps cost a memory latency per X row); pad rows carry v = 0 (and zero or
  // another epoch's exact-zero coupling), so the sum over all RA rows in row order is the sum
  // over the real ones
#pragma unroll
  for (int k = 0; k < EC_NEB; ++k) {
    const int e = 64 * k + lane;
    if (e >= nec) continue;
    const int ge = K0 + nfr + e;
    const double ae = ege[e] + phb[(int)ebd[e]], ye = rsqrt_nr(ae);
    const double zr = ezr[e];
    typedef double v2_t __attribute__((ext_vector_type(2)));
    const __attribute__((address_space(1))) v2_t* grow =
        (const __attribute__((address_space(1))) v2_t*)(Gg + (size_t)ge * mp);
    double gx_[RA];
#pragma unroll
    for (int i = 0; i < RA; i += 2) {
      const v2_t v = grow[i / 2];
      gx_[i] = v[0];
      gx_[i + 1] = v[1];
    }
    double sx = 0.0;
#pragma unroll
    for (int i = 0; i < RA; ++i) sx += gx_[i] * vx[i];
    double we;
    if (tp) {
      double s = ae * tp[TP_DELTA + nfr + ntm + e];
#pragma unroll
      for (int i = 0; i < RA; ++i) s += gx_[i] * dx[i];
      we = (zr + s) * ye;
    } else {
      we = zr * ye + normal_k(rng, (uint32_t)ge, TAG_BDRAW);
    }
    brow[nfr + ntm + e] = (we - ye * sx) * ye;
  }
}

// ------------------------------------------------------------------------------------
// btm: b draw's timing-model block, L^T v = w over columns [0, K0) with rows up to raug
// ------------------------------------------------------------------------------------
__global__ void __launch_bounds__(LBLK) lg_btm(const DevModel* __restrict__ mds, LArgs a) {
  const int c = blockIdx.x;
  const DevModel& md = mds[ds_of(a, c)];
  extern __shared__ double lsm[];
  const int K0 = md.ntm_pad, mp = md.mp, raug = md.raug;
  double* acc = lsm;          // [K0]
  double* wk = acc + K0;      // [K0]
  double* vt = wk + K0;       // [K0] solution, timing-model block
  double* dl = vt + K0;       // [raug] Delta (tape mode)
  __shared__ double bc[2];
  const int tid = threadIdx.x;
  const double* sc = a.s.sc + (size_t)c * 16;
  if (sc[SC_REDRAW] == 0.0 || sc[SC_FB] != 0.0) return;
  if (hyper_class_of(md, a.hyper_lds) == 2) return;   // lg_hyper<2> drew all of b
  const double* Gc = a.s.G2 + (size_t)c * mp * mp;   // lg_tmelim's factor (K0 > 0 here)
  double* v = a.s.v + (size_t)c * mp;
  const Rng rng = make_rng(a, c);
  const double* tp = tape_row(a, c);
  // acc_k = sum over Fourier rows i of a_ik v_i  (rows of G contiguous in k)
  for (int k = tid; k < K0; k += LBLK) {
    double s = 0.0;
    for (int i = K0; i < raug; ++i) s += Gc[(size_t)i * mp + k] * v[i];
    acc[k] = s;
  }
  if (tp) {
    for (int i = tid; i < raug; i += LBLK) dl[i] = 0.0;
    __syncthreads();
    for (int j = tid; j < md.m; j += LBLK) dl[md.ref2int[j]] = tp[TP_DELTA + j];
    __syncthreads();
    for (int k = tid; k < K0; k += LBLK) {
      double s = 0.0;
      for (int i = k; i < raug; ++i) s += Gc[(size_t)i * mp + k] * dl[i];
      const double yk = rsqrt_nr(Gc[(size_t)k * mp + k]);
      wk[k] = (Gc[(size_t)raug * mp + k] + s) * yk;
    }
  } else {
    for (int k = tid; k < K0; k += LBLK)
      wk[k] = Gc[(size_t)raug * mp + k] * rsqrt_nr(Gc[(size_t)k * mp + k]) +
              normal_k(rng, (uint32_t)k, TAG_BDRAW);
  }
  __syncthreads();
  for (int i = K0 - 1; i >= 0; --i) {
    if (tid == 0) {
      const double yi = rsqrt_nr(Gc[(size_t)i * mp + i]);
      bc[0] = (wk[i] - yi * acc[i]) * yi;
    }
    __syncthreads();
    const double vi = bc[0];
    if (tid == 0) vt[i] = vi;
    const double* row = Gc + (size_t)i * mp;
    for (int k = tid; k < i; k += LBLK) acc[k] += row[k] * vi;
    __syncthreads();
  }
  // b in reference order (Fourier part from lg_hyper in v, timing-model part in vt)
  for (int j = tid; j < md.m; j += LBLK) {
    const int ii = md.ref2int[j];
    a.st.b[(size_t)c * md.m + j] = ii < K0 ? vt[ii] : v[ii];
  }
}

// ------------------------------------------------------------------------------------
// tb: y = r - T b for every chain (gibbs.py:213,237,272) as one MFMA GEMM
// ------------------------------------------------------------------------------------
// Wave: CG groups of 16 chains x 64 TOAs (4 tiles); A = b (chains x basis), B = T^T (basis x
// TOAs) read from the column-major Tcol so a wave's B fragment is 16 consecutive TOAs.  The
// groups of a wave share the B fragments (CG x 4 MFMAs per CG + 4 loads), with TB_DEPTH
// k-steps of operands in flight.  Every y element receives the same MFMA sequence (k in
// order, the same A / B values) whatever CG is, so y is bitwise that of one group per wave.
constexpr int TB_CG = 4;      // 16-chain groups per wave (chains per wave: 64)
#ifndef GST_TB_DEPTH
#define GST_TB_DEPTH 2   // (3: measured no faster on config 5, round 6)
#endif
constexpr int TB_DEPTH = GST_TB_DEPTH;   // k-steps of operands in flight
template <int CG>
__device__ __forceinline__ void tb_tile(const DevModel& md, const LArgs& a, int t0, int cb) {
  const int lane = threadIdx.x & 63;
  const int m = md.m, npad = md.npad;
  if (t0 >= npad) return;                         // beyond this dataset's TOAs
  const int kl = lane >> 4;
  const double* bc[CG];
  bool cok[CG];
#pragma unroll
  for (int g = 0; g < CG; ++g) {
    const int ci = cb + 16 * g + (lane & 15);
    cok[g] = ci < a.C;
    bc[g] = a.st.b + (size_t)(cok[g] ? ci : cb) * m;
  }
  v4d acc[CG][4];
#pragma unroll
  for (int g = 0; g < CG; ++g)
#pragma unroll
    for (int u = 0; u < 4; ++u) acc[g][u] = (v4d){0.0, 0.0, 0.0, 0.0};
  constexpr int D = TB_DEPTH;
  double av[D][CG], bv[D][4];
  auto load = [&](int d, int k) __attribute__((always_inline)) {
    const int j = k + kl;
    const bool jok = j < m;
    const double* tc = md.Tcol + (size_t)(jok ? j : 0) * npad + t0 + (lane & 15);
#pragma unroll
    for (int g = 0; g < CG; ++g) av[d][g] = (cok[g] && jok) ? bc[g][jok ? j : 0] : 0.0;
#pragma unroll
    for (int u = 0; u < 4; ++u) bv[d][u] = jok ? tc[16 * u] : 0.0;
  };
  auto kstep = [&](int d) __attribute__((always_inline)) {
#pragma unroll
    for (int g = 0; g < CG; ++g)
#pragma unroll
      for (int u = 0; u < 4; ++u)
        acc[g][u] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[d][g], bv[d][u], acc[g][u], 0, 0, 0);
  };
  const int nks = (m + 3) / 4;                    // k-steps (the last one zero-padded)
#pragma unroll
  for (int d = 0; d < D; ++d) load(d, 4 * d);
  int ks = 0;
  for (; ks + D < nks; ks += D) {
#pragma unroll
    for (int d = 0; d < D; ++d) {
      kstep(d);
      load(d, 4 * (ks + d + D));
      __builtin_amdgcn_sched_barrier(0);
    }
  }
#pragma unroll
  for (int d = 0; d < D; ++d)
    if (ks + d < nks) kstep(d);
#pragma unroll
  for (int g = 0; g < CG; ++g)
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int cc = cb + 16 * g + kl + 4 * q;
        const int t = t0 + 16 * u + (lane & 15);
        if (cc < a.C && t < npad)
          a.s.y[(size_t)cc * a.ys + t] = (t < md.n) ? md.resid[t] - acc[g][u][q] : 0.0;
      }
}

__global__ void __launch_bounds__(LBLK) lg_tb(const DevModel* __restrict__ mds, LArgs a) {
  const int wv = threadIdx.x >> 6;
  const int t0 = blockIdx.x * 64;
  const int cw = (blockIdx.y * 4 + wv) * 16 * TB_CG;   // the wave's first chain
  if (cw >= a.C) return;
  // one dataset per 16-chain group (native.py checks it); the groups share T's fragments
  // when they share the dataset, otherwise each group runs on its own
  const int d0 = ds_of(a, cw);
  bool same = true;
#pragma unroll
  for (int g = 1; g < TB_CG; ++g)
    if (cw + 16 * g < a.C && ds_of(a, cw + 16 * g) != d0) same = false;
  if (same) {
    tb_tile<TB_CG>(mds[d0], a, t0, cw);
  } else {
    for (int g = 0; g < TB_CG; ++g)
      if (cw + 16 * g < a.C) tb_tile<1>(mds[ds_of(a, cw + 16 * g)], a, t0, cw + 16 * g);
  }
}

// ------------------------------------------------------------------------------------
// toa: theta, z, alpha, nu (gibbs.py:185-259)
// ------------------------------------------------------------------------------------
template <int TB>
__global__ void __launch_bounds__(TB) lg_toa(const DevModel* __restrict__ mds, LArgs a) {
  const int c = blockIdx.x;
  const DevModel& md = mds[ds_of(a, c)];
  if (toa_class(md.npad) != a.kclass) return;     // another class's launch runs this chain
  __shared__ double red[TB / 64];
  __shared__ double dfb[32];
  const int n = md.n, nst = a.st.nst, m = md.m, tid = threadIdx.x;
  double* zc = a.st.z + (size_t)c * nst;
  double* alc = a.st.alpha + (size_t)c * nst;
  double* poc = a.st.pout + (size_t)c * nst;
  const double* yc = a.s.y + (size_t)c * a.ys;
  const Rng rng = make_rng(a, c);
  const double* tp = tape_row(a, c);
  XVec xv;
  load_x(md, a.st, c, xv);
  double theta = a.st.theta[c], nu = a.st.nu[c];
  const WhiteNoise wn = white_noise(md, xv);
  const bool mix = (md.model == 2) || (md.model == 3);
  if ((a.mask & 8u) && mix) {
    double zs = 0.0;
    for (int t = tid; t < n; t += TB) zs += (zc[t] != 0.0) ? 1.0 : 0.0;
    zs = block_sum<TB / 64>(zs, red);
    const double aa = zs + md.mk;
    const double bb = ((double)n - zs) + md.k1mm;
    if (tp) {
      theta = tp[TP_DELTA + m];
    } else {
      const double ga = gamma_mt(aa, rng, 0u, TAG_THETA);
      const double gb = gamma_mt(bb, rng, 1u, TAG_THETA);
      theta = ga / (ga + gb);
    }
  }
  const bool fuse = (a.mask & 16u) && mix && (a.mask & 32u) && md.vary_alpha;
  const bool fuse_nu = fuse && (a.mask & 64u) && md.vary_df;
  double zs_new = 0.0, sa_new = 0.0;
  LogProd lp_new;
  if (fuse) {
    // z, alpha and nu's sums in one pass over the TOAs (each thread its own TOAs, in the
    // separate passes' order): alpha is drawn from the new z right away and kept if the new z
    // has an outlier (gibbs.py:234; the old alpha waits in the w scratch row otherwise), so
    // alpha / nu cost no extra passes over z, y, alpha.  Draws and sums are bitwise the
    // separate passes'.
    const double SQ2PI = 2.5066282746310002;  // np.sqrt(2*np.pi)
    double* wc = a.s.w + (size_t)c * a.ys;
    for (int t = tid; t < n; t += TB) {
      const double N0 = wn.n0(t);
      const double al_old = alc[t];
      const double Nv = al_old * N0;
      const double y = yc[t];
      const double sd1 = sqrt(Nv);
      const double x1 = y / sd1;
      double top = theta * (exp(-(x1 * x1) / 2.0) / SQ2PI / sd1);
      if (md.model == 3) top = theta / md.pspin;
      const double sd0 = sqrt(N0);
      const double x0 = y / sd0;
      const double bot = top + (1.0 - theta) * (exp(-(x0 * x0) / 2.0) / SQ2PI / sd0);
      double qz = top / bot;
      if (isnan(qz)) qz = 1.0;
      poc[t] = qz;
      const double pz = qz < 1.0 ? qz : 1.0;
      double u;
      if (tp) {
        u = tp[TP_DELTA + m + 1 + t];
      } else {
        double unused;
        rng.uniform2((uint32_t)t, TAG_Z, u, unused);
      }
      const double zf = (double)bern_legacy(pz, u);
      zc[t] = zf;
      const double atop = ((y * y) * zf / N0 + nu) / 2.0;
      const double G = tp ? tp[TP_DELTA + m + 1 + nst + t]
                          : gamma_mt((zf + nu) / 2.0, rng, (uint32_t)t, TAG_ALPHA);
      const double an = atop / G;
      wc[t] = al_old;
      alc[t] = an;
      zs_new += zf;
      if (fuse_nu) {
        lp_new.mul(an);
        sa_new += 1.0 / an;
      }
    }
    zs_new = block_sum<TB / 64>(zs_new, red);
    if (!(zs_new >= 1.0)) {
      // no outlier flagged: alpha keeps its values (gibbs.py:234,242), nu sums over them
      lp_new = LogProd();
      sa_new = 0.0;
      for (int t = tid; t < n; t += TB) {
        const double ao = wc[t];
        alc[t] = ao;
        lp_new.mul(ao);
        sa_new += 1.0 / ao;
      }
    }
  }
  if ((a.mask & 16u) && mix && !fuse) {
    const double SQ2PI = 2.5066282746310002;  // np.sqrt(2*np.pi)
    for (int t = tid; t < n; t += TB) {
      const double N0 = wn.n0(t);
      const double Nv = alc[t] * N0;
      const double y = yc[t];
      const double sd1 = sqrt(Nv);
      const double x1 = y / sd1;
      double top = theta * (exp(-(x1 * x1) / 2.0) / SQ2PI / sd1);
      if (md.model == 3) top = theta / md.pspin;
      const double sd0 = sqrt(N0);
      const double x0 = y / sd0;
      const double bot = top + (1.0 - theta) * (exp(-(x0 * x0) / 2.0) / SQ2PI / sd0);
      double qz = top / bot;
      if (isnan(qz)) qz = 1.0;
      poc[t] = qz;
      const double pz = qz < 1.0 ? qz : 1.0;
      double u;
      if (tp) {
        u = tp[TP_DELTA + m + 1 + t];
      } else {
        double unused;
        rng.uniform2((uint32_t)t, TAG_Z, u, unused);
      }
      zc[t] = (double)bern_legacy(pz, u);
    }
  }
  __syncthreads();
  if ((a.mask & 32u) && md.vary_alpha && !fuse) {
    double zs = 0.0;
    for (int t = tid; t < n; t += TB) zs += (zc[t] != 0.0) ? 1.0 : 0.0;
    zs = block_sum<TB / 64>(zs, red);
    if (zs >= 1.0) {
      for (int t = tid; t < n; t += TB) {
        const double zf = zc[t] != 0.0 ? 1.0 : 0.0;
        const double N0 = wn.n0(t);
        const double top = ((yc[t] * yc[t]) * zf / N0 + nu) / 2.0;
        const double G = tp ? tp[TP_DELTA + m + 1 + nst + t]
                            : gamma_mt((zf + nu) / 2.0, rng, (uint32_t)t, TAG_ALPHA);
        alc[t] = top / G;
      }
    }
  }
  __syncthreads();
  if ((a.mask & 64u) && md.vary_df) {
    double sa = sa_new;
    LogProd lp = lp_new;
    if (!fuse_nu) {
      for (int t = tid; t < n; t += TB) {
        lp.mul(alc[t]);
        sa += 1.0 / alc[t];
      }
    }
    const double S = block_sum<TB / 64>(lp.log_sum() + sa, red);
    if (tid < 64) {
      double ll = -INFINITY;
      if (tid < 30) {
        const double h = (double)(tid + 1) / 2.0;
        ll = -h * S + md.dfA[tid] - md.dfB[tid];
      }
      const double mx = wave_max(ll);
      if (tid < 30) dfb[tid] = exp(ll - mx);
    }
    __syncthreads();
    double u;
    if (tp) {
      u = tp[TP_DELTA + m + 1 + 2 * nst];
    } else {
      double unused;
      rng.uniform2(0u, TAG_DF, u, unused);
    }
    double acc8[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) acc8[j] = dfb[j];
#pragma unroll
    for (int i = 8; i < 24; i += 8)
#pragma unroll
      for (int j = 0; j < 8; ++j) acc8[j] += dfb[i + j];
    double tot = ((acc8[0] + acc8[1]) + (acc8[2] + acc8[3])) + ((acc8[4] + acc8[5]) + (acc8[6] + acc8[7]));
#pragma unroll
    for (int i = 24; i < 30; ++i) tot += dfb[i];
    double cdf[30];
    double cs = 0.0;
#pragma unroll
    for (int i = 0; i < 30; ++i) {
      cs += dfb[i] / tot;
      cdf[i] = cs;
    }
    int cnt = 0;
#pragma unroll
    for (int i = 0; i < 30; ++i) cnt += (cdf[i] / cdf[29] <= u) ? 1 : 0;
    cnt = cnt < 29 ? cnt : 29;
    nu = (double)(cnt + 1);
  }
  if (tid == 0) {
    a.st.theta[c] = theta;
    a.st.nu[c] = nu;
  }
}

}  // namespace gst
