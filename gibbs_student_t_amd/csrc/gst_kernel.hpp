// Persistent per-chain Gibbs sweep kernel for gfx950 (MI355X, CDNA4).
//
// One 64-lane wavefront owns one chain for a whole launch of `nsweeps` sweeps of the
// reference sampler (/root/reference/gibbs.py, Gibbs.sample loop gibbs.py:354-380).
// Chains are independent, so waves never synchronise with each other: there is no
// __syncthreads, only in-order same-wave LDS traffic (except in the two-waves-per-chain
// build, PAIR below, whose two waves exchange MH likelihoods once per round).
//
// Matrix layout ("8x8 cyclic"): lane = 8p + q owns elements (8r+p, 8s+q) of the symmetric
// system matrix, r >= s, in registers L[SL(r,s)].  Internal column order is
//     [ timing model (ntm) | pad to 8*K0 | Fourier (nf) | r (augmented row) | pad ]
// so that (i) the timing-model block, whose prior never changes inside a sweep, is
// eliminated once per sweep (its Schur complement S0 is kept in registers) and (ii) the
// residual column rides along as an augmented row whose elimination yields L^-1 d, i.e.
// d^T Sigma^-1 d, for free.  Every MH step of the red-noise hyper block only refactors the
// (nf+1)-row Fourier block S0 + diag(phi^-1).
//
// Stages per sweep (gibbs.py stage order, semantically binding):
//   white MH (20 steps)      gibbs.py:114-143, lnL gibbs.py:262-284
//   Gram T^T N^-1 [T|r]       gibbs.py:302-304  -- fp64 MFMA 16x16x4, T shared by all chains
//   hyper MH (10 steps)      gibbs.py:80-111,  lnL gibbs.py:288-329
//   b draw (quirk :373)       gibbs.py:145-182  -- Cholesky draw mu + L^-T eta
//   theta, z, alpha, nu       gibbs.py:185-259
#pragma once
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include <type_traits>

#include "philox.hpp"

namespace gst {

typedef double v4d __attribute__((ext_vector_type(4)));
// a global-memory double: loads through it are global_load (a generic pointer read out of
// DevModel compiles to flat_load, which also waits on the LDS counter)
typedef __attribute__((address_space(1))) double GDouble;

constexpr int NWHITE = 20;
constexpr int NHYPER = 10;
constexpr int PMAX = 16;   // sampled parameters (large path; the persistent kernel takes <= 4,
                           // its general-white-noise (GEN) instances <= 8)
constexpr int NBMAX = 8;   // backends with their own white-noise / ECORR parameters
__host__ __device__ constexpr int SL(int r, int s) { return r * (r + 1) / 2 + s; }

// Per-chain LDS (doubles), laid out so that two chains fit per SIMD (8 per CU, 20 KB each
// at J1713 sizes):
//   S0R   [64 * SL(MT-K0, 0)]  the Schur complement S0 during the hyper block, [slot][lane];
//                              outside it, scratch of the other stages (white MH variates,
//                              Gram weights + tile transposes, b-draw vectors, nu grid)
//   colq  [8 * MT]             the one published column of the elimination, [p][r]
//   mhh   [4 * NHYPER]         hyper-MH variates of the sweep
//   phbuf [8 * MT]             phi^-1 by internal column
//   colq2 [8 * (MT - KP_MIN)]  the second published column of the paired tail (rows >= KP)
// Slot column KP from which the elimination runs in column pairs (chol_pair): two columns
// per LDS hand-off.  The pair buffers hold rows r >= KP only, at row stride MT - KP (even,
// for 128-bit accesses); LDS is sized for the earliest start, KP_MIN, which keeps the extra
// LDS within two chains per SIMD (8 per CU).  kp_for: the one-chain-per-SIMD builds pair
// from KP_MIN; the 256-register two-chains-per-SIMD build only over its last slot columns
// (pairing earlier spills there, and its second wave already covers much of the hand-off
// latency).
constexpr int KP_MIN = 4;
// gram_and_tm's low-rank Gram takes sweeps with at most LR_MAX flagged TOAs (z = 1): past
// that the n-TOA MFMA Gram is cheaper, and the class Grams' share that cancels grows
constexpr int LR_MAX = 32;
constexpr double LR_ALPHA_MAX = 0x1p20;   // ... and alpha_t <= 2^20 on every flagged TOA
// the largest TOA-slot count whose two-chains-per-SIMD build the host picks (wider shapes
// run one chain per SIMD)
#ifndef GST_OCC2_NS_MAX
#define GST_OCC2_NS_MAX 8   // A/B builds override it (GST_EXTRA_CFLAGS=-DGST_OCC2_NS_MAX=16)
#endif
constexpr int OCC2_NS_MAX = GST_OCC2_NS_MAX;
__host__ __device__ constexpr int pair_pw(int MT) { return MT - KP_MIN; }
#ifndef GST_KP_OCC2
#define GST_KP_OCC2 6   // A/B builds override it (GST_EXTRA_CFLAGS=-DGST_KP_OCC2=...)
#endif
__host__ __device__ constexpr int kp_for(int OCC) { return OCC == 2 ? GST_KP_OCC2 : KP_MIN; }
// index of slot (r, s), s < K0, among the timing-model factor slots (column-major)
__host__ __device__ constexpr int tm_slot(int MT, int r, int s) {
  return s * MT - s * (s - 1) / 2 + (r - s);
}
__host__ __device__ constexpr int s0r_doubles(int MT, int K0) { return 64 * SL(MT - K0, 0); }
__host__ __device__ constexpr int lds_doubles(int MT, int K0) {
  return s0r_doubles(MT, K0) + 8 * MT + 4 * NHYPER + 8 * MT + 8 * pair_pw(MT);
}
// chains (waves) per SIMD the LDS allows with 4-chain workgroups: 2 when two workgroups
// (8 chains) fit a CU's 160 KB
__host__ __device__ constexpr int occ_for(int MT, int K0) {
  return lds_doubles(MT, K0) * 8 * 4 * 2 <= 160 * 1024 ? 2 : 1;
}
// scratch aliases inside S0R (offsets in doubles), each live only while S0 is dead
__host__ __device__ constexpr int s0r_need(int MT, int NS) {
  return (4 * NWHITE > 64 * NS + 16 * 17 ? 4 * NWHITE : 64 * NS + 16 * 17) > 7 * 8 * MT + 64
             ? (4 * NWHITE > 64 * NS + 16 * 17 ? 4 * NWHITE : 64 * NS + 16 * 17)
             : 7 * 8 * MT + 64;
}
struct DevModel {
  const double* Tmf;     // [nks][NT][64]: MFMA-packed augmented T, internal column order
  const double* Tcol;    // [m][npad]: T column-major, reference column order, zero padded
  const double* resid;   // [npad]
  const double* sig2;    // [npad]  toaerrs**2
  const double* lfreq;   // [nf]    log(Ffreqs)
  const double* ldf;     // [nf]    log(repeat(df, 2))
  const double* dfA;     // [32]    n*(nu/2)*log(nu/2)
  const double* dfB;     // [32]    n*gammaln(nu/2)
  const int* ref2int;    // [m]     reference column -> internal index
  const int* cidx;       // [npad]  noise class of each TOA (TOAs with equal sigma), or null
  const double* csig2;   // [ncls]  sigma^2 of each class
  const double* ccount;  // [ncls]  TOAs per class
  int ncls;              // 0 = per-TOA white likelihood; 1..8 = class path
  // persistent kernel, ncls > 0 (else null): per-class Grams of [T|r] in the 8x8-cyclic
  // register layout [ncls][SL(MT,0)][64] and the augmented rows [npad][8 MT] (internal
  // order), for the low-rank Gram (gram_and_tm)
  const double* Gcls;
  const double* Trow;
  int n, m, mp, nf, ntm, ntm_pad, raug, nks, npad, nslot_toa;
  int P;
  int idx_efac, idx_equad, idx_logA, idx_gamma;
  double efac_const;
  double pmin[PMAX], pmax[PMAX], lp_in[PMAX], lp_sum;
  int hind[PMAX], nh, wind[PMAX], nw;
  // general white noise (large path; the persistent kernel's GEN instances):
  // per-backend efac / log10_equad / log10_ecorr parameter indices (-1: constant / none),
  // the backend of every TOA, and the ECORR epoch columns (internal columns
  // ntm_pad + nf .. ntm_pad + nf + nec - 1, between the Fourier block and the residual row)
  int nb;
  int cls_b[8];             // backend of each noise class (classes: equal sigma AND backend)
  const int* bk;            // [npad] backend of each TOA (null when nb == 1)
  int efac_b[NBMAX], equad_b[NBMAX], ecorr_b[NBMAX];
  int nec;
  int ec_disjoint;          // every TOA in at most one ECORR column (the batch's datasets all)
  const int* ecb;           // [nec] backend of each ECORR column
  double ec_count[NBMAX];   // ECORR columns per backend
  // large path, disjoint ECORR epochs (gst_large.hpp lg_gram_ec; gx_nt = 0: not built): the
  // Gram's X part (timing model + Fourier + r + a ones column, gx_nt 16-column tiles) packed
  // as Tmf, and the epochs' TOAs in epoch order, 16 epochs per block, each block padded to
  // whole k-steps of 4: their X rows times the ECORR basis value ([nkse][gx_nt][64]), TOA
  // index and block-local epoch of each entry ([nkse * 4][2], -1 padding), block k-step starts
  const double* Tx;
  const double* Xe;
  const int* ekl;
  const int* eblk;          // [neblk + 1]
  int gx_nt, nkse, neblk;
  double sig_h, sig_w;
  double mh_cdf[5], mh_size[5];
  int model, vary_df, vary_alpha;
  double mk, k1mm, pspin;
  double tm_phiinv, logdet_phi_tm;
  double sum_lfreq, sum_ldf;  // sum_k log f_k, sum_k log df_k (closed-form log|phi|)
  double log_fyr, log_12pi2;
  unsigned long long* stamps;  // diagnostic build only (GST_STAMPS): [C][GST_NSTAMP]
};

struct DevState {
  double *x, *b, *z, *alpha, *pout, *theta, *nu;
  int* status;
  const int* dataset;  // [C] dataset of each chain (null: every chain uses dataset 0)
  int nst;             // row stride of the per-TOA arrays (max n over the datasets)
  int nd;              // number of datasets
  double* tmfac;       // [C][timing-model factor slots][64] scratch (persistent path)
  unsigned long long* prog;  // chain-sweeps started in this launch (two chains per SIMD), or
                             // null: see fair_prio
  int debug;                 // GST_DEBUG_* flags (gst_set_debug)
  unsigned long long* gram_cnt;  // [2] Grams computed: low-rank, MFMA (gst_gram_counts), or null
};
struct DevRec {
  double *x, *b, *z, *alpha, *pout, *theta, *nu;
  int nrec;
};
struct DevTape {
  const double* data;
  int stride;
};

// tape layout offsets (see gst.h)
constexpr int TP_WHITE = 0, TP_HYPER = 80, TP_DELTA = 120;

// The published column: colq[p][r] = row 8r+p of the column being eliminated, r fastest, so
// a lane's row-side (p) and column-side (q) reads are contiguous in r and go as 128-bit LDS
// loads; the 8 owner lanes (q == column residue) write it.  Row stride MT = 10 doubles puts
// the 8 p-rows of a 128-bit read in distinct bank groups (80 B apart).

// diagnostic builds: slots 0-15, 19-23 cycle sums (tools/stage_profile.py), 16-18 event counts
constexpr int GST_NSTAMP = 28;
#ifdef GST_STAMPS
#define GST_STAMP_DECL \
  unsigned long long st_acc[GST_NSTAMP] = {0}, st_t0 = 0, st_s0 = 0;
#define GST_SUB_BEGIN st_s0 = __builtin_amdgcn_s_memtime();
#define GST_COUNT(i) st_acc[i] += 1;
#define GST_SUB_END(i)                                            \
  {                                                               \
    const unsigned long long t1_ = __builtin_amdgcn_s_memtime(); \
    st_acc[i] += t1_ - st_s0;                                     \
    st_s0 = t1_;                                                  \
  }
#define GST_STAMP_START st_t0 = __builtin_amdgcn_s_memtime();
#define GST_STAMP(i)                                              \
  {                                                               \
    const unsigned long long t1_ = __builtin_amdgcn_s_memtime(); \
    st_acc[i] += t1_ - st_t0;                                     \
    st_t0 = t1_;                                                  \
  }
#define GST_STAMP_FLUSH                                             \
  if (md.stamps && lane == 0)                                       \
    for (int i_ = 0; i_ < GST_NSTAMP; ++i_) md.stamps[(size_t)c * GST_NSTAMP + i_] += st_acc[i_];
#else
#define GST_SUB_BEGIN
#define GST_COUNT(i)
#define GST_SUB_END(i)
#define GST_STAMP_DECL
#define GST_STAMP_START
#define GST_STAMP(i)
#define GST_STAMP_FLUSH
#endif

__device__ __forceinline__ double rdlane(double v, int lane) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readlane((int)(b & 0xffffffffll), lane);
  const int hi = __builtin_amdgcn_readlane((int)(b >> 32), lane);
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}

// Two chains share each SIMD in the OCC = 2 build, and the SIMD's arbiter issues the older
// wave first: the chain that arrived second ran ~27% slower per sweep than its partner and
// every launch ended with it (tools/chain_pairs.py).  Priority turns fix that:
//  * progress rule (the host passes st.prog): each chain counts its sweep into a
//    launch-wide counter (one atomic per chain-sweep, its return value consumed a sweep
//    later); a chain that has done fewer sweeps than the launch average holds the higher
//    issue priority;
//  * the first sweep of a launch, and launches without st.prog: time slices of 2^15 clocks
//    by wave-slot parity (slot-parity-1 waves hold the higher priority kPrioShare / 8
//    of the time).
// Checked at the sweep, MH-step and stage boundaries (the clock read waits only there).
constexpr unsigned kPrioShare = 5;  // 4: 8.50 M, 5: 8.65 M, 6: 8.38 M chain-sweeps/s (age favours the older wave)
__device__ __forceinline__ unsigned wave_slot_parity() {
  return __builtin_amdgcn_s_getreg((31 << 11) | (0 << 6) | 4) & 1u;  // HW_REG_HW_ID.WAVE_ID
}
struct Fair {
  unsigned slot;            // wave-slot parity
  int behind;               // progress rule: 1 = behind the launch average, -1 = no rule
};
template <int OCC>
__device__ __forceinline__ void fair_prio(const Fair& f) {
  if constexpr (OCC == 2) {
    bool high;
    if (f.behind >= 0) {
      high = f.behind != 0;
    } else {
      const unsigned long long t = __builtin_amdgcn_s_memtime();
      high = ((((unsigned)(t >> 15)) & 7u) < kPrioShare) == (f.slot != 0u);
    }
    if (high)
      __builtin_amdgcn_s_setprio(1);
    else
      __builtin_amdgcn_s_setprio(0);
  }
}

// Per-lane fp64 rows in global memory addressed as (wave-uniform buffer resource, this
// lane's byte offset, a constant byte offset in an SGPR): every access needs only the one
// lane-offset VGPR, where 64-bit per-lane pointers (base + lane + 4 KB multiples) would each
// hold two VGPRs across the sweep loop -- and get spilled, then reloaded one after another.
struct LaneRows {
  __amdgpu_buffer_rsrc_t rs;
  int vo;
};
__device__ __forceinline__ LaneRows lane_rows(const double* base, int doubles, int lane) {
  return {__builtin_amdgcn_make_buffer_rsrc(const_cast<double*>(base), 0, doubles * 8, 0x00020000),
          lane * 8};
}
__device__ __forceinline__ double lr_load(const LaneRows& b, int byte_off) {
  return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(b.rs, b.vo, byte_off, 0));
}
__device__ __forceinline__ void lr_store(const LaneRows& b, int byte_off, double v) {
  typedef unsigned int u2 __attribute__((ext_vector_type(2)));
  __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u2, v), b.rs, b.vo, byte_off, 0);
}

// Cross-lane moves within a 16-lane row by DPP (VALU speed, no LDS traffic).
template <int CTRL>
__device__ __forceinline__ double dpp(double v) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_update_dpp(0, (int)(b & 0xffffffffll), CTRL, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_update_dpp(0, (int)(b >> 32), CTRL, 0xF, 0xF, false);
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}
constexpr int DPP_XOR1 = 0xB1, DPP_XOR2 = 0x4E, DPP_ROR4 = 0x124, DPP_ROR8 = 0x128;

// Sum over the wave: quad butterflies + row rotations give every lane its 16-lane row sum,
// then the four row sums are combined in a fixed order from lanes 0/16/32/48, so the result
// is bitwise identical (uniform) in every lane.
__device__ __forceinline__ double wave_sum(double v) {
  v += dpp<DPP_XOR1>(v);
  v += dpp<DPP_XOR2>(v);
  v += dpp<DPP_ROR4>(v);
  v += dpp<DPP_ROR8>(v);
  return (rdlane(v, 0) + rdlane(v, 16)) + (rdlane(v, 32) + rdlane(v, 48));
}

__device__ __forceinline__ double wave_max(double v) {
  v = fmax(v, dpp<DPP_XOR1>(v));
  v = fmax(v, dpp<DPP_XOR2>(v));
  v = fmax(v, dpp<DPP_ROR4>(v));
  v = fmax(v, dpp<DPP_ROR8>(v));
  return fmax(fmax(rdlane(v, 0), rdlane(v, 16)), fmax(rdlane(v, 32), rdlane(v, 48)));
}

// ---- SVD noise floor of the b draw (include/gst.h gst_sweep; oracle Oracle.floor_shift) ----
// The reference draws b through sl.svd(Sigma) (gibbs.py:169-171).  When Sigma's smallest
// eigenvalues lie below ~eps ||Sigma|| (vvh17's all-outlier start, alpha = 1e10: cond ~ 1e22,
// while Sigma diagonally scaled is well conditioned) LAPACK returns them at its own rounding
// floor, ~0.3-2 x 2^-52 s_max, so its draw is in effect one from Sigma + f I -- which is what
// lets the reference's chains leave that state within ~100 sweeps (the exact draw stays there
// for thousands).  The b draw reproduces it: when the smallest pivot of
// the factor over the real columns is below FLOOR_GATE = 2^-52 x the largest (the pivot ratio
// below which LAPACK's SVD resolves those eigenvalues no longer: above it the reference's SVD
// mean agrees with the exact mean to ~1e-6), b is drawn exactly from
// Sigma + f I with f = FLOOR_C 2^-52 x the largest pivot; every other draw is the exact one.
// Each floor draw sets status bit 4 and adds 1 to the floor-draw count in bits 8..30.
constexpr double FLOOR_GATE = 0x1p-52;
#ifndef GST_FLOOR_C
#define GST_FLOOR_C 0.75  // oracle/gibbs_oracle.py FLOOR_C (tools/vvh17_escape.py calibrates it)
#endif
constexpr double FLOOR_C = GST_FLOOR_C;
constexpr int STATUS_FLOOR = 16;
constexpr int STATUS_FLOOR_COUNT = 256;   // one floor draw, counted in bits 8..30
constexpr int DEBUG_LARGE_GRAM = 2;    // large path: dense super-tile Gram (lg_gram) forced
constexpr int DEBUG_EXACT_BDRAW = 8;
constexpr int DEBUG_MFMA_GRAM = 16;   // persistent kernel: no low-rank Gram (tests, A/B)
constexpr int DEBUG_EPOCHS_LDS = 32;  // large path: ECORR-epochs-first chains on lg_hyper<2>

// Smallest / largest pivot over the real columns of a factor whose pivot of internal column
// j = 64 sl + lane is apr[sl]; real columns are [0, ntm) and [f0, f1) (the rest are unit-prior
// pads).  Wave-uniform.
__device__ __forceinline__ void pivot_range(const double (&apr)[2], int lane, int ntm, int f0,
                                            int f1, double& mn, double& mx) {
  mx = 0.0;
  mn = INFINITY;
#pragma unroll
  for (int sl = 0; sl < 2; ++sl) {
    const int j = 64 * sl + lane;
    const bool real = j < ntm || (j >= f0 && j < f1);
    mx = real ? fmax(mx, apr[sl]) : mx;
    mn = real ? fmin(mn, apr[sl]) : mn;
  }
  mx = wave_max(mx);
  mn = -wave_max(-mn);
}
__device__ __forceinline__ double floor_of(double mn, double mx) {
  return mn < FLOOR_GATE * mx ? FLOOR_C * 0x1p-52 * mx : 0.0;
}
__device__ __forceinline__ double floor_shift(const double (&apr)[2], int lane, int ntm, int f0,
                                              int f1) {
  double mn, mx;
  pivot_range(apr, lane, ntm, f0, f1, mn, mx);
  return floor_of(mn, mx);
}

// Sum over p (lane bits 3..5) of the lanes with q == qq (lane = 8p + q), uniform result.
__device__ __forceinline__ double col_sum(double v, int qq) {
  v += dpp<DPP_ROR8>(v);  // (l + 8) mod 16 == l ^ 8
  return (rdlane(v, qq) + rdlane(v, qq + 16)) + (rdlane(v, qq + 32) + rdlane(v, qq + 48));
}

// 1/sqrt(a): hardware estimate + two Newton steps (full double accuracy to ~1 ulp).
__device__ __forceinline__ double rsqrt_nr(double a) {
  double y = __builtin_amdgcn_rsq(a);
  y = y * fma(-0.5 * a * y, y, 1.5);
  y = y * fma(-0.5 * a * y, y, 1.5);
  return y;
}

// Hand-off point between lanes of one wave through LDS.  LDS instructions of a wave execute
// in issue order, so no hardware wait is needed; what must not happen is the COMPILER moving
// a load that reads another lane's data above the store that wrote it (from one lane's
// point of view the two addresses differ, so a single-thread fence does not forbid it).  A
// wavefront-scope fence is the construct that orders memory accesses across the lanes of
// the wave; it emits no instruction.
__device__ __forceinline__ void lds_order() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

// x[i] as a select chain over register values.  The empty asm makes each element an opaque
// register value: without it InstCombine turns the select of array loads into a load from a
// selected address, which keeps the whole parameter array in scratch memory (reloaded in
// every MH step of the 2-chains-per-SIMD build).
__device__ __forceinline__ double pget(const double (&x)[4], int i) {
  double a = x[0], b = x[1], c = x[2], d = x[3];
  asm("" : "+v"(a), "+v"(b), "+v"(c), "+v"(d));
  return i == 0 ? a : (i == 1 ? b : (i == 2 ? c : d));
}
// the general-white-noise instances (GEN): up to 8 parameters
__device__ __forceinline__ double pget(const double (&x)[8], int i) {
  double v[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    v[k] = x[k];
    asm("" : "+v"(v[k]));
  }
  double r = v[7];
#pragma unroll
  for (int k = 6; k >= 0; --k) r = (i == k) ? v[k] : r;
  return r;
}
__device__ __forceinline__ int iget4(const int* a, int i) {   // a[i], i < 4
  return i == 0 ? a[0] : (i == 1 ? a[1] : (i == 2 ? a[2] : a[3]));
}
template <int N>
__device__ __forceinline__ int iget(const int* a, int i) {   // a[i], i < N (4 or 8)
  if constexpr (N == 4) {
    return iget4(a, i);
  } else {
    int r = a[N - 1];
#pragma unroll
    for (int k = N - 2; k >= 0; --k) r = (i == k) ? a[k] : r;
    return r;
  }
}

// The jump (xi * sigma) * scale exactly as numpy evaluates it (gibbs.py:97,130): no FMA
// contraction, so x + jump matches the reference bit for bit.
__device__ __forceinline__ double mh_step(double xi, double sig, double scale) {
#pragma clang fp contract(off)
  return (xi * sig) * scale;
}

// numpy legacy binomial(1, p) given its uniform (inversion branch, random_binomial).
__device__ __forceinline__ int bern_legacy(double p, double u) {
  if (p == 0.0) return 0;
  if (p <= 0.5) return u > exp(log(1.0 - p)) ? 1 : 0;
  const double qq = 1.0 - p;
  return u > exp(log(1.0 - qq)) ? 0 : 1;
}

// cos(2 pi u) for u in [0, 1): folded to a quarter turn, then the Taylor series of cos or
// sin on [0, pi/4] (truncation < 1e-16), chosen by select.  Lighter than OCML's cospi
// (fewer live registers inside the per-TOA gamma loops).
__device__ __forceinline__ double cos2pi(double u) {
  double x = u < 0.5 ? u : 1.0 - u;            // cos(2 pi (1 - u)) = cos(2 pi u)
  const double sg = x > 0.25 ? -1.0 : 1.0;     // cos(2 pi (1/2 - x)) = -cos(2 pi x)
  x = x > 0.25 ? 0.5 - x : x;                  // x in [0, 1/4]
  const bool sn = x > 0.125;                   // cos(2 pi x) = sin(2 pi (1/4 - x))
  const double t = (sn ? 0.25 - x : x) * 6.283185307179586477;   // t in [0, pi/4]
  const double t2 = t * t;
  double c = 1.0 / 20922789888000.0;           // 1/16!
  c = fma(c, t2, -1.0 / 87178291200.0);
  c = fma(c, t2, 1.0 / 479001600.0);
  c = fma(c, t2, -1.0 / 3628800.0);
  c = fma(c, t2, 1.0 / 40320.0);
  c = fma(c, t2, -1.0 / 720.0);
  c = fma(c, t2, 1.0 / 24.0);
  c = fma(c, t2, -0.5);
  c = fma(c, t2, 1.0);
  double sv = 1.0 / 355687428096000.0;         // 1/17!
  sv = fma(sv, t2, -1.0 / 1307674368000.0);
  sv = fma(sv, t2, 1.0 / 6227020800.0);
  sv = fma(sv, t2, -1.0 / 39916800.0);
  sv = fma(sv, t2, 1.0 / 362880.0);
  sv = fma(sv, t2, -1.0 / 5040.0);
  sv = fma(sv, t2, 1.0 / 120.0);
  sv = fma(sv, t2, -1.0 / 6.0);
  sv = fma(sv, t2, 1.0) * t;
  return sg * (sn ? sv : c);
}

// sin(2 pi u) = cos(2 pi (u - 1/4)), the argument wrapped back into [0, 1)
__device__ __forceinline__ double sin2pi(double u) {
  return cos2pi(u < 0.25 ? u + 0.75 : u - 0.25);
}

// Box-Muller normal from one Philox draw (its cosine half).
__device__ __forceinline__ double normal_from(const Rng& rng, uint32_t index, uint32_t tag) {
  double a, b;
  rng.uniform2(index, tag, a, b);
  return sqrt(-2.0 * log(1.0 - a)) * cos2pi(b);
}

// Both Box-Muller normals of one Philox draw: normals 2k and 2k + 1 of a stream.
__device__ __forceinline__ void normal_pair(const Rng& rng, uint32_t k, uint32_t tag,
                                            double& n0, double& n1) {
  double a, b;
  rng.uniform2(k, tag, a, b);
  const double r = sqrt(-2.0 * log(1.0 - a));
  n0 = r * cos2pi(b);
  n1 = r * sin2pi(b);
}

// Normal j of a stream (one element of normal_pair(j / 2)).
__device__ __forceinline__ double normal_k(const Rng& rng, uint32_t j, uint32_t tag) {
  double n0, n1;
  normal_pair(rng, j >> 1, tag, n0, n1);
  return (j & 1u) ? n1 : n0;
}

// Marsaglia-Tsang Gamma(a, 1); a < 1 via the a+1 boost.  Attempts go in pairs: one Philox
// draw gives both Box-Muller normals, a second the two acceptance uniforms.  Bounded.
__device__ double gamma_mt(double a, const Rng& rng, uint32_t index, uint32_t tag) {
  double boost = 1.0;
  if (a < 1.0) {
    double ub, unused;
    rng.uniform2(index, tag | 0xFFFFFFu, ub, unused);
    boost = exp(log(1.0 - ub) / a);
    a += 1.0;
  }
  const double d = a - 1.0 / 3.0;
  const double cc = 1.0 / sqrt(9.0 * d);
#pragma unroll 1
  for (uint32_t att = 0; att < 128u; ++att) {
    double u1, u2, ua, ub;
    rng.uniform2(index, tag | (2u * att), u1, u2);
    rng.uniform2(index, tag | (2u * att + 1u), ua, ub);
    const double r = sqrt(-2.0 * log(1.0 - u1));
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const double xn = r * (h == 0 ? cos2pi(u2) : sin2pi(u2));
      const double u3 = h == 0 ? ua : ub;
      double v = 1.0 + cc * xn;
      if (v <= 0.0) continue;
      v = v * v * v;
      const double x2 = xn * xn;
      if (u3 < 1.0 - 0.0331 * x2 * x2) return d * v * boost;
      if (log(u3) < 0.5 * x2 + d * (1.0 - v + log(v))) return d * v * boost;
    }
  }
  return d * boost;
}

// gamma_mt for NS draws at once -- draw s with shape a[s] and Philox index index0 + 64 s,
// for the slots in `active` -- in one rejection loop, so the independent draws' dependency
// chains interleave.  Every draw consumes exactly gamma_mt's variates in gamma_mt's order,
// hence returns bitwise gamma_mt(a[s], rng, index0 + 64 s, tag).
template <int NS>
__device__ __forceinline__ void gamma_mt_slots(const double (&a)[NS], unsigned active,
                                               const Rng& rng, uint32_t index0, uint32_t tag,
                                               double (&out)[NS]) {
  double d[NS], cc[NS], boost[NS];
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    double as = a[s];
    boost[s] = 1.0;
    if (((active >> s) & 1u) && as < 1.0) {
      double ub, unused;
      rng.uniform2(index0 + 64u * s, tag | 0xFFFFFFu, ub, unused);
      boost[s] = exp(log(1.0 - ub) / as);
      as += 1.0;
    }
    d[s] = as - 1.0 / 3.0;
    cc[s] = 1.0 / sqrt(9.0 * d[s]);
    out[s] = d[s] * boost[s];                 // gamma_mt's value after 256 failed attempts
  }
  unsigned pend = active;
#pragma unroll 1
  for (uint32_t att = 0; att < 128u && pend; ++att) {
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      if (!((pend >> s) & 1u)) continue;
      double u1, u2, ua, ub;
      rng.uniform2(index0 + 64u * s, tag | (2u * att), u1, u2);
      rng.uniform2(index0 + 64u * s, tag | (2u * att + 1u), ua, ub);
      const double r = sqrt(-2.0 * log(1.0 - u1));
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        if (!((pend >> s) & 1u)) break;
        const double xn = r * (h == 0 ? cos2pi(u2) : sin2pi(u2));
        const double u3 = h == 0 ? ua : ub;
        double v = 1.0 + cc[s] * xn;
        if (v <= 0.0) continue;
        v = v * v * v;
        const double x2 = xn * xn;
        if (u3 < 1.0 - 0.0331 * x2 * x2 || log(u3) < 0.5 * x2 + d[s] * (1.0 - v + log(v))) {
          out[s] = d[s] * v * boost[s];
          pend &= ~(1u << s);
        }
      }
    }
  }
}

// Right-looking LDL^T-scaled Cholesky on the cyclic register layout.
//
// Registers keep RAW columns: after column k is eliminated, slot values hold
// a_ik = L_ik * sqrt(a_kk) (the a_kk are the pivots), so L_ik = a_ik / sqrt(a_kk) is never
// formed inside the factorisation; the rank-1 update is a_ij -= (a_ik / a_kk) * a_jk.
// After each step every lane publishes its slot column that holds the next column into
// its own LDS column buffer colq[q][.] (no owner test, no selects); step k reads the
// buffer of q = k % 8.  Rows <= k are masked on the reading side (only slot K can hold
// them).  The slot column holding column k+1 is updated first so its publication (the
// step-to-step dependency through LDS) is issued before the rest of the trailing update.
// Outputs per column: the pivot a_kk and the augmented-row entry a_{raug,k}.  Nothing is
// captured per step (the step is VALU-issue-bound): an eliminated column is frozen in the
// registers (the column-side mask zeroes every later update to it), so chol_harvest reads
// both from L after the elimination; chol_stats then gives sum log a_kk (= log|Sigma| over
// these columns, as mantissa product + exponent sum), sum a_{raug,k}^2 / a_kk (= the
// d^T Sigma^-1 d contribution) and the failure flag.
struct CholCtx {
  double* colq;   // [8][MT] the published column (paired tail: the even column, [8][PW])
  double* junk;   // [8][MT] where the other lanes' publishing stores land (see chol_publish)
  double* colq2;  // [8][MT - KP] paired tail: the odd column (rows >= KP)
  int lane, p, q, raug;
  double mant, quad;
  int expo, fail;
  // pivots a_kk and augmented-row entries a_{raug,k}: column k kept by lane k % 64 in
  // slot k / 64 (filled by chol_harvest)
  double apr[2], zr[2];
};

// Publish column 8s + QQ: its owner lanes (q == QQ) write their slot column s, rows >= s.
// Every lane stores ("pad, don't mask"): the others' stores go to the junk rows, so the
// elimination stays free of lane-divergent control flow, which at this register pressure
// makes the allocator spill kilobytes per lane.
// The published column carries zeros in its rows <= its own index (slot row s, p <= QQ: the
// frozen rows and the pivot row), so the readers' row- and column-side multipliers come out
// masked without a select of their own (one select here instead of two per reader side).
template <int MT, int QQ>
__device__ __forceinline__ void chol_publish(const double (&L)[SL(MT, 0)], CholCtx& cc, int s) {
  double* dst = (cc.q == QQ ? cc.colq : cc.junk) + MT * cc.p;
  const bool live = cc.p > QQ;
#pragma unroll
  for (int r2 = 0; r2 < MT; r2 += 2) {          // rows (r2, r2+1)
    if (r2 >= s) {  // one ds_write_b128 per row pair (16-byte aligned: MT, r2 even)
      typedef double v2_t __attribute__((ext_vector_type(2)));
      const double v0 = (r2 == s) ? (live ? L[SL(r2, s)] : 0.0) : L[SL(r2, s)];
      *(v2_t*)(dst + r2) = (v2_t){v0, L[SL(r2 + 1, s)]};
    } else if (r2 + 1 >= s)
      dst[r2 + 1] = live ? L[SL(r2 + 1, s)] : 0.0;
  }
}

// 1/a: hardware estimate (~2^-24) + one Newton step (~2e-15 relative, measured on
// MI355X by tools/ubench/rcp_acc.hip); on every column step's critical path.
__device__ __forceinline__ double rcp_nr1(double a) {
  const double y = __builtin_amdgcn_rcp(a);
  return fma(y, fma(-a, y, 1.0), y);
}

// Per-thread sum of logs as a running product: mantissa product + exponent sum (v_frexp),
// one log per thread at the end instead of one per TOA (the per-TOA log dominated the white
// block's 21 likelihood rescans; both paths).  The mantissa product is renormalised every 128 factors
// (each factor >= 1/2, so it stays far above the fp64 underflow threshold).
struct LogProd {
  double mp = 1.0;
  int ex = 0, k = 0;
  __device__ __forceinline__ void mul(double v) {
    int e;
    mp *= frexp(v, &e);
    ex += e;
    if ((++k & 127) == 0) {
      mp = frexp(mp, &e);
      ex += e;
    }
  }
  __device__ __forceinline__ double log_sum() const {
    return log(mp) + (double)ex * 0.693147180559945309417;
  }
};

// a / b for positive normal operands without the IEEE division sequence (v_div_scale /
// v_div_fmas / v_div_fixup): reciprocal estimate, one Newton step, then one residual
// correction of the quotient (within 1 ulp of the rounded quotient).
__device__ __forceinline__ double div_pos(double a, double b) {
  const double y = rcp_nr1(b);
  const double q0 = a * y;
  return fma(fma(-b, q0, a), y, q0);
}

// Raw column k as seen by this lane: rows 8r+p (lr), rows 8r+q (lc), the augmented row
// entry, the pivot and its reciprocal.
template <int MT>
struct ColView {
  double lr[MT], lc[MT];
  double akk;
  double y0, e;  // rcp estimate of 1/a_kk and its Newton residual 1 - a_kk y0
};

// 1/a_kk in two halves: the estimate and residual start the step's two dependent chains
// (the critical factor below and the trailing-update reciprocal y0 + y0 e).
template <int MT>
__device__ __forceinline__ void pivot_rcp(ColView<MT>& c) {
  c.y0 = __builtin_amdgcn_rcp(c.akk);
  c.e = fma(-c.akk, c.y0, 1.0);
}

// Rows >= K of a published column [8][STRIDE] whose first stored row is R0 (the one-column
// steps: colq, stride MT, R0 = 0; the paired tail: colq / colq2, stride MT - KP, R0 = KP).
template <int MT, int K, int STRIDE = MT, int R0 = 0>
__device__ __forceinline__ void chol_load(const double* buf, const CholCtx& cc, ColView<MT>& c) {
  static_assert(MT % 2 == 0 && STRIDE % 2 == 0 && R0 % 2 == 0 && K >= R0,
                "128-bit column loads need 16-byte alignment");
  const double* cr = buf + STRIDE * cc.p - R0;
  const double* cq = buf + STRIDE * cc.q - R0;
#pragma unroll
  for (int r2 = 0; r2 < MT; r2 += 2) {          // rows (r2, r2+1)
    if (r2 >= K) {  // 128-bit loads (16-byte aligned: MT, r2 even)
      typedef double v2_t __attribute__((ext_vector_type(2)));
      const v2_t a = *(const v2_t*)(cr + r2);
      const v2_t b = *(const v2_t*)(cq + r2);
      c.lr[r2] = a[0];
      c.lr[r2 + 1] = a[1];
      c.lc[r2] = b[0];
      c.lc[r2 + 1] = b[1];
    } else if (r2 + 1 >= K) {
      c.lr[r2 + 1] = cr[r2 + 1];
      c.lc[r2 + 1] = cq[r2 + 1];
    }
  }
}

// ---- Paired tail: two columns per LDS hand-off ------------------------------------------
// From slot column KP on, columns k and k+1 (k even, both in slot column KB) are
// published together, column k+1 still RAW with respect to column k.  Every lane applies
// column k's update to its own copy of column k+1 (one FMA per loaded row, the multiplier
// tk = a(k+1,k) / a_kk a wave-uniform scalar from the owner lanes' registers), so a hand-off
// serves two columns: the tail of the elimination is latency-bound on the ~140-cycle
// write -> read hand-off, and this halves the number of hand-offs.
// Every matrix element still receives the one-column steps' FMAs, with the same operands, in
// the same order (including which slot column takes the column-scaled form), and the
// corrected copy of column k+1 is the expression its owner lanes evaluate in the one-column
// step: the factor is bitwise that of chol_step alone.
template <int MT, int QQ, int KP>
__device__ __forceinline__ void chol_publish_pair(const double (&L)[SL(MT, 0)], CholCtx& cc,
                                                  int s) {
  constexpr int PW = MT - KP;
  const bool even = cc.q == QQ, odd = cc.q == QQ + 1;
  double* dst = (even ? cc.colq : (odd ? cc.colq2 : cc.junk)) + PW * cc.p - KP;
  const bool live = cc.p > (odd ? QQ + 1 : QQ);   // zero rows <= the column's own index
#pragma unroll
  for (int r2 = KP; r2 < MT; r2 += 2) {
    if (r2 >= s) {
      typedef double v2_t __attribute__((ext_vector_type(2)));
      const double v0 = (r2 == s) ? (live ? L[SL(r2, s)] : 0.0) : L[SL(r2, s)];
      *(v2_t*)(dst + r2) = (v2_t){v0, L[SL(r2 + 1, s)]};
    } else if (r2 + 1 >= s)
      dst[r2 + 1] = live ? L[SL(r2 + 1, s)] : 0.0;
  }
}

// Publish columns 8KB + QQ and 8KB + QQ + 1 (slot column KB already updated by every earlier
// column), load both, and turn the odd one into its value after the even column's update.
// Returns nothing; n0 / n1 are ready for chol_pair (pivots and reciprocals set).
template <int MT, int KB, int QQ, int KP>
__device__ __forceinline__ void pair_handoff(double (&L)[SL(MT, 0)], CholCtx& cc,
                                             ColView<MT>& n0, ColView<MT>& n1) {
  constexpr int PW = MT - KP;
  static_assert(QQ % 2 == 0 && KB >= KP && KP % 2 == 0 && KP >= KP_MIN,
                "pairs start at even columns of the paired tail");
  lds_order();                       // the previous pair's loads precede the overwrite
  chol_publish_pair<MT, QQ, KP>(L, cc, KB);
  const double a22 = rdlane(L[SL(KB, KB)], 9 * QQ);       // a(k, k)
  const double a32 = rdlane(L[SL(KB, KB)], 9 * QQ + 8);   // a(k+1, k)
  const double a33 = rdlane(L[SL(KB, KB)], 9 * QQ + 9);   // a(k+1, k+1), before column k
  lds_order();
  ColView<MT> raw;
  chol_load<MT, KB, PW, KP>(cc.colq, cc, n0);
  chol_load<MT, KB, PW, KP>(cc.colq2, cc, raw);
  n0.akk = a22;
  pivot_rcp<MT>(n0);
  // the one-column step's factor of column k+1's owner lanes (lc[K1] y0 refined)
  const double t = a32 * n0.y0;
  const double tk = fma(t, n0.e, t);
  n1.akk = fma(-a32, tk, a33);
  pivot_rcp<MT>(n1);
#pragma unroll
  for (int r = KB; r < MT; ++r) {
    n1.lr[r] = fma(-n0.lr[r], tk, raw.lr[r]);
    n1.lc[r] = fma(-n0.lc[r], tk, raw.lc[r]);
  }
  // rows <= k+1 of slot KB: frozen / pivot rows of column k+1, as its publication would carry
  n1.lr[KB] = (cc.p > QQ + 1) ? n1.lr[KB] : 0.0;
  n1.lc[KB] = (cc.q > QQ + 1) ? n1.lc[KB] : 0.0;
}

// Columns k = 8K + KK and k+1 (KK even); c0 / c1 as pair_handoff leaves them.
template <int MT, int K, int KK, int KEND, int KP>
__device__ __forceinline__ void chol_pair(double (&L)[SL(MT, 0)], CholCtx& cc, ColView<MT>& c0,
                                          ColView<MT>& c1) {
  static_assert(KK % 2 == 0, "pairs start at even columns");
  constexpr int k = 8 * K + KK;
  constexpr int KB = (KK == 6) ? K + 1 : K;   // slot column of columns k+2, k+3
  constexpr int QB = (KK + 2) & 7;
  constexpr bool NEXT = k + 2 < KEND;
  static_assert(k + 2 <= KEND, "the paired tail covers an even number of columns");
  // column k's column-scaled factor (its "critical" slot column is K, which holds k+1)
  const double t0 = c0.lc[K] * c0.y0;
  const double tk0 = fma(t0, c0.e, t0);
  const double sk0 = fma(c0.y0, c0.e, c0.y0);
  // column k+1's (its critical slot column is KB, which holds k+2)
  const double t1 = c1.lc[KB < MT ? KB : K] * c1.y0;
  const double tk1 = fma(t1, c1.e, t1);
  const double sk1 = fma(c1.y0, c1.e, c1.y0);
  ColView<MT> n0, n1;
  if constexpr (KB < MT) {
    // critical path: slot column KB (columns k+2, k+3) by column k, then by column k+1
#pragma unroll
    for (int r = KB; r < MT; ++r) {
      double v = L[SL(r, KB)];
      if constexpr (KB == K)
        v = fma(-c0.lr[r], tk0, v);
      else
        v = fma(-(c0.lr[r] * sk0), c0.lc[KB], v);
      L[SL(r, KB)] = fma(-c1.lr[r], tk1, v);
    }
    if constexpr (NEXT) pair_handoff<MT, KB, QB, KP>(L, cc, n0, n1);
  }
  // the rest of the two columns' trailing update (row-scaled, as the one-column steps)
  double lrs0[MT], lrs1[MT];
#pragma unroll
  for (int r = K; r < MT; ++r) {
    lrs0[r] = c0.lr[r] * sk0;
    lrs1[r] = c1.lr[r] * sk1;
  }
#pragma unroll
  for (int s = K; s < MT; ++s) {
    if (s == KB) continue;
#pragma unroll
    for (int r = s; r < MT; ++r) {
      if (s == K) {
        // KK == 6: slot column K is column k's critical one (it holds k+1); column k+1 (the
        // slot's last) leaves it alone
        L[SL(r, s)] = fma(-c0.lr[r], tk0, L[SL(r, s)]);
      } else {
        const double v = fma(-lrs0[r], c0.lc[s], L[SL(r, s)]);
        L[SL(r, s)] = fma(-lrs1[r], c1.lc[s], v);
      }
    }
  }
  if constexpr (NEXT) chol_pair<MT, KB, QB, KEND, KP>(L, cc, n0, n1);
}

// Step k = 8K + KK, software-pipelined: the slot column holding column k+1 is updated
// and published first, column k+1's loads and pivot reciprocal are issued, and only then
// does the rest of step k's trailing update run (covering their latency).
template <int MT, int K, int KK, int KEND, int KP>
__device__ __forceinline__ void chol_step(double (&L)[SL(MT, 0)], CholCtx& cc,
                                          ColView<MT>& cur) {
  constexpr int k = 8 * K + KK;
  constexpr int K1 = (KK == 7) ? K + 1 : K;  // slot column of column k+1
  constexpr int KK1 = (KK + 1) & 7;
  constexpr bool NEXT = k + 1 < KEND;
  // rows <= k of slot K arrive as zeros (chol_publish): frozen entries stay untouched
  // column k+1 starts the paired tail: publish it together with k+2 (pair_handoff)
  constexpr bool TOPAIR = NEXT && K1 >= KP;
  static_assert(!TOPAIR || KK1 == 0, "the paired tail starts at a slot column");
  ColView<MT> nxt, nxt2;
  if constexpr (K1 < MT) {
    // critical path: slot column K1 (holds column k+1).  Its factor a_{8K1+q,k} / a_kk is
    // one value per lane (lc y0 refined by the Newton term), so the published column
    // feeds this FMA directly: LDS load -> FMA and rcp -> mul -> FMA -> FMA are the two
    // step-to-step chains (the row-scaled lrs below stay off them).
    const double t0 = cur.lc[K1] * cur.y0;
    const double tk = fma(t0, cur.e, t0);
#pragma unroll
    for (int r = K1; r < MT; ++r) L[SL(r, K1)] = fma(-cur.lr[r], tk, L[SL(r, K1)]);
    if constexpr (TOPAIR) {
      pair_handoff<MT, K1, 0, KP>(L, cc, nxt, nxt2);
    } else if constexpr (NEXT) {
      lds_order();                   // column k's loads precede its overwrite
      chol_publish<MT, KK1>(L, cc, K1);
      nxt.akk = rdlane(L[SL(K1, K1)], 9 * KK1);
      lds_order();
      chol_load<MT, K1>(cc.colq, cc, nxt);
      pivot_rcp<MT>(nxt);
    }
  }
  // lrs = a_ik / a_kk for the rest of the trailing update (one multiply per row, then one
  // FMA per element)
  const double sk = fma(cur.y0, cur.e, cur.y0);
  double lrs[MT];
#pragma unroll
  for (int r = K; r < MT; ++r) lrs[r] = cur.lr[r] * sk;
  // off the critical path: the rest of the trailing update
#pragma unroll
  for (int s = K; s < MT; ++s) {
    if (s == K1 || (KK == 7 && s == K)) continue;  // slot column K is done when KK == 7
#pragma unroll
    for (int r = s; r < MT; ++r) L[SL(r, s)] = fma(-lrs[r], cur.lc[s], L[SL(r, s)]);
  }
  if constexpr (TOPAIR)
    chol_pair<MT, K1, 0, KEND, KP>(L, cc, nxt, nxt2);
  else if constexpr (NEXT)
    chol_step<MT, K1, KK1, KEND, KP>(L, cc, nxt);
}

// Eliminate columns [8*KLO, KEND) (compile-time: no branch between steps), updating the
// trailing slots.
template <int MT, int KLO, int KEND, int KP>
__device__ __forceinline__ void chol_range(double (&L)[SL(MT, 0)], CholCtx& cc) {
  static_assert(KEND > 8 * KLO && KEND <= 8 * MT, "bad elimination range");
  if constexpr (KLO >= KP) {
    ColView<MT> c0, c1;
    pair_handoff<MT, KLO, 0, KP>(L, cc, c0, c1);
    chol_pair<MT, KLO, 0, KEND, KP>(L, cc, c0, c1);
  } else {
    chol_publish<MT, 0>(L, cc, KLO);
    ColView<MT> c;
    c.akk = rdlane(L[SL(KLO, KLO)], 0);
    lds_order();
    chol_load<MT, KLO>(cc.colq, cc, c);
    pivot_rcp<MT>(c);
    chol_step<MT, KLO, 0, KEND, KP>(L, cc, c);
  }
  lds_order();
}

// The same elimination without the next column's prefetch (one ColView live instead of
// two): used for the timing-model columns, where every slot of L is still live and the
// register budget of two chains per SIMD has no room for the double buffer.
template <int MT, int K, int KK, int KEND>
__device__ __forceinline__ void chol_step_lean(double (&L)[SL(MT, 0)], CholCtx& cc) {
  constexpr int k = 8 * K + KK;
  constexpr int K1 = (KK == 7) ? K + 1 : K;
  constexpr int KK1 = (KK + 1) & 7;
  ColView<MT> cur;
  lds_order();                       // the previous step's loads precede this publication
  chol_publish<MT, KK>(L, cc, K);
  cur.akk = rdlane(L[SL(K, K)], 9 * KK);
  lds_order();
  chol_load<MT, K>(cc.colq, cc, cur);
  pivot_rcp<MT>(cur);
  // rows <= k of slot K arrive as zeros (chol_publish): frozen entries stay untouched
  const double sk = fma(cur.y0, cur.e, cur.y0);
#pragma unroll
  for (int s = K; s < MT; ++s) {
    if (KK == 7 && s == K) continue;   // slot column K is complete
#pragma unroll
    for (int r = s; r < MT; ++r) L[SL(r, s)] = fma(-(cur.lr[r] * sk), cur.lc[s], L[SL(r, s)]);
  }
  if constexpr (k + 1 < KEND) chol_step_lean<MT, K1, KK1, KEND>(L, cc);
}

template <int MT, int KLO, int KEND>
__device__ __forceinline__ void chol_range_lean(double (&L)[SL(MT, 0)], CholCtx& cc) {
  static_assert(KEND > 8 * KLO && KEND <= 8 * MT, "bad elimination range");
  chol_step_lean<MT, KLO, 0, KEND>(L, cc);
  lds_order();
}

// Lane-parallel statistics of an elimination over columns [KLO, KEND) from the per-lane
// pivots / aug entries (lane k % 64 of apr[k / 64], zr[k / 64]): prod a_kk as mantissa
// product + exponent sum (log taken once by the caller), sum a_{raug,k}^2 / a_kk and the
// failure flag, all wave-uniform.  Branch-free on purpose: a lane-divergent region here,
// inside the register-critical hyper block, makes the allocator spill ~1.4 KB per lane.
__device__ __forceinline__ double bperm(double v, int src_lane) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_ds_bpermute(4 * src_lane, (int)(b & 0xffffffffll));
  const int hi = __builtin_amdgcn_ds_bpermute(4 * src_lane, (int)(b >> 32));
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}

// After an elimination over columns [KLO, KEND): the pivot of column j = 8K+q is frozen in
// lane (q,q) slot (K,K) and its augmented-row entry in lane (RA%8, q) slot (RA/8, K); lane
// j % 64 of apr / zr[j / 64] fetches both (one lane permute per slot column, no branch).
template <int MT, int KLO, int KEND, int RA>
__device__ __forceinline__ void chol_harvest(const double (&L)[SL(MT, 0)], CholCtx& cc) {
  constexpr int R = RA / 8, PA = RA % 8;
  static_assert(KEND <= RA && RA < 8 * MT, "augmented row below the eliminated columns");
#pragma unroll
  for (int K = KLO / 8; K <= (KEND - 1) / 8; ++K) {
    const double vd = bperm(L[SL(K, K)], 9 * cc.q);
    const double vz = bperm(L[SL(R, K)], 8 * PA + cc.q);
    const int j = 8 * K + cc.q;
    const bool in = (j >= KLO) && (j < KEND);
#pragma unroll
    for (int sl = 0; sl < 2; ++sl) {
      const bool mine = in && (8 * sl + cc.p == K);
      cc.apr[sl] = mine ? vd : cc.apr[sl];
      cc.zr[sl] = mine ? vz : cc.zr[sl];
    }
  }
}

template <int KLO, int KEND>
__device__ __forceinline__ void chol_stats(CholCtx& cc) {
  double mm = 1.0, qd = 0.0;
  int ee = 0, f = 0;
#pragma unroll
  for (int sl = 0; sl < 2; ++sl) {
    const int j = 64 * sl + cc.lane;
    const bool in = (j >= KLO) && (j < KEND);
    const double a = in ? cc.apr[sl] : 1.0, z = in ? cc.zr[sl] : 0.0;
    f |= !(a > 0.0) ? 1 : 0;
    int e;
    mm *= frexp(a, &e);
    ee += e;
    qd = fma(z * z, rcp_nr1(a), qd);
  }
  mm *= dpp<DPP_XOR1>(mm);
  mm *= dpp<DPP_XOR2>(mm);
  mm *= dpp<DPP_ROR4>(mm);
  mm *= dpp<DPP_ROR8>(mm);
  cc.mant = (rdlane(mm, 0) * rdlane(mm, 16)) * (rdlane(mm, 32) * rdlane(mm, 48));
  cc.expo = (int)wave_sum((double)ee);
  cc.quad = wave_sum(qd);
  cc.fail = __ballot(f) != 0ull ? 1 : 0;
}

// WPB = chains (waves) per workgroup (4 = one per SIMD; the host picks 2 or 1 when the
// launch has fewer chains than CUs x 4, so the chains spread over every CU).  OCC = chains
// per SIMD the kernel is compiled for: 2 caps it at 256 registers per lane (VGPR + AGPR)
// so that two workgroups share a CU and each SIMD interleaves two chains' dependency
// chains (the kernel is latency-bound per wave).
// PAIR (with WPB = 2): the two waves of a workgroup run ONE chain, for launches with at most
// one chain per two SIMDs (config 3's 512 chains).  Both waves run every stage on identical
// state and variates; in the hyper block they evaluate different MH points per round -- the
// next proposal, and the one after it on the branch the chain's acceptance history predicts
// -- and exchange the lnL values through LDS, so that a round settles one or two MH steps
// (DESIGN.md section 8).
// GEN: the general white-noise model (per-backend efac / equad, ECORR epoch columns in the
// hyper block, up to 8 parameters; gibbs.py:64-77); pair mode too since round 6.
template <int MT, int NS, int K0, int RA, bool TAPE, int WPB = 4, int OCC = 1, bool PAIR = false,
          bool GEN = false>
__global__ void __launch_bounds__(64 * WPB, OCC)
    gst_sweep_kernel(const DevModel* __restrict__ mds, const DevState st, const DevRec rec, const DevTape tape,
                     int C, int nsweeps, long long sweep0, int record_every, unsigned mask,
                     unsigned long long seed, long long chain0, int eval_only, double* out_w,
                     double* out_h) {
  static_assert(!PAIR || (WPB == 2 && !TAPE), "pair mode: one chain per 2-wave workgroup");
  constexpr int PX = GEN ? 8 : 4;     // parameters held in registers
  constexpr int NSL = SL(MT, 0);
  constexpr int NT = MT / 2;          // 16-wide MFMA tiles
  constexpr int NTT = NT * (NT + 1) / 2;
  constexpr int MP = 8 * MT;
  constexpr int NTMS = NSL - SL(MT - K0, 0);  // timing-model factor slots (s < K0)
  constexpr int TB_LD = 17;
  constexpr int S0RD = s0r_doubles(MT, K0);
  static_assert(s0r_need(MT, NS) <= S0RD, "S0 region too small for the stage scratch");
  __shared__ double smem[WPB][lds_doubles(MT, K0)];
  __shared__ double xchg[PAIR ? 2 : 1][2][2];  // pair mode: [round parity][wave] {lnL, failed}
  __shared__ int xdrew[PAIR ? 1 : 1];          // pair mode: the b draw happened this sweep
  __shared__ double xfloor[1];                 // pair mode: the owner's floor_shift
  // pair mode: z / pout and alpha of the TOA slots the other wave drew (slot s belongs to
  // wave s & 1), exchanged after each stage
  __shared__ double xpo[PAIR ? NS : 1][PAIR ? 64 : 1], xal[PAIR ? NS : 1][PAIR ? 64 : 1];
  __shared__ double xyv[PAIR ? NS : 1][PAIR ? 64 : 1];   // pair mode: the drawer's y = r - T b
  __shared__ unsigned long long xzm[PAIR ? NS : 1];
  __shared__ unsigned gcnt[WPB][2];            // Grams by path (gst_gram_counts)

  const int lane = threadIdx.x & 63;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int c = PAIR ? (int)blockIdx.x : (int)blockIdx.x * WPB + wv;
  const int role = PAIR ? wv : 0;   // pair mode: which of the chain's two waves
  if (c >= C) return;
  // the chain's dataset (run_sims grids batch many datasets x models per launch): every
  // field of md is wave-uniform, so it is read with scalar loads
  const int ds = st.dataset ? __builtin_amdgcn_readfirstlane(st.dataset[c]) : 0;
  if ((unsigned)ds >= (unsigned)st.nd) {  // bad index: flag the chain, touch nothing else
    if (lane == 0 && st.status) st.status[c] |= 4;
    return;
  }
  const DevModel& md = mds[ds];
  const int nst = st.nst;
  const int p = lane >> 3, q = lane & 7;
  Fair fair{OCC == 2 ? wave_slot_parity() : 0u, -1};
  unsigned long long prog_ret = 0ull;  // lane 0: this sweep's ticket from st.prog
  GST_STAMP_DECL

  double* S0R = smem[wv];             // S0 during the hyper block, else stage scratch
  double* colq = S0R + S0RD;          // [8][MT] the published column
  double* mhh = colq + 8 * MT;        // [10][4] hyper MH variates
  double* phbuf = mhh + 4 * NHYPER;   // phi^-1 by internal index; eliminations' junk rows
  double* colq2 = phbuf + 8 * MT;     // [8][PW] paired tail: the odd published column
  double* S0 = S0R + lane;            // S0[64 * slot]
  // scratch inside S0R (S0 is dead outside the hyper block):
  double* mhw = S0R;                  // [20][4] white MH variates (sweep start .. white block)
  double* vbuf = S0R;                 // Gram weights, 64*NS
  double* tbuf = S0R + 64 * NS;       // 16 x TB_LD Gram tile transpose
  double* zraw = S0R;                 // b draw: a_{raug,k}
  double* apiv = zraw + MP;           //   pivots a_kk
  double* wvec = apiv + MP;           //   back-substitution rhs
  double* xbuf = wvec + MP;           //   Delta, solution (internal order)
  double* yinv = xbuf + MP;           //   1/sqrt(a_kk)
  double* bsc = yinv + MP;            //   b in reference order (T b input)
  double* tdg = bsc + MP;             //   8 x 8 diagonal-block transposes
  double* dfbuf = S0R;                // nu grid: weights [32], probabilities [32]
  // the TM factor slots (s < K0) wait in global scratch while the hyper block runs
  // per-chain rows of the state arrays: wave-uniform base pointers (SGPRs), so every
  // per-lane access is base + 32-bit lane offset
  const LaneRows tmf =
      lane_rows(st.tmfac + ((size_t)c * (PAIR ? 2 : 1) + role) * NTMS * 64, NTMS * 64, lane);
  double* const xrow = st.x + (size_t)c * md.P;
  double* const brow = st.b + (size_t)c * md.m;
  double* const zrow = st.z + (size_t)c * nst;
  double* const arow = st.alpha + (size_t)c * nst;
  double* const prow = st.pout + (size_t)c * nst;

  static_assert(RA >= 8 * K0 + 1 && RA < 8 * MT, "augmented row out of range");
  const int n = md.n, m = md.m, P = md.P;
  constexpr int raug = RA;
  const int npad = md.npad;
  const long long gch = chain0 + c;

  Rng rng;
  rng.k0 = (uint32_t)(seed & 0xffffffffull);
  rng.k1 = (uint32_t)(seed >> 32);
  rng.chain = (uint32_t)gch;
  rng.sweep = 0;

  // ---------------- load chain state ----------------
  double xv[PX] = {};
#pragma unroll
  for (int j = 0; j < PX; ++j)
    if (j < P) xv[j] = xrow[j];
  double theta = st.theta[c];
  double nu = st.nu[c];
  for (int j = lane; j < MP; j += 64) bsc[j] = (j < m) ? brow[j] : 0.0;
  for (int j = lane; j < MP; j += 64) phbuf[j] = 0.0;

  // per-TOA chain state in registers: alpha, y = r - T b, pout and the z bits; the data
  // (r, sigma^2, noise class) is re-read from the dataset's L2-resident arrays where used
  double al[NS], yv[NS], po[NS];
  double wcls = 0.0;  // lane u < ncls: W_u of the current white block
  unsigned zb = 0u, vmask = 0u;
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    const int t = 64 * s + lane;
    const bool ok = t < n;
    vmask |= ok ? (1u << s) : 0u;
    al[s] = ok ? arow[t] : 1.0;
    po[s] = ok ? prow[t] : 0.0;
    const double zz = ok ? zrow[t] : 0.0;
    zb |= (zz != 0.0) ? (1u << s) : 0u;
    yv[s] = 0.0;
  }
  double rrr[OCC == 1 ? NS : 1];   // one-wave-per-SIMD builds: the lanes' residuals, as s2r
  if constexpr (OCC == 1) {
#pragma unroll
    for (int s = 0; s < NS; ++s) rrr[s] = ((vmask >> s) & 1u) ? md.resid[64 * s + lane] : 0.0;
  }
  auto RR = [&](int s) __attribute__((always_inline)) -> double {
    if constexpr (OCC == 1)
      return rrr[s];
    else
      return md.resid[64 * s + lane];
  };
  // one-wave-per-SIMD builds: sigma^2 of the lane's TOAs in registers for the launch (the
  // per-TOA white likelihood reads it 21 times a sweep, each a pointer load, a global load
  // and a wait without machine LICM); the two-chains-per-SIMD build has no registers to spare
  double s2r[OCC == 1 ? NS : 1];
  if constexpr (OCC == 1) {
#pragma unroll
    for (int s = 0; s < NS; ++s) s2r[s] = ((vmask >> s) & 1u) ? md.sig2[64 * s + lane] : 0.0;
  }
  auto S2 = [&](int s) __attribute__((always_inline)) -> double {
    if constexpr (OCC == 1)
      return s2r[s];
    else
      return md.sig2[64 * s + lane];
  };
  int status = 0, nfloor = 0;   // nfloor: b draws at the SVD noise floor in this launch
  // Grams computed in this launch by path (gst_gram_counts): low-rank (class Grams + rank-1
  // updates on the VALU) and n-TOA fp64 MFMA, counted in LDS (registers held across the sweep
  // loop raised the two-chains-per-SIMD build's spill by 32 B/lane)
  if (lane == 0) {
    gcnt[wv][0] = 0u;
    gcnt[wv][1] = 0u;
  }
  lds_order();

  // y = r - T b (gibbs.py:213,237,272): 8 columns x NS TOA slots of loads in flight
  auto compute_Tb = [&]() __attribute__((always_inline)) {
    double tb[NS];
#pragma unroll
    for (int s = 0; s < NS; ++s) tb[s] = 0.0;
    const int nsl = md.nslot_toa;
    const double* tc = md.Tcol;
    int j = 0;
#pragma unroll 1
    for (; j + 8 <= m; j += 8) {   // (16 columns per round: 2% slower, spills)
      double tv[8][NS], bj[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
#pragma unroll
        for (int s = 0; s < NS; ++s)
          tv[u][s] = tc[(j + u) * npad + 64 * (s < nsl ? s : nsl - 1) + lane];
        bj[u] = bsc[j + u];
      }
#pragma unroll
      for (int u = 0; u < 8; ++u)
#pragma unroll
        for (int s = 0; s < NS; ++s) tb[s] = fma(tv[u][s], bj[u], tb[s]);
    }
#pragma unroll 1
    for (; j < m; ++j) {
      const double bjj = bsc[j];
#pragma unroll
      for (int s = 0; s < NS; ++s)
        tb[s] = fma(tc[j * npad + 64 * (s < nsl ? s : nsl - 1) + lane], bjj, tb[s]);
    }
#pragma unroll
    for (int s = 0; s < NS; ++s) yv[s] = (s < nsl) ? RR(s) - tb[s] : 0.0;
  };

  // sum of log-priors (gibbs.py:337-339): every prior is uniform, so the sum is the
  // host-evaluated constant (Python sum order) when all parameters are in bounds, else -inf
  // one-wave-per-SIMD builds (registers to spare): the prior bounds and efac choice held in
  // registers for the launch instead of re-read from the model descriptor at every call
  // (no machine LICM in this build: each read was a load and a wait)
  double hpmin[PX], hpmax[PX], hlp = 0.0, hefc = 1.0;
  int hief = -1;
  if constexpr (OCC == 1) {
#pragma unroll
    for (int j = 0; j < PX; ++j) {
      hpmin[j] = j < P ? md.pmin[j] : 0.0;
      hpmax[j] = j < P ? md.pmax[j] : 0.0;
    }
    hlp = md.lp_sum;
    hief = md.idx_efac;
    hefc = md.efac_const;
  }
  auto lnprior = [&](const double (&xq)[PX]) __attribute__((always_inline)) -> double {
    bool in = true;
#pragma unroll
    for (int j = 0; j < PX; ++j) {
      if (OCC == 1) {
        if (j < P) in = in && (xq[j] >= hpmin[j]) && (xq[j] <= hpmax[j]);
      } else {
        if (j < P) in = in && (xq[j] >= md.pmin[j]) && (xq[j] <= md.pmax[j]);
      }
    }
    return in ? (OCC == 1 ? hlp : md.lp_sum) : -INFINITY;
  };

  auto efac2_of = [&](const double (&xq)[PX]) __attribute__((always_inline)) -> double {
    const double ef = OCC == 1 ? (hief >= 0 ? pget(xq, hief) : hefc)
                               : (md.idx_efac >= 0 ? pget(xq, md.idx_efac) : md.efac_const);
    return ef * ef;
  };

  // GEN: N0 = efac_b^2 sigma^2 + 10^(2 equad_b) of the TOA's backend b (gibbs.py:262-284 with
  // the enterprise white-noise signal per backend).  The parameter indices of each of the
  // lane's TOA slots and of its noise class (lane u < ncls) are held for the launch.
  int gef[GEN ? NS : 1], geq[GEN ? NS : 1], gcef = -1, gceq = 0;
  if constexpr (GEN) {
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      const int b = ((vmask >> s) & 1u) && md.bk ? md.bk[64 * s + lane] : 0;
      gef[s] = md.efac_b[b];
      geq[s] = md.equad_b[b];
    }
    const int cb = lane < md.ncls ? md.cls_b[lane] : 0;
    gcef = md.efac_b[cb];
    gceq = md.equad_b[cb];
  }
  auto gen_n0 = [&](const double (&xq)[PX], double s2, int ie, int iq)
      __attribute__((always_inline)) -> double {
    const double ef = ie >= 0 ? pget(xq, ie) : md.efac_const;
    return ef * ef * s2 + exp(2.0 * pget(xq, iq) * 2.302585092994045684);
  };
  // N0 of noise class k (wave-uniform k)
  auto cls_n0 = [&](const double (&xq)[PX], int k) __attribute__((always_inline)) -> double {
    const int b = md.cls_b[k];
    return gen_n0(xq, md.csig2[k], md.efac_b[b], md.equad_b[b]);
  };

  // white-noise conditional likelihood (gibbs.py:262-284).  Class path: TOAs with equal
  // sigma share N0 = efac^2 sigma^2 + Q, so with a_t = alpha_t^z_t
  //   sum_t log N_t = sum_t log a_t + sum_u c_u log N0_u,
  //   sum_t y_t^2 / N_t = sum_u W_u / N0_u,   W_u = sum_{t in u} y_t^2 / a_t,
  // where sum log a_t and W_u are fixed for the whole white block (b, alpha, z fixed).
  const int hncls = md.ncls, hieq = md.idx_equad;   // read once for the launch (scalars)
  double wcls_la = 0.0;   // sum_t log a_t
  auto white_prep = [&]() __attribute__((always_inline)) {
    if (md.ncls == 0) return;
    double la = 0.0;
#pragma unroll
    for (int s = 0; s < NS; ++s)
      if ((vmask >> s) & 1u) la += ((zb >> s) & 1u) ? log(al[s]) : 0.0;
    wcls_la = wave_sum(la);
    // only the TOA slots of this chain's dataset: a ragged batch's shorter datasets have
    // fewer than 64 NS entries of cidx
    int cls[NS];
#pragma unroll
    for (int s = 0; s < NS; ++s) cls[s] = ((vmask >> s) & 1u) ? md.cidx[64 * s + lane] : -1;
    for (int u = 0; u < md.ncls; ++u) {
      double w = 0.0;
#pragma unroll
      for (int s = 0; s < NS; ++s)
        if (((vmask >> s) & 1u) && cls[s] == u)
          w += yv[s] * yv[s] / (((zb >> s) & 1u) ? al[s] : 1.0);
      w = wave_sum(w);
      if (lane == u) wcls = w;
    }
  };
  // Q = 10^(2 equad) is passed in: the MH steps carry it (Q_q = Q_x * 10^(2 delta)).
  auto lnl_white = [&](const double (&xq)[PX], double Q) __attribute__((always_inline)) -> double {
    const double ef2 = efac2_of(xq);
    if (GEN && hncls == 1) {
      const double N0 = cls_n0(xq, 0);
      return -0.5 * ((wcls_la + md.ccount[0] * log(N0)) + rdlane(wcls, 0) / N0);
    }
    if (!GEN && hncls == 1) {  // uniform: no reduction
      const double N0 = ef2 * md.csig2[0] + Q;
      return -0.5 * ((wcls_la + md.ccount[0] * log(N0)) + rdlane(wcls, 0) / N0);
    }
    double sl = 0.0, sq = 0.0;
    if (hncls > 1) {
      if (lane < md.ncls) {
        const double N0 = GEN ? gen_n0(xq, md.csig2[lane], gcef, gceq) : ef2 * md.csig2[lane] + Q;
        sl = md.ccount[lane] * log(N0);
        sq = wcls / N0;
      }
      sl = wave_sum(sl) + wcls_la;
      sq = wave_sum(sq);
      return -0.5 * (sl + sq);
    }
    LogProd lp;
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      if (vmask & (1u << s)) {
        double N0;
        if constexpr (GEN)
          N0 = gen_n0(xq, S2(s), gef[s], geq[s]);
        else
          N0 = ef2 * S2(s) + Q;
        const double N = ((zb >> s) & 1u ? al[s] : 1.0) * N0;
        lp.mul(N);
        sq += div_pos(yv[s] * yv[s], N);
      }
    }
    sl = wave_sum(lp.log_sum());
    sq = wave_sum(sq);
    return -0.5 * (sl + sq);
  };

  // MH variates of one sweep (30 steps: 20 white then 10 hyper), produced in parallel by
  // lanes 0..29: u_scale, parameter index, jump normal, log(u_accept) (gibbs.py:95-104,
  // 128-137).  Tape mode copies the reference's recorded values instead.
  auto mh_variates = [&](const double* tp) __attribute__((always_inline)) {
    if (lane < NWHITE + NHYPER) {
      const bool white = lane < NWHITE;
      const int step = white ? lane : lane - NWHITE;
      double us, par, xi, la;
      if (TAPE) {
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
        par = (double)(white ? iget<PX>(md.wind, k) : iget<PX>(md.hind, k));
      }
      int cnt = 0;
#pragma unroll
      for (int i = 0; i < 5; ++i) cnt += (md.mh_cdf[i] <= us) ? 1 : 0;
      cnt = cnt < 4 ? cnt : 4;
      const double scale = md.mh_size[0] * (cnt == 0) + md.mh_size[1] * (cnt == 1) +
                           md.mh_size[2] * (cnt == 2) + md.mh_size[3] * (cnt == 3) +
                           md.mh_size[4] * (cnt == 4);
      const double delta = mh_step(xi, white ? md.sig_w : md.sig_h, scale);
      double* e = white ? mhw + 4 * step : mhh + 4 * step;
      e[0] = par;
      e[1] = delta;
      e[2] = la;
      e[3] = exp(2.0 * delta * 2.302585092994045684);
    }
    lds_order();
  };

  // MH proposal of global step gs (gibbs.py:90-97 / 123-130): q = x with q[par] += delta;
  // returns log(u_accept).  E receives 10^(2 delta) (equad moves rescale Q by it).
  auto propose = [&](const double (&xq)[PX], double (&qv)[PX], int gs, double& E, int& par)
      __attribute__((always_inline)) -> double {
    const double* e = gs < NWHITE ? mhw + 4 * gs : mhh + 4 * (gs - NWHITE);
    par = (int)e[0];
    const double delta = e[1];
    E = e[3];
#pragma unroll
    for (int j = 0; j < PX; ++j) qv[j] = (j == par) ? xq[j] + delta : xq[j];
    return e[2];
  };

  // ---------------- matrix state ----------------
  double L[NSL];
  double ld_tm_m = 1.0, quad_tm = 0.0, logdetN = 0.0, rNr = 0.0;
  double tm_apr = 1.0, tm_zr = 0.0;       // timing-model columns' pivots / aug entries
  double f_apr[2] = {1.0, 1.0}, f_zr[2] = {0.0, 0.0};  // last factorisation's
  int ld_tm_e = 0, fail_tm = 0;

  // SVD noise floor f of this sweep's b draw (floor_shift; 0 except on the floor redo)
  double fshift = 0.0;
  // Gram: G = T_aug^T diag(1/N) T_aug on fp64 MFMA, then TM elimination -> S0.
  auto gram_and_tm = [&](const double (&xq)[PX]) __attribute__((always_inline)) {
    const double ef2 = efac2_of(xq);
    const double Q = exp(2.0 * pget(xq, md.idx_equad) * 2.302585092994045684);
    double sr = 0.0;
    LogProd lp;
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      const int t = 64 * s + lane;
      double w = 0.0;
      if (vmask & (1u << s)) {
        double N0;
        if constexpr (GEN)
          N0 = gen_n0(xq, S2(s), gef[s], geq[s]);
        else
          N0 = ef2 * S2(s) + Q;
        const double N = ((zb >> s) & 1u ? al[s] : 1.0) * N0;
        lp.mul(N);
        const double rs = RR(s);
        sr += rs * rs / N;
        w = 1.0 / N;
      }
      vbuf[t] = w;
    }
    logdetN = wave_sum(lp.log_sum());
    rNr = wave_sum(sr);
    lds_order();
    GST_SUB_BEGIN
    // Low-rank Gram (one backend, <= 8 noise classes, at most LR_MAX flagged TOAs): the
    // weights are c_k (1 / alpha_t)^z_t with c_k = 1 / N0 of the TOA's noise class, so
    //   G = sum_k c_k G_k + sum_{t: z_t = 1} c_k(t) (1 / alpha_t - 1) [T|r]_t [T|r]_t^T
    // with the per-class Grams G_k of the dataset (DevModel::Gcls) -- the same T^T N^-1 [T|r]
    // (gibbs.py:302-304) at a cost of the class terms plus one rank-1 update per flagged TOA
    // instead of the MFMA Gram over all n TOAs (config 2: ~7 flagged of 130).
    // Taken only while every flagged TOA's alpha is at most LR_ALPHA_MAX: the rank-1 terms
    // subtract c_k (1 - 1 / alpha_t) of a class Gram's share, so a direction fixed by flagged
    // TOAs alone keeps an absolute error ~eps c_k |row|^2 against its true c_k |row|^2 / alpha_t
    // (relative ~eps alpha_t); past the bound (vvh17's fixed alpha = 1e10) the MFMA Gram runs.
    int nout = 0;
    bool big = false;
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      nout += __popcll(__ballot(((zb & vmask) >> s) & 1u));
      big = big || ((((zb & vmask) >> s) & 1u) && al[s] > LR_ALPHA_MAX);
    }
    if (md.Gcls && nout <= LR_MAX && !(st.debug & DEBUG_MFMA_GRAM) && __ballot(big) == 0ull) {
      __hip_atomic_fetch_add(&gcnt[wv][0], lane == 0 ? 1u : 0u, __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_WAVEFRONT);
#pragma unroll
      for (int i = 0; i < SL(MT, 0); ++i) L[i] = 0.0;
#pragma unroll 1
      for (int k = 0; k < md.ncls; ++k) {
        const double ck = 1.0 / (GEN ? cls_n0(xq, k) : ef2 * md.csig2[k] + Q);
        const GDouble* gk = (const GDouble*)md.Gcls + (size_t)k * SL(MT, 0) * 64 + lane;
#pragma unroll
        for (int i = 0; i < SL(MT, 0); ++i) L[i] = fma(ck, gk[64 * i], L[i]);
      }
      // flagged TOAs, one rank-1 update each: c_k (1 / alpha_t - 1) = w_t - c_k, with the
      // weight w_t = 1 / N_t the loop above left in vbuf
#pragma unroll 1
      for (int s = 0; s < NS; ++s) {
        unsigned long long bm = __ballot(((zb & vmask) >> s) & 1u);
#pragma unroll 1
        while (bm) {
          const int t = 64 * s + __builtin_ctzll(bm);
          bm &= bm - 1;
          const int k = md.ncls > 1 ? md.cidx[t] : 0;
          const double v = vbuf[t] - 1.0 / (GEN ? cls_n0(xq, k) : ef2 * md.csig2[k] + Q);
          // [T|r]_t at internal columns 8 r + p (row side) and 8 r + q (column side): each
          // lane's MT entries are contiguous in Trow ([t][i % 8][i / 8]), 128-bit loads
          typedef double v2_t __attribute__((ext_vector_type(2)));
          const GDouble* tr = (const GDouble*)md.Trow + (size_t)t * 8 * MT;
          const __attribute__((address_space(1))) v2_t* trp =
              (const __attribute__((address_space(1))) v2_t*)(tr + MT * p);
          const __attribute__((address_space(1))) v2_t* trq =
              (const __attribute__((address_space(1))) v2_t*)(tr + MT * q);
          double tp_[MT], tq_[MT];
#pragma unroll
          for (int r = 0; r < MT; r += 2) {
            const v2_t a = trp[r / 2], b = trq[r / 2];
            tp_[r] = a[0];
            tp_[r + 1] = a[1];
            tq_[r] = b[0];
            tq_[r + 1] = b[1];
          }
#pragma unroll
          for (int r = 0; r < MT; ++r) {
            const double vr = v * tp_[r];
#pragma unroll
            for (int s2 = 0; s2 <= r; ++s2) L[SL(r, s2)] = fma(vr, tq_[s2], L[SL(r, s2)]);
          }
        }
      }
      GST_SUB_END(9)
    } else {
    __hip_atomic_fetch_add(&gcnt[wv][1], lane == 0 ? 1u : 0u, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_WAVEFRONT);
    if constexpr (PAIR) {
    // Two waves per chain (PAIR): wave 0 computes the
    // even Gram tiles, wave 1 the odd ones (each its own MFMA pipe), then the tiles are swapped
    // through the two waves' stage-scratch regions (4 tiles per wave per round, 2 rounds)
    // and both waves hold the whole Gram, bitwise the single wave's (same MFMA sequence per
    // tile).
    auto gram_tiles = [&](auto own_c) __attribute__((always_inline)) {
      constexpr int OWN = decltype(own_c)::value;
      auto mine = [](int T) { return OWN == 0 || (T & 1) == OWN - 1; };
      v4d acc[NTT];
#pragma unroll
      for (int i = 0; i < NTT; ++i) acc[i] = (v4d){0.0, 0.0, 0.0, 0.0};
      const int tl = lane >> 4;
      // two k-steps in flight: each operand set is reloaded (for k-step ks + 2) right after
      // its MFMAs have issued, so a T load has two k-steps (30 MFMAs) to arrive from L2
      double ta[NT], tb[NT], wa, wb;
      auto tload = [&](double (&t)[NT], double& w, int ks) __attribute__((always_inline)) {
        const GDouble* src = (const GDouble*)md.Tmf + (size_t)ks * NT * 64;
#pragma unroll
        for (int X = 0; X < NT; ++X) t[X] = src[X * 64 + lane];
        w = vbuf[4 * ks + tl];
      };
      auto kstep = [&](const double (&t)[NT], const double wt) __attribute__((always_inline)) {
#pragma unroll
        for (int I = 0; I < NT; ++I) {
          const double av = t[I] * wt;
#pragma unroll
          for (int J = 0; J <= I; ++J) {
            const int T = I * (I + 1) / 2 + J;
            if (mine(T)) acc[T] = __builtin_amdgcn_mfma_f64_16x16x4f64(av, t[J], acc[T], 0, 0, 0);
          }
        }
      };
      // an even number of k-steps (Tmf and the weights are zero past n: a padding k-step
      // adds exact zeros), so the loop body has no conditional load and the wait before a
      // set's MFMAs covers only that set (a branch in the body made the compiler wait for
      // both sets at the top of every iteration); the scheduling barriers keep the order
      const int nksp = (md.nks + 1) & ~1;
      tload(ta, wa, 0);
      tload(tb, wb, 1);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll 1
      for (int ks = 0; ks + 2 < nksp; ks += 2) {
        kstep(ta, wa);
        tload(ta, wa, ks + 2);
        __builtin_amdgcn_sched_barrier(0);
        kstep(tb, wb);
        tload(tb, wb, ks + 3);
        __builtin_amdgcn_sched_barrier(0);
      }
      kstep(ta, wa);
      kstep(tb, wb);
      GST_SUB_END(9)
      // MFMA C layout (col = lane&15, row = lane>>4 + 4 reg) -> cyclic register layout
      if constexpr (OWN == 0) {
#pragma unroll
        for (int I = 0; I < NT; ++I) {
#pragma unroll
          for (int J = 0; J <= I; ++J) {
            const v4d a = acc[I * (I + 1) / 2 + J];
#pragma unroll
            for (int g = 0; g < 4; ++g) tbuf[(tl + 4 * g) * TB_LD + (lane & 15)] = a[g];
            lds_order();
#pragma unroll
            for (int dr = 0; dr < 2; ++dr)
#pragma unroll
              for (int ds = 0; ds < 2; ++ds) {
                const int r = 2 * I + dr, s = 2 * J + ds;
                if (r >= s) L[SL(r, s)] = tbuf[(8 * dr + p) * TB_LD + 8 * ds + q];
              }
            lds_order();
          }
        }
      } else {
        constexpr int TS = 16 * TB_LD;  // one padded tile
        static_assert(4 * TS <= s0r_doubles(MT, K0), "tile swap exceeds the stage scratch");
#pragma unroll
        for (int rnd = 0; rnd < 2; ++rnd) {
#pragma unroll
          for (int I = 0; I < NT; ++I)
#pragma unroll
            for (int J = 0; J <= I; ++J) {
              const int T = I * (I + 1) / 2 + J;
              if ((T >> 3) == rnd && mine(T)) {
                double* dst = smem[OWN - 1] + ((T >> 1) & 3) * TS;
#pragma unroll
                for (int g = 0; g < 4; ++g) dst[(tl + 4 * g) * TB_LD + (lane & 15)] = acc[T][g];
              }
            }
          __syncthreads();
#pragma unroll
          for (int I = 0; I < NT; ++I)
#pragma unroll
            for (int J = 0; J <= I; ++J) {
              const int T = I * (I + 1) / 2 + J;
              if ((T >> 3) != rnd) continue;
              const double* src = smem[T & 1] + ((T >> 1) & 3) * TS;
#pragma unroll
              for (int dr = 0; dr < 2; ++dr)
#pragma unroll
                for (int ds = 0; ds < 2; ++ds) {
                  const int r = 2 * I + dr, s = 2 * J + ds;
                  if (r >= s) L[SL(r, s)] = src[(8 * dr + p) * TB_LD + 8 * ds + q];
                }
            }
          __syncthreads();
        }
      }
    };
      if (role == 0)
        gram_tiles(std::integral_constant<int, 1>{});
      else
        gram_tiles(std::integral_constant<int, 2>{});
    } else {
    v4d acc[NTT];
#pragma unroll
    for (int i = 0; i < NTT; ++i) acc[i] = (v4d){0.0, 0.0, 0.0, 0.0};
    const int tl = lane >> 4;
    // two k-steps in flight: each operand set is reloaded (for k-step ks + 2) right after
    // its MFMAs have issued, so a T load has two k-steps (30 MFMAs) to arrive from L2
    double ta[NT], tb[NT], wa, wb;
    auto tload = [&](double (&t)[NT], double& w, int ks) __attribute__((always_inline)) {
      const GDouble* src = (const GDouble*)md.Tmf + (size_t)ks * NT * 64;
#pragma unroll
      for (int X = 0; X < NT; ++X) t[X] = src[X * 64 + lane];
      w = vbuf[4 * ks + tl];
    };
    auto kstep = [&](const double (&t)[NT], const double wt) __attribute__((always_inline)) {
#pragma unroll
      for (int I = 0; I < NT; ++I) {
        const double av = t[I] * wt;
#pragma unroll
        for (int J = 0; J <= I; ++J) {
          acc[I * (I + 1) / 2 + J] =
              __builtin_amdgcn_mfma_f64_16x16x4f64(av, t[J], acc[I * (I + 1) / 2 + J], 0, 0, 0);
        }
      }
    };
    // an even number of k-steps (Tmf and the weights are zero past n: a padding k-step
    // adds exact zeros), so the loop body has no conditional load and the wait before a
    // set's MFMAs covers only that set (a branch in the body made the compiler wait for
    // both sets at the top of every iteration); the scheduling barriers keep the order
    const int nksp = (md.nks + 1) & ~1;
    tload(ta, wa, 0);
    tload(tb, wb, 1);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll 1
    for (int ks = 0; ks + 2 < nksp; ks += 2) {
      kstep(ta, wa);
      tload(ta, wa, ks + 2);
      __builtin_amdgcn_sched_barrier(0);
      kstep(tb, wb);
      tload(tb, wb, ks + 3);
      __builtin_amdgcn_sched_barrier(0);
    }
    kstep(ta, wa);
    kstep(tb, wb);
    GST_SUB_END(9)
    // MFMA C layout (col = lane&15, row = lane>>4 + 4 reg) -> cyclic register layout
#pragma unroll
    for (int I = 0; I < NT; ++I) {
#pragma unroll
      for (int J = 0; J <= I; ++J) {
        const v4d a = acc[I * (I + 1) / 2 + J];
#pragma unroll
        for (int g = 0; g < 4; ++g) tbuf[(tl + 4 * g) * TB_LD + (lane & 15)] = a[g];
        lds_order();
#pragma unroll
        for (int dr = 0; dr < 2; ++dr)
#pragma unroll
          for (int ds = 0; ds < 2; ++ds) {
            const int r = 2 * I + dr, s = 2 * J + ds;
            if (r >= s) L[SL(r, s)] = tbuf[(8 * dr + p) * TB_LD + 8 * ds + q];
          }
        lds_order();
      }
    }
    }
    }
    // timing-model prior (1/tm_weight) on its diagonal; unit pivots on the pad columns
#pragma unroll
    for (int s = 0; s < K0; ++s) {
      const int j = 8 * s + q;
      if (p == q) L[SL(s, s)] = (j < md.ntm) ? (L[SL(s, s)] + md.tm_phiinv) + fshift : 1.0;
    }
    CholCtx cc{colq, phbuf, colq2, lane, p, q, raug, 1.0, 0.0, 0, 0, {1.0, 1.0}, {0.0, 0.0}};
    GST_SUB_END(10)
    chol_range_lean<MT, 0, 8 * K0>(L, cc);
    chol_harvest<MT, 0, 8 * K0, RA>(L, cc);
    chol_stats<0, 8 * K0>(cc);
    GST_SUB_END(11)
    tm_apr = cc.apr[0];
    tm_zr = cc.zr[0];
    ld_tm_m = cc.mant;
    ld_tm_e = cc.expo;
    quad_tm = cc.quad;
    fail_tm = cc.fail;
#pragma unroll
    for (int r = K0; r < MT; ++r)
#pragma unroll
      for (int s = K0; s <= r; ++s) S0[64 * SL(r - K0, s - K0)] = L[SL(r, s)];
    // the frozen timing-model columns: parked in global scratch until the b draw
#pragma unroll
    for (int s = 0; s < K0; ++s)
#pragma unroll
      for (int r = s; r < MT; ++r) lr_store(tmf, 512 * tm_slot(MT, r, s), L[SL(r, s)]);
  };

  // log f_k and log df_k of this lane's Fourier column (f = lane; every instance has
  // RA - ntm_pad <= 64), held for the launch: loaded from global memory inside every
  // likelihood they put an L2 round trip in front of each MH step's phi computation
  static_assert(RA - 8 * K0 <= 64, "one Fourier column per lane");
  const bool f_live = lane < RA - md.ntm_pad && lane < md.nf;
  const double lfreq_l = f_live ? md.lfreq[lane] : 0.0;
  const double ldf_l = f_live ? md.ldf[lane] : 0.0;
  // GEN: the ECORR epoch columns follow the Fourier block (lanes nf .. nf + nec - 1); the
  // lane's ecorr parameter index, or -1
  int geci = -1;
  if constexpr (GEN) {
    const int e = lane - md.nf;
    if (e >= 0 && e < md.nec && lane < RA - md.ntm_pad) geci = md.ecorr_b[md.ecb[e]];
  }

  // b-marginalised likelihood at xq (gibbs.py:288-329); factor left in L.
  // the descriptor scalars of lnl_hyper, read once for the launch (wave-uniform: scalar
  // registers), not at each of the ~11 calls per sweep
  const int hidxA = md.idx_logA, hidxg = md.idx_gamma, hntmp = md.ntm_pad, hnf = md.nf;
  const double hl12 = md.log_12pi2, hlfyr = md.log_fyr, hslf = md.sum_lfreq,
               hsldf = md.sum_ldf, hldtm = md.logdet_phi_tm;
  auto lnl_hyper = [&](const double (&xq)[PX], int& failed) __attribute__((always_inline)) -> double {
    GST_COUNT(16)
    GST_SUB_BEGIN
    const double lA = pget(xq, hidxA);
    const double g = pget(xq, hidxg);
    // log phi_k = 2 lA ln10 - log(12 pi^2) + (g-3) log fyr - g log f_k + log df_k
    const double lc = 2.0 * lA * 2.302585092994045684 - hl12 + (g - 3.0) * hlfyr;
    // S0 first: its 36 LDS loads are in flight while phi^-1 is computed (exp)
#pragma unroll
    for (int r = K0; r < MT; ++r)
#pragma unroll
      for (int s = K0; s <= r; ++s) L[SL(r, s)] = S0[64 * SL(r - K0, s - K0)];
    // Fourier columns, then the unit-prior dummies that pad a smaller model up to this
    // instance's RA (zero Gram rows: each is eliminated as an exact no-op)
    if constexpr (GEN) {
      // ECORR column of backend b: phi = 10^(2 ecorr_b) (as the large path, gst_large.hpp)
      if (lane < RA - hntmp)
        phbuf[hntmp + lane] =
            f_live ? exp(-(lc - g * lfreq_l + ldf_l)) + fshift
                   : (geci >= 0 ? exp(-2.0 * pget(xq, geci) * 2.302585092994045684) + fshift : 1.0);
    } else {
      if (lane < RA - hntmp)
        phbuf[hntmp + lane] = f_live ? exp(-(lc - g * lfreq_l + ldf_l)) + fshift : 1.0;
    }
    // phbuf doubles as the eliminations' junk rows: restore the one other entry read
    // below, the augmented row's (no prior on the residual column)
    if (lane == 63) phbuf[raug] = 0.0;
    // sum_k log phi_k in closed form (no reduction on the critical path)
    double logdet_phi = ((double)hnf * lc - g * hslf + hsldf) + hldtm;
    if constexpr (GEN) {
      for (int b = 0; b < md.nb; ++b)   // log 10^(2 ecorr_b) per ECORR column of backend b
        if (md.ec_count[b] > 0.0)
          logdet_phi += md.ec_count[b] * (2.0 * pget(xq, md.ecorr_b[b]) * 2.302585092994045684);
    }
    lds_order();
#pragma unroll
    for (int r = K0; r < MT; ++r)
      if (p == q) L[SL(r, r)] += phbuf[8 * r + p];
    CholCtx cc{colq, phbuf, colq2, lane, p, q, raug, 1.0, 0.0, 0, 0, {tm_apr, 1.0}, {tm_zr, 0.0}};
    GST_SUB_END(7)
    chol_range<MT, K0, RA, kp_for(OCC)>(L, cc);
    GST_SUB_END(8)
    chol_harvest<MT, 8 * K0, RA, RA>(L, cc);
    chol_stats<8 * K0, RA>(cc);
    GST_SUB_END(19)
    f_apr[0] = cc.apr[0];
    f_apr[1] = cc.apr[1];
    f_zr[0] = cc.zr[0];
    f_zr[1] = cc.zr[1];
    const double mant = cc.mant, quad = cc.quad;
    const int expo = cc.expo;
    failed = cc.fail | fail_tm;
    if (failed) return -INFINITY;
    // log|Sigma| = sum log a_kk (pivots of the LDL^T-scaled elimination)
    const double ld_sigma = log(ld_tm_m * mant) + (double)(ld_tm_e + expo) * 0.693147180559945309417;
    double ll = -0.5 * (logdetN + rNr);
    ll += 0.5 * ((quad_tm + quad) - ld_sigma - logdet_phi);
    return ll;
  };

  // pair mode: both waves write the records (identical state): b and the TOA slots split
  const bool rec_on = record_every > 0 && !eval_only && (PAIR || role == 0);
  int hacc = 0, hrej = 0;   // pair mode: hyper-MH acceptance history (branch prediction)
  GST_STAMP_START
  compute_Tb();
  if (eval_only) nsweeps = 1;

#pragma unroll 1
  for (int it = 0; it < nsweeps; ++it) {
    if (OCC == 2 && st.prog) {
      // last sweep's ticket (arrived long ago): behind if fewer sweeps than the average
      if (it > 0) {
        const unsigned long long g = __builtin_amdgcn_readfirstlane((unsigned)prog_ret) |
                                     ((unsigned long long)__builtin_amdgcn_readfirstlane(
                                          (unsigned)(prog_ret >> 32)) << 32);
        fair.behind = (unsigned long long)(it - 1) * (unsigned long long)C < g ? 1 : 0;
      }
      // (this sweep's ticket is taken after its Gram, gram_and_tm's caller below)
    }
    fair_prio<OCC>(fair);
    rng.sweep = (uint32_t)(sweep0 + it);
    const double* tp = TAPE ? tape.data + ((size_t)c * nsweeps + it) * tape.stride : nullptr;
    if (st.debug & 1) {
      // GST_DEBUG_POISON: between two sweeps a chain's state is exactly what the records
      // hold (x, b, z, alpha, pout, theta, nu; y = r - T b and the z bits in registers are
      // functions of it), so every LDS word of the chain and its parked timing-model factor
      // are dead here.  Overwrite them with a NaN pattern: a sweep that read any of them
      // before writing it would carry the NaN into its draws, and the chains would no longer
      // be bitwise those of an ordinary launch (tests/test_gpu_invariants.py).
      const double poison = __longlong_as_double(0x7ff4dead7ff4deadll);
      for (int j = lane; j < lds_doubles(MT, K0); j += 64) smem[wv][j] = poison;
      for (int j = 0; j < NTMS; ++j) lr_store(tmf, 512 * j, poison);
      lds_order();
    }

    // ---- record the state at the start of the sweep (gibbs.py:355-361)
    if (rec_on && (it % record_every) == 0) {
      const int ri = it / record_every;
      if (ri < rec.nrec) {
        const size_t base = (size_t)c * rec.nrec + ri;
        if (rec.x && lane < P && role == 0) rec.x[base * P + lane] = pget(xv, lane);
        // from the state row, not bsc: bsc shares S0R with S0 and is stale after a sweep
        // that skipped the b draw (gibbs.py:373)
        if (rec.b)
          for (int j = lane + 64 * role; j < m; j += (PAIR ? 128 : 64)) rec.b[base * m + j] = brow[j];
#pragma unroll
        for (int s = 0; s < NS; ++s) {
          const int t = 64 * s + lane;
          if ((vmask & (1u << s)) && (!PAIR || (s & 1) == role)) {
            if (rec.z) rec.z[base * nst + t] = (double)((zb >> s) & 1u);
            if (rec.alpha) rec.alpha[base * nst + t] = al[s];
            if (rec.pout) rec.pout[base * nst + t] = po[s];
          }
        }
        if (lane == 0 && role == 0) {
          if (rec.theta) rec.theta[base] = theta;
          if (rec.nu) rec.nu[base] = nu;
        }
      }
    }

    const double x_last0 = pget(xv, P - 1);  // chain[ii, -1]
    GST_SUB_BEGIN
    if (!eval_only) mh_variates(tp);
    GST_SUB_END(20)
    GST_STAMP(0)

    // ---- white-noise MH block (gibbs.py:114-143); step -1 = the initial lnlike0
    if ((mask & 1u) && !eval_only && !GEN && md.ncls > 0) {
      // Noise-class path: a likelihood is a few scalar ops (no TOA reduction), so the
      // block is a serial chain of log/divide latencies.  Evaluate it speculatively:
      // for the next D steps, lane 2^j - 1 + b evaluates step s0+j's proposal on the
      // accept/reject path b (bit i = step s0+i accepted); the decisions are then read
      // back lane by lane.  Every value is computed with the sequential code's exact
      // operation order, so the decisions and the final state are bitwise identical.
      GST_SUB_BEGIN
      white_prep();
      GST_SUB_END(21)
      constexpr int D = 6;
      double Wu[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) Wu[u] = (u < md.ncls) ? rdlane(wcls, u) : 0.0;
      auto lnl_lane = [&](const double (&xq)[PX], double Q) __attribute__((always_inline)) -> double {
        const double ef2 = efac2_of(xq);
        if (md.ncls == 1) {
          const double N0 = ef2 * md.csig2[0] + Q;
          return -0.5 * ((wcls_la + md.ccount[0] * log(N0)) + Wu[0] / N0);
        }
        double sl = 0.0, sq = 0.0;
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          if (u < md.ncls) {
            const double N0 = ef2 * md.csig2[u] + Q;
            sl += md.ccount[u] * log(N0);
            sq += Wu[u] / N0;
          }
        }
        return -0.5 * ((sl + wcls_la) + sq);
      };
      const int ieq = md.idx_equad;
      double Qx = exp(2.0 * pget(xv, ieq) * 2.302585092994045684);
      double l0 = lnl_lane(xv, Qx), p0 = lnprior(xv);
      // this lane's node: level j, path b
      const int node = lane + 1;
      const int j = 31 - __builtin_clz(node);          // node in [2^j, 2^(j+1))
      const int b = node - (1 << j);
#pragma unroll 1
      for (int s0 = 0; s0 < NWHITE; s0 += D) {
        const int nd = (NWHITE - s0) < D ? (NWHITE - s0) : D;
        GST_SUB_BEGIN
        // the round's D steps (parameter, delta, log u, 10^(2 delta)) in registers: every
        // LDS load issues up front, and each lane's walk down its path is straight-line
        // selects instead of a divergent loop of dependent loads
        int pr[D];
        double dl[D], lu[D], ev[D];
#pragma unroll
        for (int i = 0; i < D; ++i) {
          const int gs = (s0 + i) < NWHITE ? s0 + i : NWHITE - 1;
          pr[i] = (int)mhw[4 * gs + 0];
          dl[i] = mhw[4 * gs + 1];
          lu[i] = mhw[4 * gs + 2];
          ev[i] = mhw[4 * gs + 3];
        }
        double xq[PX], Q = Qx;
#pragma unroll
        for (int t = 0; t < PX; ++t) xq[t] = xv[t];
#pragma unroll
        for (int i = 0; i < D - 1; ++i) {
          const bool on = i < j && ((b >> i) & 1);
#pragma unroll
          for (int t = 0; t < PX; ++t) xq[t] = (on && t == pr[i]) ? xq[t] + dl[i] : xq[t];
          Q = (on && pr[i] == ieq) ? Q * ev[i] : Q;
        }
        // the proposal of step s0 + j from the node's state (propose(): q[par] += delta)
        int par = pr[0];
        double delta = dl[0], E = ev[0];
#pragma unroll
        for (int i = 1; i < D; ++i) {
          par = j == i ? pr[i] : par;
          delta = j == i ? dl[i] : delta;
          E = j == i ? ev[i] : E;
        }
        double qv[PX];
#pragma unroll
        for (int t = 0; t < PX; ++t) qv[t] = (t == par) ? xq[t] + delta : xq[t];
        double p1 = -INFINITY, l1 = 0.0;
        if (j < nd) {
          const double Qq = (par == ieq) ? Q * E : Q;
          p1 = lnprior(qv);
          if (p1 != -INFINITY) l1 = lnl_lane(qv, Qq);
        }
        GST_SUB_END(22)
        int path = 0;
#pragma unroll
        for (int jj = 0; jj < D; ++jj) {
          if (jj < nd) {
            const int L = (1 << jj) - 1 + path;
            const double pl = rdlane(p1, L);
            const double ll = rdlane(l1, L);
            if (pl != -INFINITY && (ll + pl) - (l0 + p0) > lu[jj]) {
              l0 = ll;
              p0 = pl;
              path |= 1 << jj;
            }
          }
        }
        GST_SUB_END(15)
        // apply the accepted moves in order (the sequential code's xv = qv, Qx = Qq)
#pragma unroll
        for (int i = 0; i < D; ++i) {
          const bool on = i < nd && ((path >> i) & 1);
#pragma unroll
          for (int t = 0; t < PX; ++t) xv[t] = (on && t == pr[i]) ? xv[t] + dl[i] : xv[t];
          Qx = (on && pr[i] == ieq) ? Qx * ev[i] : Qx;
        }
      }
    } else if ((mask & 1u) || eval_only) {
      white_prep();
      double l0 = 0.0, p0 = 0.0;
      double Qx = exp(2.0 * pget(xv, hieq) * 2.302585092994045684);
#pragma unroll 1
      for (int step = -1; step < NWHITE; ++step) {
        if ((step & 3) == 0) fair_prio<OCC>(fair);
        double qv[PX], luacc = 0.0, Qq = Qx;
        if (step < 0) {
#pragma unroll
          for (int j = 0; j < PX; ++j) qv[j] = xv[j];
        } else {
          double E;
          int par;
          luacc = propose(xv, qv, step, E, par);
          if (par == hieq) Qq = Qx * E;
        }
        const double p1 = lnprior(qv);
        // out-of-prior: (l1 + -inf) - (l0 + p0) is -inf or NaN, never > log(u): skip lnL
        if (step >= 0 && p1 == -INFINITY) continue;
        GST_SUB_BEGIN
        const double l1 = lnl_white(qv, Qq);
        GST_SUB_END(15)
        if (step < 0) {
          l0 = l1;
          p0 = p1;
          if (eval_only) {
            if (lane == 0) out_w[c] = l1;
            break;
          }
          continue;
        }
        if ((l1 + p1) - (l0 + p0) > luacc) {
#pragma unroll
          for (int j = 0; j < PX; ++j) xv[j] = qv[j];
          l0 = l1;
          p0 = p1;
          Qx = Qq;
        }
      }
    }

    GST_STAMP(1)
    // ---- Gram + red-noise hyper MH block (gibbs.py:80-111, 288-329) + b draw (145-182)
    // step -1: initial lnlike0; steps 0..9: proposals; step NHYPER: refactor at the final
    // x for the b draw when the factor left in registers belongs to a rejected proposal.
    bool redraw = false;
    int fb = 0;
    int owner = 0;   // the wave whose registers hold the factor at the final x (pair mode)
    if constexpr (PAIR) {
      if (mask & 6u) {
        double l0 = 0.0, p0 = 0.0;
        owner = -1;
        bool init = (mask & 2u) != 0;
        int j = init ? 0 : NHYPER, rp = 0;
        // first step >= s whose proposal from xb is inside the prior (the others are
        // rejected without a likelihood, gibbs.py:100-104 with lnprior = -inf)
        auto next_in = [&](const double (&xb)[PX], int s) __attribute__((always_inline)) -> int {
          for (; s < NHYPER; ++s) {
            double qv[PX], E;
            int par;
            (void)propose(xb, qv, NWHITE + s, E, par);
            if (lnprior(qv) != -INFINITY) break;
          }
          return s;
        };
        // one sequential MH step (gibbs.py:99-110) at step s with the lnL of its point
        auto decide = [&](int s, double l1, bool f1, int who) __attribute__((always_inline)) {
          if (f1) status |= 1;
          double qv[PX], E;
          int par;
          const double luacc = propose(xv, qv, NWHITE + s, E, par);
          const double p1 = lnprior(qv);
          if ((l1 + p1) - (l0 + p0) > luacc) {
            GST_COUNT(18)
#pragma unroll
            for (int t = 0; t < PX; ++t) xv[t] = qv[t];
            l0 = l1;
            p0 = p1;
            owner = who;
            ++hacc;
            return true;
          }
          owner = -1;
          ++hrej;
          return false;
        };
        // pass 1 (rare): the b draw's factor at the SVD noise floor, Sigma + f I (floor_shift)
#pragma unroll 1
        for (int pass = 0; pass < 2; ++pass) {
        gram_and_tm(xv);   // both waves: identical S0 in each wave's own LDS region
        if (fail_tm) status |= 1;
        GST_STAMP(2)
        // Each round wave 0 evaluates the next point the sequential sampler needs (the
        // initial x, then the next in-prior proposal sa) and wave 1 a speculative one: the
        // step after sa on the branch (accept / reject) the chain's acceptance history
        // predicts, else on the other branch, else -- no proposal left -- the current x
        // (the reject branch's final state, for the b draw).  A last round refactors the
        // final x when no wave holds its factor and the b draw needs it.
#pragma unroll 1
        while (true) {
          const int sa = init ? -1 : next_in(xv, j);
          bool fin = false;
          if (sa >= NHYPER) {
            if (!(mask & 4u)) break;
            redraw = true;
#pragma unroll
            for (int t = 0; t < PX; ++t)
              if (t < P) redraw = redraw && (xv[t] != x_last0);      // gibbs.py:373
            if (mask & 128u) redraw = true;
            if (!redraw || owner >= 0) break;
            fin = true;
          }
          double qa[PX];
#pragma unroll
          for (int t = 0; t < PX; ++t) qa[t] = xv[t];
          int kind = 0, sb = NHYPER;   // wave 1: 0 idle, 1 accept branch, 2 reject branch, 3 x
          if (!fin) {
            if (!init) {
              double E;
              int par;
              (void)propose(xv, qa, NWHITE + sa, E, par);
            }
            const int sbR = next_in(xv, sa + 1);
            const int sbA = init ? NHYPER : next_in(qa, sa + 1);
            if (!init && hacc >= hrej && sbA < NHYPER) {
              kind = 1;
              sb = sbA;
            } else if (sbR < NHYPER) {
              kind = 2;
              sb = sbR;
            } else if (!init && (mask & 4u) && owner != 1) {
              kind = 3;
            }
          }
          double xq[PX];
#pragma unroll
          for (int t = 0; t < PX; ++t) xq[t] = role == 0 ? qa[t] : xv[t];
          if (role == 1 && (kind == 1 || kind == 2)) {
            double E;
            int par;
            (void)propose(kind == 1 ? qa : xv, xq, NWHITE + sb, E, par);
          }
          GST_COUNT(17)
          double lm = 0.0;
          int fm = 0;
          if (role == 0 || kind != 0) lm = lnl_hyper(xq, fm);
          if (lane == 0) {
            xchg[rp][role][0] = lm;
            xchg[rp][role][1] = (double)fm;
          }
          __syncthreads();
          const double lA = xchg[rp][0][0], lB = xchg[rp][1][0];
          const bool fA = xchg[rp][0][1] != 0.0, fB = xchg[rp][1][1] != 0.0;
          rp ^= 1;   // the next round writes the other buffer: no second barrier needed
          if (fin) {
            fb = fA;
            owner = 0;
            break;
          }
          const int prev = owner;
          if (init) {
            if (fA) status |= 1;
            l0 = lA;
            p0 = lnprior(xv);
            owner = fA ? -1 : 0;
            init = false;
            j = NHYPER;
            if (kind == 2) {
              decide(sb, lB, fB, 1);
              j = sb + 1;
            }
          } else if (decide(sa, lA, fA, 0)) {
            j = sa + 1;
            if (kind == 1) {
              decide(sb, lB, fB, 1);
              j = sb + 1;
            }
          } else {
            j = sa + 1;
            if (kind == 2) {
              decide(sb, lB, fB, 1);
              j = sb + 1;
            } else if (kind == 3) {
              owner = fB ? -1 : 1;
            } else if (kind == 0 && prev == 1) {
              owner = 1;   // wave 1 sat out: its factor of x is intact
            }
          }
        }
        if (pass == 1 || !redraw || fb || (st.debug & DEBUG_EXACT_BDRAW)) break;
        // the owner wave holds the factor at the final x; both waves take its floor decision
        const double fs =
            role == owner ? floor_shift(f_apr, lane, md.ntm, md.ntm_pad, md.ntm_pad + md.nf + (GEN ? md.nec : 0)) : 0.0;
        if (role == owner && lane == 0) xfloor[0] = fs;
        __syncthreads();
        fshift = xfloor[0];
        __syncthreads();
        if (fshift == 0.0) break;
        status |= STATUS_FLOOR;
        ++nfloor;
        owner = -1;   // a final round refactors x (the MH decisions stand)
        init = false;
        j = NHYPER;
        }
        fshift = 0.0;
      }
    } else if ((mask & (6u | 256u)) || eval_only) {
      bool Lvalid = false;
      double l0 = 0.0, p0 = 0.0;
      // GST_STAGE_GRAM (256, timing diagnostic): the Gram and the timing-model elimination only
      const int first = (mask & 256u) ? NHYPER + 1 : (((mask & 2u) || eval_only) ? -1 : NHYPER);
      // pass 1 (rare): the registers hold the factor at the final x and Sigma is beyond fp64
      // resolution -- refactor x's Sigma + f I for the b draw (floor_shift; the MH decisions
      // stand).  One copy of the Gram / hyper-block code serves both passes (an inlined
      // second copy of it raised the 256-register build's spill)
#pragma unroll 1
      for (int pass = 0; pass < 2; ++pass) {
      gram_and_tm(xv);
      // the sweep's progress ticket (fair_prio), issued where only LDS and register work
      // follows (the hyper MH): its return is awaited at the next sweep's start instead of by
      // the next global load (taken at the sweep's start, the atomic's latency stalled the
      // record / MH-variate stage; round-5 A/B: 20-sweep line +1%, 500 sweeps unchanged)
      if (OCC == 2 && st.prog && pass == 0 && lane == 0)
        prog_ret = __hip_atomic_fetch_add(st.prog, 1ull, __ATOMIC_RELAXED,
                                          __HIP_MEMORY_SCOPE_AGENT);
      if (fail_tm) status |= 1;
      GST_STAMP(2)
#pragma unroll 1
      for (int step = pass ? NHYPER : first; step <= NHYPER; ++step) {
        fair_prio<OCC>(fair);
        double qv[PX], luacc = 0.0;
        if (step == NHYPER) {
          if (eval_only || !(mask & 4u)) break;
          redraw = true;
#pragma unroll
          for (int j = 0; j < PX; ++j)
            if (j < P) redraw = redraw && (xv[j] != x_last0);   // gibbs.py:373
          if (mask & 128u) redraw = true;                        // direct update_b call
          if (!redraw || Lvalid) break;
        }
        if (step < 0 || step == NHYPER) {
#pragma unroll
          for (int j = 0; j < PX; ++j) qv[j] = xv[j];
        } else {
          double E;
          int par;
          luacc = propose(xv, qv, NWHITE + step, E, par);
        }
        const double p1 = lnprior(qv);
        if (step >= 0 && step < NHYPER && p1 == -INFINITY) continue;
        int f1 = 0;
        const double l1 = lnl_hyper(qv, f1);
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
          if (eval_only) {
            if (lane == 0) out_h[c] = l1;
            break;
          }
          continue;
        }
        if ((l1 + p1) - (l0 + p0) > luacc) {
          GST_COUNT(18)
#pragma unroll
          for (int j = 0; j < PX; ++j) xv[j] = qv[j];
          l0 = l1;
          p0 = p1;
          Lvalid = true;
        } else {
          Lvalid = false;
        }
      }
      if (pass == 1 || eval_only || !redraw || fb || (st.debug & DEBUG_EXACT_BDRAW)) break;
      fshift = floor_shift(f_apr, lane, md.ntm, md.ntm_pad, md.ntm_pad + md.nf + (GEN ? md.nec : 0));
      if (__builtin_expect(fshift == 0.0, 1)) break;
      status |= STATUS_FLOOR;
      ++nfloor;
      Lvalid = false;
      }
      fshift = 0.0;
    }
    if (eval_only) return;
    GST_STAMP(3)

    bool drew = false;
    if (redraw && role == owner) {
      if (fb) {
        status |= 2;
      } else {
        drew = true;
        GST_SUB_BEGIN
#pragma unroll
        for (int s = 0; s < K0; ++s)
#pragma unroll
          for (int r = s; r < MT; ++r) L[SL(r, s)] = lr_load(tmf, 512 * tm_slot(MT, r, s));
        // y_k = 1/sqrt(a_kk); z = L^-1 d has z_k = zraw_k * y_k; L_ik = a_ik * y_k
#pragma unroll
        for (int sl = 0; sl < 2; ++sl) {
          const int j = 64 * sl + lane;
          if (j < MP) {
            apiv[j] = f_apr[sl];
            zraw[j] = f_zr[sl];
          }
        }
        lds_order();
        for (int j = lane; j < raug; j += 64) yinv[j] = rsqrt_nr(apiv[j]);
        lds_order();
        // rhs w = z + eta
        if (TAPE) {
          // eta = L^T Delta, so that L^-T eta equals the reference's U S^-1/2 xi
          for (int j = lane; j < MP; j += 64) xbuf[j] = 0.0;
          lds_order();
          for (int j = lane; j < m; j += 64) xbuf[md.ref2int[j]] = tp[TP_DELTA + j];
          lds_order();
#pragma unroll
          for (int s = 0; s < MT; ++s) {
            double part = 0.0;
            const int j = 8 * s + q;
#pragma unroll
            for (int r = s; r < MT; ++r) {
              const int i = 8 * r + p;
              part += (i >= j && i < raug) ? L[SL(r, s)] * xbuf[i] : 0.0;
            }
            part += __shfl_xor(part, 8, 64);
            part += __shfl_xor(part, 16, 64);
            part += __shfl_xor(part, 32, 64);
            if (p == 0 && j < raug) wvec[j] = (zraw[j] + part) * yinv[j];
          }
        } else {
          // normals 2l and 2l + 1 of the b-draw stream from lane l's one Philox draw
          if (2 * lane < raug) {
            double n0, n1;
            normal_pair(rng, (uint32_t)lane, TAG_BDRAW, n0, n1);
            const int j0 = 2 * lane, j1 = 2 * lane + 1;
            wvec[j0] = zraw[j0] * yinv[j0] + n0;
            if (j1 < raug) wvec[j1] = zraw[j1] * yinv[j1] + n1;
          }
        }
        lds_order();
        GST_SUB_END(12)
        // back substitution L^T v = w, descending columns:
        // v_k = (w_k - y_k * sum_{i>k} a_ik v_i) * y_k
        double vr[MT];
#pragma unroll
        for (int r = 0; r < MT; ++r) vr[r] = 0.0;
#pragma unroll
        for (int K = MT - 1; K >= 0; --K) {
          // rows of the slots below K are solved: their part of every column 8K+q is one
          // per-lane sum, reduced over p once per slot column (every lane (p, q) gets the
          // sum of column 8K+q); the 8 in-slot columns are then solved with uniform values
          double pe = 0.0, po2 = 0.0;
#pragma unroll
          for (int r = K + 1; r < MT; r += 2) {
            pe = fma(L[SL(r, K)], vr[r], pe);
            if (r + 1 < MT) po2 = fma(L[SL(r + 1, K)], vr[r + 1], po2);
          }
          double acc = pe + po2;
          acc += dpp<DPP_ROR8>(acc);  // (l + 8) mod 16 == l ^ 8: p and p ^ 1
          acc += __shfl_xor(acc, 16, 64);
          acc += __shfl_xor(acc, 32, 64);
          // diagonal block, transposed through LDS: dcol[i] = a_{8K+i, 8K+q}
          tdg[8 * q + p] = L[SL(K, K)];
          lds_order();
          double dcol[8];
#pragma unroll
          for (int i = 0; i < 8; ++i) dcol[i] = tdg[8 * q + i];
          const int kq = 8 * K + q;
          const double wq = wvec[kq], yq = yinv[kq];
          lds_order();
          double vmine = 0.0;
#pragma unroll
          for (int kk = 7; kk >= 0; --kk) {
            if (8 * K + kk >= raug) continue;
            // lanes q == kk now hold sum_{i>k} a_ik v_i of column k = 8K + kk
            const double vq = (wq - yq * acc) * yq;
            const double vk = rdlane(vq, kk);
            vmine = (q == kk) ? vk : vmine;
            acc = fma(dcol[kk], vk, acc);  // row k's term of the columns q < kk
          }
          xbuf[kq] = vmine;  // zero for the pad columns k >= raug
          lds_order();
          vr[K] = xbuf[8 * K + p];
        }
        lds_order();
        GST_SUB_END(13)
        for (int j = lane; j < m; j += 64) {
          const double bj = xbuf[md.ref2int[j]];
          bsc[j] = bj;
          brow[j] = bj;                   // the state array is the chain's b
        }
        lds_order();
        compute_Tb();
        GST_SUB_END(14)
      }
    }
    if constexpr (PAIR) {
      // hand the new b to the other wave: its copy of bsc, then its own y = r - T b
      if (mask & 6u) {
        if (drew) {
          double* pb = smem[role ^ 1] + (bsc - smem[role]);
          for (int j = lane; j < m; j += 64) pb[j] = bsc[j];
          // and its y = r - T b (compute_Tb's values: the partner copies them instead of
          // repeating the T b product)
          if (owner >= 0) {
#pragma unroll
            for (int s = 0; s < NS; ++s) xyv[s][lane] = yv[s];
          }
        }
        if (role == (owner >= 0 ? owner : 0) && lane == 0) xdrew[0] = drew ? 1 : 0;
        __syncthreads();
        const bool got = xdrew[0] != 0;
        if (got && role != owner) {
          if (owner >= 0) {
#pragma unroll
            for (int s = 0; s < NS; ++s) yv[s] = xyv[s][lane];
          } else {
            compute_Tb();
          }
        }
        __syncthreads();   // xdrew and xyv are rewritten next sweep
      }
    }

    GST_STAMP(4)
    fair_prio<OCC>(fair);
    GST_SUB_BEGIN
    // ---- outlier block: theta (gibbs.py:185-198)
    const double ef2 = efac2_of(xv);
    const double Q = exp(2.0 * pget(xv, md.idx_equad) * 2.302585092994045684);
    const bool mix = (md.model == 2) || (md.model == 3);
    if ((mask & 8u) && mix) {
      int zs = 0;
#pragma unroll
      for (int s = 0; s < NS; ++s) zs += __popcll(__ballot(((zb & vmask) >> s) & 1u));
      const double a = (double)zs + md.mk;
      const double b = ((double)n - (double)zs) + md.k1mm;
      if (TAPE) {
        theta = tp[TP_DELTA + m];
      } else {
        // Gamma(a) on lane 0, Gamma(b) on lane 1 (and its copies), side by side
        const double g = gamma_mt(lane == 0 ? a : b, rng, lane == 0 ? 0u : 1u, TAG_THETA);
        const double ga = rdlane(g, 0), gb = rdlane(g, 1);
        theta = ga / (ga + gb);
      }
    }
    fair_prio<OCC>(fair);
    GST_SUB_END(23)
    // ---- z (gibbs.py:201-226)
    // pair mode: each wave draws z and alpha for its half of the TOA slots (Philox is keyed
    // by TOA, so every draw is the one the single-wave kernel makes) and takes the other
    // half from its partner through LDS
    const unsigned mine = PAIR ? (vmask & (role ? 0xAAAAAAAAu : 0x55555555u)) : vmask;
    if ((mask & 16u) && mix) {
      const double SQ2PI = 2.5066282746310002;  // np.sqrt(2*np.pi)
#pragma unroll
      for (int s = 0; s < NS; ++s) {
        if (mine & (1u << s)) {
          const int t = 64 * s + lane;
          double N0;
          if constexpr (GEN)
            N0 = gen_n0(xv, S2(s), gef[s], geq[s]);
          else
            N0 = ef2 * S2(s) + Q;
          const double Nv = al[s] * N0;
          const double y = yv[s];
          const double sd1 = sqrt(Nv);
          const double x1 = y / sd1;
          double top = theta * (exp(-(x1 * x1) / 2.0) / SQ2PI / sd1);
          if (md.model == 3) top = theta / md.pspin;
          const double sd0 = sqrt(N0);
          const double x0 = y / sd0;
          const double bot = top + (1.0 - theta) * (exp(-(x0 * x0) / 2.0) / SQ2PI / sd0);
          double qz = top / bot;
          if (isnan(qz)) qz = 1.0;
          po[s] = qz;
          const double pz = qz < 1.0 ? qz : 1.0;
          double u;
          if (TAPE) {
            u = tp[TP_DELTA + m + 1 + t];
          } else {
            double unused;
            rng.uniform2((uint32_t)t, TAG_Z, u, unused);
          }
          const int zz = bern_legacy(pz, u);
          zb = (zb & ~(1u << s)) | ((unsigned)zz << s);
        }
      }
      if constexpr (PAIR) {
#pragma unroll
        for (int s = 0; s < NS; ++s) {
          const unsigned long long bm = __ballot((zb >> s) & 1u);
          if ((s & 1) == role) {
            xpo[s][lane] = po[s];
            if (lane == 0) xzm[s] = bm;
          }
        }
        __syncthreads();
#pragma unroll
        for (int s = 0; s < NS; ++s) {
          if ((s & 1) != role) {
            po[s] = xpo[s][lane];
            zb = (zb & ~(1u << s)) | ((unsigned)((xzm[s] >> lane) & 1ull) << s);
          }
        }
        // the partner's reads complete before either wave can overwrite its slots again
        // (a later sweep's z stage; a launch's stage mask need not hold a barrier between)
        __syncthreads();
      }
    }
    fair_prio<OCC>(fair);
    GST_SUB_END(24)
    // ---- alpha (gibbs.py:229-242)
    if ((mask & 32u) && md.vary_alpha) {
      int zs = 0;
#pragma unroll
      for (int s = 0; s < NS; ++s) zs += __popcll(__ballot(((zb & vmask) >> s) & 1u));
      if (zs >= 1) {
        double G[NS];
        if (TAPE) {
#pragma unroll
          for (int s = 0; s < NS; ++s) G[s] = tp[TP_DELTA + m + 1 + nst + 64 * s + lane];
        } else {
          // all of the lane's TOAs in one rejection loop (independent draws, so their
          // Philox / log / sqrt chains interleave); each TOA's variates and acceptance
          // sequence are exactly gamma_mt's (the large path draws them that way)
          double sh[NS];
#pragma unroll
          for (int s = 0; s < NS; ++s) sh[s] = ((double)((zb >> s) & 1u) + nu) / 2.0;
          gamma_mt_slots<NS>(sh, mine, rng, (uint32_t)lane, TAG_ALPHA, G);
        }
#pragma unroll
        for (int s = 0; s < NS; ++s) {
          if (mine & (1u << s)) {
            const double zf = (double)((zb >> s) & 1u);
            double N0;
            if constexpr (GEN)
              N0 = gen_n0(xv, S2(s), gef[s], geq[s]);
            else
              N0 = ef2 * S2(s) + Q;
            const double top = ((yv[s] * yv[s]) * zf / N0 + nu) / 2.0;
            al[s] = top / G[s];
          }
        }
        if constexpr (PAIR) {
#pragma unroll
          for (int s = 0; s < NS; ++s)
            if ((s & 1) == role) xal[s][lane] = al[s];
          __syncthreads();
#pragma unroll
          for (int s = 0; s < NS; ++s)
            if ((s & 1) != role) al[s] = xal[s][lane];
          __syncthreads();   // as for z: reads done before the next write of these slots
        }
      }
    }
    GST_SUB_END(25)
    GST_STAMP(5)
    // ---- nu (gibbs.py:244-259, 331-335)
    if ((mask & 64u) && md.vary_df) {
      double sa = 0.0;
#pragma unroll
      for (int s = 0; s < NS; ++s)
        if (vmask & (1u << s)) sa += log(al[s]) + 1.0 / al[s];
      const double S = wave_sum(sa);
      double ll = -INFINITY;
      if (lane < 30) {
        const double h = (double)(lane + 1) / 2.0;
        ll = -h * S + md.dfA[lane] - md.dfB[lane];
      }
      const double mx = wave_max(ll);
      if (lane < 30) dfbuf[lane] = exp(ll - mx);
      lds_order();
      double u;
      if (TAPE) {
        u = tp[TP_DELTA + m + 1 + 2 * nst];
      } else {
        double unused;
        rng.uniform2(0u, TAG_DF, u, unused);
      }
      // numpy pairwise sum of 30 (8 accumulators), normalise, sequential cumsum, choice
      double acc8[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) acc8[j] = dfbuf[j];
#pragma unroll
      for (int i = 8; i < 24; i += 8)
#pragma unroll
        for (int j = 0; j < 8; ++j) acc8[j] += dfbuf[i + j];
      double tot = ((acc8[0] + acc8[1]) + (acc8[2] + acc8[3])) +
                   ((acc8[4] + acc8[5]) + (acc8[6] + acc8[7]));
#pragma unroll
      for (int i = 24; i < 30; ++i) tot += dfbuf[i];
      // p_i = e_i / tot on lane i (one division per lane, not 30 per lane), the cumsum in
      // numpy's sequential order over the published p's (each lane keeps its own prefix),
      // then lane i tests cdf_i / cdf_29 <= u and the ballot counts (searchsorted 'right')
      const double pl = lane < 30 ? dfbuf[lane] / tot : 0.0;
      if (lane < 30) dfbuf[32 + lane] = pl;
      lds_order();
      double cs = 0.0, mine = 0.0;
#pragma unroll
      for (int i = 0; i < 30; ++i) {
        cs += dfbuf[32 + i];
        mine = (i == lane) ? cs : mine;
      }
      int cnt = __popcll(__ballot(lane < 30 && mine / cs <= u));
      cnt = cnt < 29 ? cnt : 29;
      nu = (double)(cnt + 1);
      lds_order();
    }
  }

  GST_STAMP(6)
  if (role != 0) return;   // pair mode: wave 0 writes the chain's state
  GST_STAMP_FLUSH
  // ---------------- write back ----------------
  if (lane < P) xrow[lane] = pget(xv, lane);
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    const int t = 64 * s + lane;
    if (vmask & (1u << s)) {
      zrow[t] = (double)((zb >> s) & 1u);
      arow[t] = al[s];
      prow[t] = po[s];
    }
  }
  lds_order();   // the Gram counters' LDS adds precede their read
  if (lane == 0) {
    st.theta[c] = theta;
    st.nu[c] = nu;
    if (st.status) st.status[c] = (st.status[c] | status) + nfloor * STATUS_FLOOR_COUNT;
    if (st.gram_cnt) {
      __hip_atomic_fetch_add(st.gram_cnt, (unsigned long long)gcnt[wv][0], __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_fetch_add(st.gram_cnt + 1, (unsigned long long)gcnt[wv][1],
                             __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

}  // namespace gst
