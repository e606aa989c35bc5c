/*
 * gst.h -- C ABI of the MI355X-native batched Gibbs sampler (libgst.so).
 *
 * Drop-in boundary for the reference's Python sampler `Gibbs` (/root/reference/gibbs.py).
 * The reference has no FFI: its "interface" is the Python class.  These entry points are
 * what a ctypes (or cgo/JNI) binding of that class binds; INTEGRATION.md shows the
 * ctypes stub.  Each entry point names the reference code it replaces.
 *
 * Conventions
 *  - every function returns int: 0 = ok, < 0 = error; gst_last_error() gives the message
 *    (thread-local).  No C++ exception crosses the ABI.
 *  - all chain buffers are DEVICE pointers owned by the caller (PyTorch-ROCm tensors'
 *    data_ptr()), fp64, laid out chain-major (struct-of-arrays); the library owns only the
 *    model constants it uploads in gst_model_set and its own scratch.
 *  - `stream` is a hipStream_t (may be NULL = default stream).  No host synchronisation
 *    happens inside gst_sweep; gst_sync() waits for the stream.
 *  - one ctx per device; not re-entrant across threads, and used from one stream at a
 *    time: its scratch (the persistent path's parked timing-model factors and sweep
 *    counter, the large path's per-chain buffers) is shared by all of its launches and
 *    indexed by launch-local chain, so two concurrent gst_sweep calls on different streams
 *    would race on it.  Scratch grows with stream-ordered allocation (hipMallocAsync /
 *    hipFreeAsync on the launch's stream), never with a device-synchronising hipFree.
 */
#ifndef GST_H_
#define GST_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GST_ABI_VERSION 6

/* Outlier model kind: Gibbs(model=...) (gibbs.py:9,32,187-226). */
enum gst_outlier_model {
  GST_MODEL_GAUSSIAN = 0,
  GST_MODEL_T = 1,
  GST_MODEL_MIXTURE = 2,
  GST_MODEL_VVH17 = 3
};

/* Stage mask for gst_sweep (the per-sweep stage order of gibbs.py:363-380). */
enum gst_stage {
  GST_STAGE_WHITE = 1u << 0, /* update_white_params  gibbs.py:114-143 */
  GST_STAGE_HYPER = 1u << 1, /* update_hyper_params  gibbs.py:80-111 */
  GST_STAGE_B = 1u << 2,     /* update_b             gibbs.py:145-182 (+ quirk :373) */
  GST_STAGE_THETA = 1u << 3, /* update_theta         gibbs.py:185-198 */
  GST_STAGE_Z = 1u << 4,     /* update_z             gibbs.py:201-226 */
  GST_STAGE_ALPHA = 1u << 5, /* update_alpha         gibbs.py:229-242 */
  GST_STAGE_DF = 1u << 6,    /* update_df            gibbs.py:244-259 */
  GST_STAGE_ALL = 0x7fu,
  GST_STAGE_B_FORCE = 1u << 7, /* draw b regardless of the gibbs.py:373 test (direct call) */
  /* Timing diagnostic, not a reference stage: compute the Gram T^T N^-1 [T|r] and eliminate
   * the timing-model columns (the first half of update_hyper_params' first likelihood,
   * gibbs.py:302-304,321) and nothing else of the red-noise block; the chain state is not
   * changed by it.  bench.py times it to report the Gram stage's fp64 utilisation.  Always
   * runs one wave per chain. */
  GST_STAGE_GRAM = 1u << 8
};

/* Model + sampler configuration.  Host pointers; copied by gst_model_set.
 * Replaces: the pta protocol calls (gibbs.py:29,35,154-158,209-210,268-269,297-301,339)
 * and the Gibbs constructor options (gibbs.py:9-51). */
typedef struct gst_model_desc {
  int n;           /* TOAs */
  int m;           /* basis columns = nfourier + ntm (reference order [Fourier | TM]) */
  int nfourier;    /* 2 * components */
  int ntm;         /* timing-model columns */
  int nparams;     /* P <= 4, sorted by name as enterprise does */
  const double* T;         /* n x m, row-major, reference column order */
  const double* residuals; /* n, seconds */
  const double* toaerrs;   /* n, seconds */
  const double* ffreqs;    /* nfourier (= repeat(f, 2)) */
  double tm_weight;        /* timing-model prior variance (1e40, run_sims.py:27-29) */
  /* parameter roles: index into the P-vector or -1 */
  int idx_efac, idx_equad, idx_log10_A, idx_gamma;
  double efac_const;       /* used when idx_efac < 0 */
  const double* pmin;      /* P uniform prior bounds */
  const double* pmax;
  const int* hyper_idx;    /* hyper parameter indices (gibbs.py:64-69) */
  int n_hyper;
  const int* white_idx;    /* white parameter indices (gibbs.py:72-77) */
  int n_white;
  /* outlier model (Gibbs kwargs) */
  int model;               /* enum gst_outlier_model */
  int vary_df;
  int vary_alpha;
  int theta_prior_beta;    /* theta_prior == 'beta' */
  double mprior;           /* m (a-priori outlier probability) */
  double pspin;            /* vvh17 only */
  const double* df_A;      /* 30: n*(nu/2)*log(nu/2) for nu=1..30 (gibbs.py:333-334) */
  const double* df_B;      /* 30: n*gammaln(nu/2) */
  /* General white noise (ABI 3; all zero / NULL = the classic single-backend model above).
   * The reference treats any efac / equad parameter as white and any ecorr parameter as
   * hyper (gibbs.py:64-77), e.g. the notebook's J1643-1224 model (efac, equad and an ECORR
   * basis, gibbs_likelihood.ipynb cell 2) or per-backend selections.  Such models run on
   * the large path (GST_PATH_LARGE; AUTO picks it); nparams may then be up to 16. */
  int nbackend;            /* backends with their own parameters, 1..8 (0 = 1) */
  const int* backend;      /* n: backend of each TOA (NULL: all 0) */
  const int* efac_idx;     /* nbackend: parameter index of each backend's efac, -1 =
                              efac_const (NULL: idx_efac for every backend) */
  const int* equad_idx;    /* nbackend: each backend's log10_equad (NULL: idx_equad) */
  const int* ecorr_idx;    /* nbackend: each backend's log10_ecorr, -1 = none (NULL: none) */
  int n_ecorr;             /* ECORR basis columns: the LAST n_ecorr columns of T, prior
                              variance 10^(2 log10_ecorr) of their backend; m = nfourier +
                              ntm + n_ecorr.  Epochs are normally disjoint (each TOA in at
                              most one ECORR column, enterprise's quantised basis); the large
                              path then eliminates them first, and only then:
                              gst_model_set checks the basis, and a batch with any TOA in two
                              ECORR columns takes the general elimination (ABI 6) */
  const int* ecorr_backend;/* n_ecorr: backend of each ECORR column */
} gst_model_desc;

/* Per-chain state, device pointers, chain-major.  x[C*P], b[C*m], z/alpha/pout[C*nmax]
 * (nmax = largest n of the model's datasets; TOAs t >= n of a chain's dataset are never
 * touched), theta/nu[C]; status[C] may be NULL, else flags are OR-ed into it:
 *   status & 1 (bit 0)  a Cholesky failure was seen in the hyper block (lnL = -inf);
 *   status & 2 (bit 1)  the b-draw factorisation failed and b was kept;
 *   status & 4 (bit 2)  dataset index out of range: the persistent path does not run the
 *                       chain, the large path runs it on dataset 0;
 *   status & 8 (bit 3)  large path: the chain's aligned 16-chain group mixes datasets;
 *   status & 16 (bit 4) informational: a b draw ran at the SVD noise floor (Sigma beyond
 *                       fp64 resolution, e.g. vvh17's all-outlier start; see gst_sweep);
 *   status >> 8 (ABI 5) the number of b draws made at the SVD noise floor (each adds 256), so
 *                       that a caller who zeroes status can count them over any window.
 * dataset[C] gives each chain's dataset index into the batch passed to
 * gst_model_set_batch; it may be NULL when there is one dataset. */
typedef struct gst_state {
  double* x;
  double* b;
  double* z;
  double* alpha;
  double* pout;
  double* theta;
  double* nu;
  int* status;
  const int* dataset;
} gst_state;

/* Chain records (Gibbs.sample's chain/bchain/zchain/... arrays, gibbs.py:344-361):
 * device pointers shaped [C][nrec][...] (per-TOA arrays [C][nrec][nmax]); any pointer may
 * be NULL to skip that array.
 * Sweep i of a launch is stored at record (i / record_every) when i % record_every == 0,
 * holding the state at the START of the sweep, as the reference does (gibbs.py:355-361). */
typedef struct gst_records {
  double* x;
  double* b;
  double* z;
  double* alpha;
  double* pout;
  double* theta;
  double* nu;
  int nrec;
} gst_records;

/* Injected-variate tape (parity mode), device pointer [C][nsweeps][stride] fp64 with
 * stride = gst_tape_stride(nmax, m) (n = nmax below).  Per chain-sweep layout:
 *   [0,80)   white MH step s: u_scale, param index, jump normal, accept uniform
 *   [80,120) hyper MH step s: same
 *   [120,120+m)  b draw term Delta = U S^-1/2 xi in reference order
 *   then: beta value; n binomial uniforms; n gamma values; dof-choice uniform. */
typedef struct gst_tape {
  const double* data;
  int stride;
} gst_tape;

int gst_version(void);
int gst_tape_stride(int n, int m);
int gst_last_error(char* buf, size_t len);

int gst_ctx_create(int device, void** ctx);
int gst_ctx_destroy(void* ctx);

/* Upload model constants (replaces the pta object, gibbs.py:29-35). */
int gst_model_set(void* ctx, const gst_model_desc* desc);

/* Upload a batch of `ndatasets` models at once (one Gibbs object per dataset x outlier
 * model in run_sims.py:80-113, e.g. the outlier / no_outlier pair of simulate_data.py at
 * several thetas, each under the five outlier models).  The descriptors must agree in
 * m, nfourier, ntm, nparams, parameter roles and hyper/white index sets; n, the data,
 * priors and the outlier-model options may differ.  Chains pick their dataset through
 * gst_state.dataset.  On the large path every aligned group of 16 chains must share one
 * dataset (its Gram and T b kernels stage one dataset's T per group); a chain whose group
 * mixes datasets is flagged with status & 8 (bit 3). */
int gst_model_set_batch(void* ctx, const gst_model_desc* descs, int ndatasets);

/* Number of datasets, largest n (row stride of per-TOA state/records) and tape stride. */
int gst_model_info(void* ctx, int* ndatasets, int* nmax, int* tape_stride);

/* Run `nsweeps` Gibbs sweeps for chains [0, nchains) (Gibbs.sample's loop body,
 * gibbs.py:354-380).  `tape` NULL or tape->data NULL -> on-device Philox4x32-10 variates
 * keyed by (seed, chain0 + c), counters by (sweep0 + i, stage, index): results do not
 * depend on how chains are sharded over launches or GPUs.
 * b draw (gibbs.py:145-182): exact Cholesky draw b = Sigma^-1 d + L^-T eta, except where
 * Sigma is beyond fp64 resolution -- its smallest LDL^T pivot (timing-model-first order, real
 * columns) below 2^-52 of its largest, p_max.  There the reference's sl.svd returns the small
 * eigenvalues at LAPACK's rounding floor (~0.3-2 x 2^-52 x s_max) and its draw is in effect
 * that of Sigma + f I; this path draws from Sigma + f I with f = 0.75 x 2^-52 p_max (flags
 * status & 16 and counts the draw in status >> 8), which reproduces the reference's escape
 * from vvh17's all-outlier start.  ABI 4 gated at 1e-14.
 * GST_DEBUG_EXACT_BDRAW turns the floor off. */
int gst_sweep(void* ctx, const gst_state* state, const gst_records* rec,
              const gst_tape* tape, int nchains, int nsweeps, long long sweep0,
              int record_every, unsigned stage_mask, unsigned long long seed,
              long long chain0, void* stream);

/* Evaluate the two likelihoods for K (state, x) pairs without sampling:
 *   out_white[k] = get_lnlikelihood_white(x_k)  (gibbs.py:262-284)
 *   out_hyper[k] = get_lnlikelihood(x_k)        (gibbs.py:288-329)
 * using chain k's b, z, alpha from `state` (x from state->x). */
int gst_eval_lnlike(void* ctx, const gst_state* state, int nchains, double* out_white,
                    double* out_hyper, void* stream);

int gst_sync(void* ctx, void* stream);

/* Execution path.  The persistent path keeps a whole chain in one wavefront for all of a
 * launch's sweeps (n <= 512 and up to 30 red-noise components with <= 16 timing-model
 * columns, 26 with <= 24, n <= 1024 for the 30-component / 16-column shape; smaller models
 * run padded with unit-prior dummy columns; the general white-noise model -- per-backend
 * efac / equad, ECORR columns, up to 8 parameters -- with <= 16 timing-model columns, up to
 * 60 Fourier + ECORR columns and n <= 512); the
 * large path runs
 * each sweep as a pipeline of kernels (fp64-MFMA Gram shared by all chains, blocked
 * timing-model elimination, LDS-resident red-noise MH, MFMA T b, per-TOA passes) for
 * large n and m (BASELINE config 5).  AUTO (default) picks persistent when it fits.
 * gst_set_path must precede gst_model_set. */
enum gst_path { GST_PATH_AUTO = 0, GST_PATH_PERSISTENT = 1, GST_PATH_LARGE = 2 };
int gst_set_path(void* ctx, int path);
int gst_get_path(void* ctx, int* path);

/* Waves per chain on the persistent path.  A sampling launch with at most one chain per two
 * SIMDs (C <= 2 x CUs, e.g. BASELINE config 3's 512 chains) runs each chain on two waves
 * that split the red-noise MH block's likelihood evaluations (AUTO, the default); the
 * chain's draws are bitwise those of the one-wave kernel.  GST_WAVES_ONE / GST_WAVES_TWO
 * force either kernel for every sampling launch (tape-mode and gst_eval_lnlike launches
 * always run one wave per chain).  Since round 6 the general white-noise model (per-backend
 * white noise, ECORR columns) has the two-wave kernel too. */
enum gst_waves { GST_WAVES_AUTO = 0, GST_WAVES_ONE = 1, GST_WAVES_TWO = 2 };
int gst_set_waves(void* ctx, int waves);

/* Diagnostics of the persistent path.  GST_DEBUG_POISON: at the start of every sweep each
 * chain overwrites all of its LDS and its parked timing-model factor scratch with a NaN
 * pattern; since a chain carries no state between sweeps beyond its state arrays, a launch
 * with this flag must give bitwise the same chains as one without (a read of any stale word
 * would surface as NaN / different draws).  Costs time; never set in production. */
/* Large path: GST_DEBUG_LARGE_GRAM forces the 64x64 super-tile Gram (lg_gram) where the
 * one-wave-per-chain Gram (lg_gram_small) would run; the two give bitwise the same G.  It also
 * turns off the structured ECORR Gram (lg_gram_ec, round 6: disjoint ECORR epochs eliminated
 * first -- only G_xx, the epochs' diagonal and their couplings, by MFMA), whose G blocks agree
 * with the dense Gram's to rounding (summation order).
 * GST_DEBUG_LARGE_HYPER forces the LDS-resident hyper kernel (lg_hyper) where the register-
 * resident one (lg_hyper_reg) would run: same variates and decisions, likelihoods within
 * rounding; and the blocked global-memory elimination (lg_hyper<1>) where the ECORR-epochs-
 * first one (lg_hyper<2>) would run: likelihoods within rounding, b draws of the same law.
 * Test switches (the defaults are the faster kernels). */
/* GST_DEBUG_EXACT_BDRAW: every b draw is the exact draw from Sigma, also beyond fp64
 * resolution (no SVD noise floor, see gst_sweep). */
/* The floor gate's pivot order: the timing-model-first LDL^T (real columns) on the
 * persistent path and the large path's classes 0 / 1 and register kernels; the large path's
 * class 2 (ECORR epochs eliminated first, lg_hyper<2>) gates on the pivots of its own order
 * [ECORR | TM | Fourier].  Pivot ratios depend on the order, so near the 2^-52 gate the two
 * orders can decide a draw differently (both draw exactly from Sigma or Sigma + f I). */
/* GST_DEBUG_MFMA_GRAM (ABI 5): the persistent kernel computes every Gram on the MFMA path,
 * never the low-rank one (datasets of <= 8 noise classes, at most 32 flagged TOAs: the
 * per-class Grams plus one rank-1 update per flagged TOA); the two agree
 * to rounding. */
/* GST_DEBUG_EPOCHS_LDS (ABI 6): large-path chains whose ECORR epochs are eliminated first run
 * the 256-thread LDS kernel lg_hyper<2> instead of the one-wave register kernel
 * lg_hyper_ecr (timing model <= 16 columns, Fourier block <= 46 columns); same elimination
 * order, likelihoods and b draws equal to rounding.  A/B and test switch. */
enum gst_debug {
  GST_DEBUG_POISON = 1,
  GST_DEBUG_LARGE_GRAM = 2,
  GST_DEBUG_LARGE_HYPER = 4,
  GST_DEBUG_EXACT_BDRAW = 8,
  GST_DEBUG_MFMA_GRAM = 16,
  GST_DEBUG_EPOCHS_LDS = 32
};
int gst_set_debug(void* ctx, int flags);

/* Per-kernel timing of the large path (HIP events around every launch of the next
 * gst_sweep / gst_eval_lnlike calls while enabled).  gst_kernel_times fills ms[k] (summed
 * milliseconds) and launches[k] for kernel kinds k < nkinds (enum gst_kernel_kind). */
enum gst_kernel_kind {
  GST_K_RECORD = 0, GST_K_WHITE = 1, GST_K_GRAM = 2, GST_K_TMELIM = 3,
  GST_K_HYPER = 4, GST_K_BTM = 5, GST_K_TB = 6, GST_K_TOA = 7, GST_K_COUNT = 8
};
int gst_set_timing(void* ctx, int on);
int gst_kernel_times(void* ctx, double* ms, int* launches, int nkinds);

/* Diagnostic builds (-DGST_STAMPS) only: per-chain per-stage s_memtime cycle sums (slots
 * 0-15 and 19-23) and event counts (16: red-noise likelihoods, 17: two-wave rounds, 18:
 * accepted red-noise proposals) are accumulated into dev_buf[C][24]; returns an error in
 * production builds. */
int gst_debug_stamps(void* ctx, unsigned long long* dev_buf);

/* Kernel-level timing of the last gst_sweep on its stream (hipEvents), milliseconds. */
int gst_last_sweep_ms(void* ctx, double* ms);

/* Grams T^T N^-1 [T|r] (gibbs.py:302-304) computed since the last reset, by path (ABI 6):
 *   counts[0]  persistent kernel, low-rank: the dataset's per-class Grams plus one rank-1
 *              update per flagged TOA, on the VALU (<= 8 noise classes, <= 32 flagged TOAs,
 *              every flagged alpha <= 2^20);
 *   counts[1]  persistent kernel, the n-TOA fp64 MFMA Gram;
 *   counts[2]  large path, fp64 MFMA Gram (lg_gram / lg_gram_small), chains x launches.
 * One count per chain per Gram (the floor pass recomputes it: counted again).  Synchronises
 * the device.  reset != 0 zeroes the counters after reading them. */
int gst_gram_counts(void* ctx, long long* counts, int reset);

/* Test hook (ABI 6): n draws of the kernel's own samplers into the DEVICE array out, Philox
 * keyed by (seed, call), for distribution tests of the samplers themselves:
 *   kind 0  gamma_mt(a): Marsaglia-Tsang Gamma(a, 1), a < 1 by the a + 1 boost (the theta
 *           stage's Gammas);
 *   kind 1  Beta(a, b) = Ga / (Ga + Gb) from two gamma_mt draws (update_theta, gibbs.py:196);
 *   kind 2  gamma_mt_slots<4>, the alpha stage's interleaved Gamma(a) draws (gibbs.py:239);
 *           n a multiple of 256.
 * n <= 2^31.  Needs no context; runs on the current device. */
int gst_debug_variates(int kind, double a, double b, long long n, unsigned long long seed,
                       unsigned call, double* out, void* stream);

/* Batched synthetic pulsars on the current device: the simulate_data.py:10-39 recipe for
 * `ndatasets` datasets in one launch (one workgroup per dataset), Philox variates keyed by
 * (seed, dataset0 + d).  Replaces simulate_data() + the par/tim round trip through
 * libstempo (simulate_data.py:12-37, run_sims.py:41-51).  All pointers are DEVICE pointers;
 * per-dataset outputs are [ndatasets][n].
 *   error bars   toaerrs[n] if given, else 10^(-7 + 0.2 N(0,1)) s         (:15)
 *   red noise    red[n] if given (e.g. red.txt), else F (sqrt(phi) N(0,1)) with the power
 *                law phi_k = A^2/(12 pi^2) fyr^(gamma-3) f_k^-gamma df_k        (:21)
 *   outliers     z_t ~ Bernoulli(theta)                                   (:24)
 *   residuals    red + ((1 - z) err + z sigma_out) xi, xi ~ N(0,1) or Student-t(dof) for
 *                dof > 0, then the timing model refit out: r - U (U^T r)  (:26)
 *   clean twin   (residuals_clean may be NULL) the no_outlier dataset (:35-37): outlier
 *                TOAs deleted (their entries set to 0) and the timing model refit on the
 *                kept TOAs (needs ntm <= 64).
 * Limits: nfourier <= 512, ntm <= 512. */
typedef struct gst_sim_desc {
  int n, nfourier, ntm, ndatasets;
  const double* F;        /* [n][nfourier] Fourier basis (may be NULL when red is given) */
  const double* log_f;    /* [nfourier] log f_k (Hz) */
  const double* log_df;   /* [nfourier] log df_k */
  double log_fyr;         /* log(1 / yr in Hz) */
  const double* U;        /* [n][ntm] orthonormal timing-model basis (SVD of M) */
  const double* red;      /* [n] fixed red-noise realisation (s) or NULL */
  const double* toaerrs;  /* [n] fixed error bars (s) or NULL */
  const double* theta;    /* [ndatasets] outlier fraction */
  const double* sigma_out;/* [ndatasets] outlier scatter (s) */
  const double* log10_A;  /* [ndatasets] red-noise amplitude (power-law draw) */
  const double* gamma;    /* [ndatasets] red-noise spectral index */
  const double* dof;      /* [ndatasets] Student-t dof of the white noise, <= 0: Gaussian */
  unsigned long long seed;
  long long dataset0;     /* global index of dataset 0 (shards give the same datasets) */
  double* residuals;      /* out [ndatasets][n] */
  double* toaerrs_out;    /* out [ndatasets][n] */
  double* z;              /* out [ndatasets][n] injected outlier flags (0 / 1) */
  double* residuals_clean;/* out [ndatasets][n] or NULL */
} gst_sim_desc;
int gst_simulate(const gst_sim_desc* desc, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* GST_H_ */
