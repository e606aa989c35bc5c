// C ABI of libgst.so (declared in include/gst.h): context, model upload, sweep launch.
//
// The host side only packs model constants into the layouts the kernel wants and picks
// the template instance (matrix slots MT, TOA slots NS, timing-model panels K0, tape or
// Philox variates).  All chain state lives in caller-owned device buffers.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <algorithm>
#include <cstring>
#include <string>
#include <vector>

#include "gst.h"
#include "gst_kernel.hpp"
#include "gst_shapes.h"
#include "gst_large.hpp"
#include "gst_sim.hpp"

namespace {

thread_local std::string g_err;

int fail(const std::string& msg) {
  g_err = msg;
  return -1;
}

#define HIP_OK(expr)                                                              \
  do {                                                                            \
    hipError_t e_ = (expr);                                                       \
    if (e_ != hipSuccess)                                                         \
      return fail(std::string(#expr) + ": " + hipGetErrorString(e_));             \
  } while (0)

struct Ctx {
  int device = 0;
  bool has_model = false;
  std::vector<gst::DevModel> hmd;  // host copies, one per dataset
  gst::DevModel* dmd = nullptr;    // device array [nd] (in allocs)
  int nd = 0, nmax = 0, m = 0, raug = 0;
  int MT = 0, NS = 0, K0 = 0, WPB = 4;
  bool gen = false;                // persistent path: the general white-noise instances
  int ncu = 256;                   // compute units of the device (workgroup sizing)
  double* tmfac = nullptr;         // persistent path: timing-model factor scratch
  unsigned long long* prog = nullptr;  // persistent path: launch-wide sweep counter (fair_prio)
  size_t tmfac_bytes = 0;
  int path_req = GST_PATH_AUTO;    // gst_set_path
  int path = GST_PATH_PERSISTENT;  // chosen by gst_model_set
  int waves = GST_WAVES_AUTO;      // gst_set_waves
  int debug = 0;                   // gst_set_debug
  unsigned long long* gram_cnt = nullptr;  // persistent path: [2] Grams by path (gst_gram_counts)
  unsigned long long gram_large = 0;       // large path: chain Grams launched (lg_gram*)
  std::vector<void*> allocs;
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  bool timed = false;
  // large path: scratch sized for scratch_C chains, per-kernel timing events
  gst::LScratch ls{};
  int scratch_C = 0;
  size_t lds_tm = 0, lds_hyper = 0, lds_btm = 0, lds_hyper_big = 0, lds_hyper_ec = 0;
  bool hyper_big = false;          // large path: a hyper block past HYPER_LDS_MAX (G3 scratch)
  bool hyper_ec = false;           // ... of ECORR epochs, eliminated first (lg_hyper<2>, no G3)
  bool timing = false;
  std::vector<hipEvent_t> evpool;
  std::vector<int> evkind;  // kind of event pair i (events 2i, 2i+1)
  size_t evused = 0;
};

// Scratch that grows inside a launch call is allocated and freed stream-ordered
// (hipMallocAsync / hipFreeAsync on the launch's stream): no device synchronisation inside
// gst_sweep, and a buffer is released only after the work queued before it on that stream.
void free_scratch(Ctx* cx, hipStream_t st) {
  for (double* p : {cx->ls.G, cx->ls.G2, cx->ls.y, cx->ls.w, cx->ls.sc, cx->ls.v, cx->ls.G3})
    if (p) (void)hipFreeAsync(p, st);
  cx->ls = gst::LScratch{};
  cx->scratch_C = 0;
}

int upload(Ctx* cx, const void* host, size_t bytes, void** dev) {
  void* p = nullptr;
  HIP_OK(hipMalloc(&p, bytes > 0 ? bytes : 16));
  if (bytes) HIP_OK(hipMemcpy(p, host, bytes, hipMemcpyHostToDevice));
  cx->allocs.push_back(p);
  *dev = p;
  return 0;
}

void free_tmfac(Ctx* cx, hipStream_t st) {
  if (cx->tmfac) (void)hipFreeAsync(cx->tmfac, st);
  cx->tmfac = nullptr;
  cx->tmfac_bytes = 0;
}

// Model replacement / context teardown (outside any launch): wait for the device, then
// release everything.
void free_model(Ctx* cx) {
  (void)hipDeviceSynchronize();
  for (void* p : cx->allocs) (void)hipFree(p);
  cx->allocs.clear();
  cx->hmd.clear();
  cx->dmd = nullptr;
  cx->nd = 0;
  cx->has_model = false;
  free_scratch(cx, nullptr);
  free_tmfac(cx, nullptr);
  (void)hipDeviceSynchronize();
}

using gst::kfn_t;

// The instance for a shape (gst_shapes.h; each shape's instances live in their own
// translation unit, gst_inst.hip).  wpb: chains per workgroup (4, or 2 / 1 for sampling
// launches with fewer chains than fill every SIMD; tape-mode parity launches always use 4).
// occ2: the two-chains-per-SIMD build (256 registers per lane), picked when the launch has
// more chains than SIMDs; with at most one chain per SIMD the uncapped build keeps more of
// each chain in registers.  pair: two waves per chain (gst_set_waves).
// gen: the general white-noise model's instances (GEN shapes).
kfn_t pick(int MT, int NS, int K0, int RA, bool gen, bool tape, int wpb, bool occ2,
           bool pair = false) {
#define GST_CASE(mt, ns, k0, ra, g)                                              \
  if (MT == mt && NS == ns && K0 == k0 && RA == ra && (gen ? 1 : 0) == g)        \
    return gst::GST_PICK_NAME(mt, ns, k0, ra, g)(tape, wpb, occ2, pair);
  GST_SHAPES(GST_CASE)
#undef GST_CASE
  return nullptr;
}

// Register-resident shapes (MT, K0, RA), smallest first: a model with nf Fourier and ntm
// timing-model columns runs in the first with 8 K0 >= ntm and RA - 8 K0 >= nf, padded.
// General white-noise models (GEN) have their own shapes; nf counts the Fourier and the ECORR
// columns there (both sit in the hyper block).
struct Shape {
  int MT, K0, RA;
};
const Shape kShapes[] = {{8, 2, 56}, {10, 2, 76}, {10, 3, 76}};
const Shape kShapesGen[] = {{8, 2, 62}, {10, 2, 76}};

const Shape* shape_for(int nf, int ntm, bool gen = false) {
  const Shape* tab = gen ? kShapesGen : kShapes;
  const int nt = gen ? (int)(sizeof kShapesGen / sizeof(Shape)) : (int)(sizeof kShapes / sizeof(Shape));
  for (int i = 0; i < nt; ++i)
    if (8 * tab[i].K0 >= (ntm > 0 ? ntm : 1) && tab[i].RA - 8 * tab[i].K0 >= nf) return &tab[i];
  return nullptr;
}

int round_up(int a, int b) { return (a + b - 1) / b * b; }

// gst_debug_variates: the kernel's own samplers, one draw (kind 0, 1) or four (kind 2) per
// thread, Philox keyed by (seed, chain 0xFFFFFFF0, sweep = call, index, TAG_DEBUG).
constexpr uint32_t TAG_DEBUG = 14u << 24;
__global__ void __launch_bounds__(256) debug_variates_kernel(int kind, double a, double b,
                                                             long long n, unsigned long long seed,
                                                             unsigned call, double* out) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  gst::Rng rng;
  rng.k0 = (uint32_t)(seed & 0xffffffffull);
  rng.k1 = (uint32_t)(seed >> 32);
  rng.chain = 0xFFFFFFF0u;
  rng.sweep = call;
  if (kind == 0) {              // gamma_mt(a): the theta stage's Gamma
    if (i < n) out[i] = gst::gamma_mt(a, rng, (uint32_t)i, TAG_DEBUG);
  } else if (kind == 1) {       // the theta stage's Beta(a, b) = Ga / (Ga + Gb)
    if (i < n) {
      const double ga = gst::gamma_mt(a, rng, (uint32_t)(2 * i), TAG_DEBUG);
      const double gb = gst::gamma_mt(b, rng, (uint32_t)(2 * i + 1), TAG_DEBUG);
      out[i] = ga / (ga + gb);
    }
  } else {                      // gamma_mt_slots<4>: the alpha stage's interleaved Gammas
    const long long w = i >> 6, l = i & 63;
    if (256 * w < n) {
      const double sh[4] = {a, a, a, a};
      double g[4];
      gst::gamma_mt_slots<4>(sh, 0xFu, rng, (uint32_t)(256 * w + l), TAG_DEBUG, g);
#pragma unroll
      for (int s = 0; s < 4; ++s) out[256 * w + 64 * s + l] = g[s];
    }
  }
}

}  // namespace

extern "C" {

int gst_version(void) { return GST_ABI_VERSION; }

int gst_tape_stride(int n, int m) { return gst::TP_DELTA + m + 2 + 2 * n; }

int gst_last_error(char* buf, size_t len) {
  if (!buf || !len) return -1;
  std::snprintf(buf, len, "%s", g_err.c_str());
  return 0;
}

int gst_ctx_create(int device, void** ctx) {
  if (!ctx) return fail("gst_ctx_create: null ctx");
  int ndev = 0;
  HIP_OK(hipGetDeviceCount(&ndev));
  if (device < 0 || device >= ndev) return fail("gst_ctx_create: bad device index");
  HIP_OK(hipSetDevice(device));
  Ctx* cx = new Ctx();
  cx->device = device;
  hipDeviceProp_t prop;
  HIP_OK(hipGetDeviceProperties(&prop, device));
  cx->ncu = prop.multiProcessorCount > 0 ? prop.multiProcessorCount : 256;
  HIP_OK(hipEventCreate(&cx->ev0));
  HIP_OK(hipEventCreate(&cx->ev1));
  HIP_OK(hipMalloc(&cx->prog, 256));   // fair_prio's launch-wide sweep counter
  HIP_OK(hipMalloc(&cx->gram_cnt, 2 * sizeof(unsigned long long)));
  HIP_OK(hipMemset(cx->gram_cnt, 0, 2 * sizeof(unsigned long long)));
  *ctx = cx;
  return 0;
}

int gst_ctx_destroy(void* ctx) {
  Ctx* cx = static_cast<Ctx*>(ctx);
  if (!cx) return 0;
  (void)hipSetDevice(cx->device);
  free_model(cx);
  if (cx->prog) (void)hipFree(cx->prog);
  if (cx->gram_cnt) (void)hipFree(cx->gram_cnt);
  for (hipEvent_t e : cx->evpool) (void)hipEventDestroy(e);
  if (cx->ev0) (void)hipEventDestroy(cx->ev0);
  if (cx->ev1) (void)hipEventDestroy(cx->ev1);
  delete cx;
  return 0;
}

// Pack one dataset's constants (shapes already validated) into device buffers owned by cx.
// ntm_pad / raug: the internal positions of the first Fourier column and of the residual
// row; a persistent-kernel instance larger than the model leaves unit-prior dummy columns
// between the Fourier block and the residual row.
static int pack_dataset(Ctx* cx, const gst_model_desc* d, gst::DevModel& md, int ntm_pad,
                        int raug, int MT) {
  const int n = d->n, m = d->m, nf = d->nfourier, ntm = d->ntm, P = d->nparams;
  const int nec = d->n_ecorr;
  const int mpad = round_up(raug + 1, 16);
  const int npad = 64 * ((n + 63) / 64);

  // internal column order: [TM | pad | Fourier | ECORR | r | pad]; reference order
  // [Fourier | TM | ECORR]
  std::vector<int> ref2int(m), int2ref(mpad, -1);
  for (int j = 0; j < nf; ++j) ref2int[j] = ntm_pad + j;
  for (int j = 0; j < ntm; ++j) ref2int[nf + j] = j;
  for (int j = 0; j < nec; ++j) ref2int[nf + ntm + j] = ntm_pad + nf + j;
  for (int j = 0; j < m; ++j) int2ref[ref2int[j]] = j;
  const int NT = mpad / 16;
  const int nks = round_up(n, 4) / 4;
  // k-steps padded with zeros to whole 64-TOA chunks (the large path's Gram stages 16)
  std::vector<double> Tmf((size_t)(npad / 4) * NT * 64, 0.0);
  for (int ks = 0; ks < nks; ++ks)
    for (int X = 0; X < NT; ++X)
      for (int l = 0; l < 64; ++l) {
        const int t = 4 * ks + (l >> 4);
        const int i = 16 * X + (l & 15);
        double v = 0.0;
        if (t < n) {
          if (i == raug)
            v = d->residuals[t];
          else if (i < mpad && int2ref[i] >= 0)
            v = d->T[(size_t)t * m + int2ref[i]];
        }
        Tmf[((size_t)ks * NT + X) * 64 + l] = v;
      }
  std::vector<double> Tcol((size_t)m * npad, 0.0), resid(npad, 0.0), sig2(npad, 0.0);
  for (int t = 0; t < n; ++t) {
    for (int j = 0; j < m; ++j) Tcol[(size_t)j * npad + t] = d->T[(size_t)t * m + j];
    resid[t] = d->residuals[t];
    sig2[t] = d->toaerrs[t] * d->toaerrs[t];
  }
  // red-noise spectrum pieces: log f_k and log df_k (df from f[::2], enterprise powerlaw)
  std::vector<double> lf(nf), ldf(nf);
  for (int k = 0; k < nf; ++k) {
    lf[k] = std::log(d->ffreqs[k]);
    const int pair = k / 2;
    const double prev = pair == 0 ? 0.0 : d->ffreqs[2 * (pair - 1)];
    ldf[k] = std::log(d->ffreqs[2 * pair] - prev);
  }
  // noise classes: TOAs with bit-identical sigma share N0 in the white likelihood
  // (and equal backend: N0 = efac_b^2 sigma^2 + 10^(2 equad_b) depends on both)
  std::vector<double> csig2;
  std::vector<double> ccount;
  std::vector<int> cback;
  std::vector<int> cidx(npad, -1);
  for (int t = 0; t < n; ++t) {
    const double v = d->toaerrs[t] * d->toaerrs[t];
    const int bt = (d->nbackend > 1 && d->backend) ? d->backend[t] : 0;
    int u = 0;
    while (u < (int)csig2.size() && (csig2[u] != v || cback[u] != bt)) ++u;
    if (u == (int)csig2.size()) {
      if (csig2.size() >= 8) break;
      csig2.push_back(v);
      ccount.push_back(0.0);
      cback.push_back(bt);
    }
    cidx[t] = u;
    ccount[u] += 1.0;
  }
  int ncls = (int)csig2.size();
  for (int t = 0; t < n; ++t)
    if (cidx[t] < 0) ncls = 0;  // more than 8 distinct sigmas: per-TOA path
  double slf = 0.0, sldf = 0.0;
  for (int k = 0; k < nf; ++k) {
    slf += lf[k];
    sldf += ldf[k];
  }
  std::vector<double> dfA(32, 0.0), dfB(32, 0.0);
  for (int k = 0; k < 30; ++k) {
    dfA[k] = d->df_A[k];
    dfB[k] = d->df_B[k];
  }

  md = gst::DevModel{};
  void* ptr;
  if (upload(cx, Tmf.data(), Tmf.size() * 8, &ptr)) return -1;
  md.Tmf = (const double*)ptr;
  if (upload(cx, Tcol.data(), Tcol.size() * 8, &ptr)) return -1;
  md.Tcol = (const double*)ptr;
  if (upload(cx, resid.data(), resid.size() * 8, &ptr)) return -1;
  md.resid = (const double*)ptr;
  if (upload(cx, sig2.data(), sig2.size() * 8, &ptr)) return -1;
  md.sig2 = (const double*)ptr;
  if (upload(cx, lf.data(), lf.size() * 8, &ptr)) return -1;
  md.lfreq = (const double*)ptr;
  if (upload(cx, ldf.data(), ldf.size() * 8, &ptr)) return -1;
  md.ldf = (const double*)ptr;
  if (upload(cx, dfA.data(), dfA.size() * 8, &ptr)) return -1;
  md.dfA = (const double*)ptr;
  if (upload(cx, dfB.data(), dfB.size() * 8, &ptr)) return -1;
  md.dfB = (const double*)ptr;
  if (upload(cx, ref2int.data(), ref2int.size() * sizeof(int), &ptr)) return -1;
  md.ref2int = (const int*)ptr;
  md.ncls = ncls;
  for (int u = 0; u < 8; ++u) md.cls_b[u] = u < ncls ? cback[u] : 0;
  if (ncls > 0) {
    if (upload(cx, cidx.data(), cidx.size() * sizeof(int), &ptr)) return -1;
    md.cidx = (const int*)ptr;
    if (upload(cx, csig2.data(), csig2.size() * 8, &ptr)) return -1;
    md.csig2 = (const double*)ptr;
    if (upload(cx, ccount.data(), ccount.size() * 8, &ptr)) return -1;
    md.ccount = (const double*)ptr;
  }
  md.sum_lfreq = slf;
  md.sum_ldf = sldf;
  // Persistent kernel, <= 8 noise classes: the Gram of the augmented basis per
  // class, G_k = sum_{t in class k} [T|r]_t [T|r]_t^T (long double, rounded once), in the
  // kernel's 8x8-cyclic register layout [k][slot][lane], and the augmented rows
  // [T|r]_t in internal order, stored [t][i % 8][i / 8] (a lane's row entries 8 r + p,
  // r = 0 .. MT-1, are contiguous: 128-bit loads).  With them a sweep's Gram T^T N^-1 [T|r] is
  //   sum_k c_k G_k + sum_{t: z_t = 1} c_k(t) (1 / alpha_t - 1) [T|r]_t [T|r]_t^T,
  // c_k = 1 / (efac_b^2 sigma_k^2 + 10^(2 equad_b)): N_t = alpha_t^z_t N0_k(t) (gibbs.py:154,
  // 297-304), a rank-(outlier count) update instead of the n-TOA MFMA Gram (gst_kernel.hpp
  // gram_and_tm; the kernel takes it while at most LR_MAX TOAs are flagged).
  md.Gcls = nullptr;
  md.Trow = nullptr;
  if (MT > 0 && ncls > 0) {
    const int W = 8 * MT, NSL = MT * (MT + 1) / 2;
    std::vector<double> trow((size_t)npad * W, 0.0);
    for (int t = 0; t < n; ++t)
      for (int i = 0; i < W; ++i) {
        double v = 0.0;
        if (i == raug)
          v = d->residuals[t];
        else if (i < mpad && int2ref[i] >= 0)
          v = d->T[(size_t)t * m + int2ref[i]];
        trow[(size_t)t * W + (i & 7) * MT + (i >> 3)] = v;   // [t][i % 8][i / 8]
      }
    std::vector<long double> acc((size_t)ncls * W * W, 0.0L);
    for (int t = 0; t < n; ++t) {
      long double* a = acc.data() + (size_t)cidx[t] * W * W;
      const double* row = trow.data() + (size_t)t * W;
      auto at = [&](int i) { return row[(i & 7) * MT + (i >> 3)]; };
      for (int i = 0; i < W; ++i) {
        const double ri = at(i);
        if (ri == 0.0) continue;
        for (int j = 0; j <= i; ++j) a[(size_t)i * W + j] += (long double)ri * at(j);
      }
    }
    std::vector<double> gcls((size_t)ncls * NSL * 64, 0.0);
    for (int k = 0; k < ncls; ++k)
      for (int r = 0; r < MT; ++r)
        for (int sl = 0; sl <= r; ++sl)
          for (int l = 0; l < 64; ++l) {
            const int i = 8 * r + (l >> 3), j = 8 * sl + (l & 7);
            const long double v = i >= j ? acc[((size_t)k * W + i) * W + j]
                                         : acc[((size_t)k * W + j) * W + i];
            gcls[((size_t)k * NSL + gst::SL(r, sl)) * 64 + l] = (double)v;
          }
    if (upload(cx, trow.data(), trow.size() * 8, &ptr)) return -1;
    md.Trow = (const double*)ptr;
    if (upload(cx, gcls.data(), gcls.size() * 8, &ptr)) return -1;
    md.Gcls = (const double*)ptr;
  }

  md.n = n;
  md.m = m;
  md.mp = mpad;
  md.nf = nf;
  md.ntm = ntm;
  md.ntm_pad = ntm_pad;
  md.raug = raug;
  md.nks = nks;
  md.npad = npad;
  md.nslot_toa = npad / 64;
  md.P = P;
  md.idx_efac = d->idx_efac;
  md.idx_equad = d->idx_equad;
  md.idx_logA = d->idx_log10_A;
  md.idx_gamma = d->idx_gamma;
  md.efac_const = d->efac_const;
  for (int j = 0; j < gst::PMAX; ++j) {
    md.pmin[j] = j < P ? d->pmin[j] : 0.0;
    md.pmax[j] = j < P ? d->pmax[j] : 0.0;
    md.lp_in[j] = j < P ? -std::log(d->pmax[j] - d->pmin[j]) : 0.0;
    md.hind[j] = j < d->n_hyper ? d->hyper_idx[j] : d->hyper_idx[0];
    md.wind[j] = j < d->n_white ? d->white_idx[j] : d->white_idx[0];
  }
  // general white noise: per-backend parameter indices, per-TOA backend, ECORR columns
  const int nb = d->nbackend > 0 ? d->nbackend : 1;
  md.nb = nb;
  for (int b = 0; b < gst::NBMAX; ++b) {
    md.efac_b[b] = b < nb ? (d->efac_idx ? d->efac_idx[b] : d->idx_efac) : -1;
    md.equad_b[b] = b < nb ? (d->equad_idx ? d->equad_idx[b] : d->idx_equad) : d->idx_equad;
    md.ecorr_b[b] = b < nb && d->ecorr_idx ? d->ecorr_idx[b] : -1;
    md.ec_count[b] = 0.0;
  }
  md.nec = nec;
  md.bk = nullptr;
  md.ecb = nullptr;
  if (nb > 1) {
    std::vector<int> bk(npad, 0);
    for (int t = 0; t < n; ++t) bk[t] = d->backend ? d->backend[t] : 0;
    if (upload(cx, bk.data(), bk.size() * sizeof(int), &ptr)) return -1;
    md.bk = (const int*)ptr;
  }
  if (nec > 0) {
    std::vector<int> eb(nec);
    for (int e = 0; e < nec; ++e) {
      eb[e] = d->ecorr_backend ? d->ecorr_backend[e] : 0;
      md.ec_count[eb[e]] += 1.0;
    }
    if (upload(cx, eb.data(), eb.size() * sizeof(int), &ptr)) return -1;
    md.ecb = (const int*)ptr;
  }
  // large path, disjoint ECORR epochs: the structured Gram's operands (gst_large.hpp
  // lg_gram_ec), when [timing model | Fourier | r | 1] fits four 16-column tiles
  md.Tx = md.Xe = nullptr;
  md.ekl = md.eblk = nullptr;
  md.gx_nt = md.nkse = md.neblk = 0;
  const int Q = ntm_pad + nf;
  bool ec_disj = MT == 0 && nec > 0;
  for (int t = 0; ec_disj && t < n; ++t) {
    int nz = 0;
    for (int e = 0; e < nec; ++e) nz += d->T[(size_t)t * m + nf + ntm + e] != 0.0;
    ec_disj = nz <= 1;
  }
  if (ec_disj && Q + 2 <= 64) {
    const int NX = (Q + 2 + 15) / 16;
    // compact [X | r | 1] row q of TOA t (the ones column stays zero here: lg_gram_ec's G_xx
    // does not use it)
    auto xval = [&](int t, int q) -> double {
      if (q < Q) return int2ref[q] >= 0 ? d->T[(size_t)t * m + int2ref[q]] : 0.0;
      return q == Q ? d->residuals[t] : 0.0;
    };
    std::vector<double> tx((size_t)(npad / 4) * NX * 64, 0.0);
    for (int ks = 0; ks < nks; ++ks)
      for (int X = 0; X < NX; ++X)
        for (int l = 0; l < 64; ++l) {
          const int t = 4 * ks + (l >> 4);
          if (t < n) tx[((size_t)ks * NX + X) * 64 + l] = xval(t, 16 * X + (l & 15));
        }
    // the epochs' TOAs (ascending), 16 epochs per block, each block padded to whole k-steps
    std::vector<std::vector<int>> etoa(nec);
    for (int t = 0; t < n; ++t)
      for (int e = 0; e < nec; ++e)
        if (d->T[(size_t)t * m + nf + ntm + e] != 0.0) etoa[e].push_back(t);
    const int neblk = (nec + 15) / 16;
    std::vector<int> eblk(neblk + 1, 0), ent_t, ent_e;
    for (int b = 0; b < neblk; ++b) {
      eblk[b] = (int)ent_t.size() / 4;
      for (int e = 16 * b; e < std::min(nec, 16 * b + 16); ++e)
        for (int t : etoa[e]) {
          ent_t.push_back(t);
          ent_e.push_back(e - 16 * b);
        }
      while (ent_t.size() % 4) {
        ent_t.push_back(-1);
        ent_e.push_back(-1);
      }
    }
    eblk[neblk] = (int)ent_t.size() / 4;
    const int nkse = std::max(16, round_up(eblk[neblk], 16));
    ent_t.resize((size_t)nkse * 4, -1);
    ent_e.resize((size_t)nkse * 4, -1);
    std::vector<double> xe((size_t)nkse * NX * 64, 0.0);
    std::vector<int> ekl((size_t)nkse * 8, -1);
    for (int p = 0; p < 4 * nkse; ++p) {
      ekl[2 * p] = ent_t[p];
      ekl[2 * p + 1] = ent_e[p];
    }
    for (int b = 0; b < neblk; ++b)
      for (int p = 4 * eblk[b]; p < 4 * eblk[b + 1]; ++p) {
        const int t = ent_t[p];
        if (t < 0) continue;
        const int e = 16 * b + ent_e[p];
        const double u = d->T[(size_t)t * m + nf + ntm + e];
        const int ks = p / 4, k = p % 4;
        for (int X = 0; X < NX; ++X)
          for (int j = 0; j < 16; ++j) {
            const int q = 16 * X + j;
            const double v = q == Q + 1 ? u * u : u * xval(t, q);
            xe[((size_t)ks * NX + X) * 64 + 16 * k + j] = v;
          }
      }
    if (upload(cx, tx.data(), tx.size() * 8, &ptr)) return -1;
    md.Tx = (const double*)ptr;
    if (upload(cx, xe.data(), xe.size() * 8, &ptr)) return -1;
    md.Xe = (const double*)ptr;
    if (upload(cx, ekl.data(), ekl.size() * sizeof(int), &ptr)) return -1;
    md.ekl = (const int*)ptr;
    if (upload(cx, eblk.data(), eblk.size() * sizeof(int), &ptr)) return -1;
    md.eblk = (const int*)ptr;
    md.gx_nt = NX;
    md.nkse = nkse;
    md.neblk = neblk;
  }
  md.lp_sum = 0.0;  // Python sum() order (gibbs.py:339)
  for (int j = 0; j < P; ++j) md.lp_sum += md.lp_in[j];
  md.nh = d->n_hyper;
  md.nw = d->n_white;
  md.sig_h = 0.05 * d->n_hyper;
  md.sig_w = 0.05 * d->n_white;
  const double probs[5] = {0.1, 0.15, 0.5, 0.15, 0.1};
  const double sizes[5] = {0.1, 0.5, 1.0, 3.0, 10.0};
  double cs = 0.0, cdf[5];
  for (int i = 0; i < 5; ++i) {
    cs += probs[i];
    cdf[i] = cs;
  }
  for (int i = 0; i < 5; ++i) {
    md.mh_cdf[i] = cdf[i] / cdf[4];
    md.mh_size[i] = sizes[i];
  }
  md.model = d->model;
  md.vary_df = d->vary_df;
  md.vary_alpha = d->vary_alpha;
  if (d->theta_prior_beta) {
    md.mk = n * d->mprior;
    md.k1mm = n * (1.0 - d->mprior);
  } else {
    md.mk = 1.0;
    md.k1mm = 1.0;
  }
  md.pspin = d->pspin;
  md.tm_phiinv = 1.0 / d->tm_weight;
  md.logdet_phi_tm = ntm * std::log(d->tm_weight);
  md.log_fyr = std::log(1.0 / (365.25 * 86400.0));
  md.log_12pi2 = std::log(12.0) + 2.0 * std::log(M_PI);
  return 0;
}

// ECORR epochs are disjoint when no TOA has a nonzero entry in two of the last n_ecorr
// columns of T (lg_hyper<2>'s elimination takes the ECORR block of T^T N^-1 T as diagonal)
static bool ecorr_disjoint(const gst_model_desc* d) {
  const int m = d->m, nec = d->n_ecorr;
  for (int t = 0; t < d->n; ++t) {
    int nz = 0;
    for (int j = m - nec; j < m; ++j) nz += d->T[(size_t)t * m + j] != 0.0;
    if (nz > 1) return false;
  }
  return true;
}

static int check_desc(const gst_model_desc* d) {
  const int n = d->n, m = d->m, nf = d->nfourier, ntm = d->ntm, P = d->nparams;
  const int nec = d->n_ecorr, nb = d->nbackend > 0 ? d->nbackend : 1;
  if (n <= 0 || nec < 0 || m != nf + ntm + nec || nf <= 0 || ntm < 0)
    return fail("gst_model_set: bad sizes");
  if (P < 1 || P > gst::PMAX) return fail("gst_model_set: nparams must be 1..16");
  if (nb > gst::NBMAX) return fail("gst_model_set: at most 8 backends");
  if (d->idx_equad < 0 || d->idx_log10_A < 0 || d->idx_gamma < 0)
    return fail("gst_model_set: equad, log10_A and gamma parameters are required");
  if (d->n_hyper < 1 || d->n_hyper > P || d->n_white < 1 || d->n_white > P)
    return fail("gst_model_set: bad hyper/white index sets");
  if (!d->T || !d->residuals || !d->toaerrs || !d->ffreqs || !d->pmin || !d->pmax ||
      !d->hyper_idx || !d->white_idx || !d->df_A || !d->df_B)
    return fail("gst_model_set: null array in model descriptor");
  if ((nb > 1 && !d->backend) || (nec > 0 && (!d->ecorr_backend || !d->ecorr_idx)))
    return fail("gst_model_set: backend / ECORR arrays missing");
  for (int t = 0; nb > 1 && t < n; ++t)
    if (d->backend[t] < 0 || d->backend[t] >= nb) return fail("gst_model_set: bad backend index");
  for (int b = 0; b < nb; ++b) {
    const int ef = d->efac_idx ? d->efac_idx[b] : d->idx_efac;
    const int eq = d->equad_idx ? d->equad_idx[b] : d->idx_equad;
    const int ec = d->ecorr_idx ? d->ecorr_idx[b] : -1;
    if (ef >= P || eq < 0 || eq >= P || ec >= P) return fail("gst_model_set: bad parameter index");
  }
  for (int e = 0; e < nec; ++e) {
    const int b = d->ecorr_backend[e];
    if (b < 0 || b >= nb || d->ecorr_idx[b] < 0)
      return fail("gst_model_set: ECORR column without an ecorr parameter");
  }
  return 0;
}

// The classic model of the register-resident kernel: one backend, no ECORR, P <= 4.
static bool classic(const gst_model_desc* d) {
  return (d->nbackend <= 1) && d->n_ecorr == 0 && d->nparams <= 4 && d->n_hyper <= 4 &&
         d->n_white <= 4;
}
// The general white-noise model its GEN instances take: per-backend efac / equad (<= 8
// backends), ECORR epoch columns in the hyper block, up to 8 parameters.
static bool general_fits(const gst_model_desc* d) {
  return d->nparams <= 8 && d->n_hyper <= 8 && d->n_white <= 8 &&
         (d->nbackend > 0 ? d->nbackend : 1) <= gst::NBMAX;
}

// Datasets of one batch share the sampler structure: basis shape, parameter roles and the
// MH index sets.  n (ragged run_sims datasets), the data and the outlier model may differ.
static int same_structure(const gst_model_desc* a, const gst_model_desc* b) {
  if (a->m != b->m || a->nfourier != b->nfourier || a->ntm != b->ntm ||
      a->nparams != b->nparams || a->idx_efac != b->idx_efac || a->idx_equad != b->idx_equad ||
      a->idx_log10_A != b->idx_log10_A || a->idx_gamma != b->idx_gamma ||
      a->n_hyper != b->n_hyper || a->n_white != b->n_white || a->n_ecorr != b->n_ecorr ||
      (a->nbackend > 1 ? a->nbackend : 1) != (b->nbackend > 1 ? b->nbackend : 1))
    return 0;
  for (int j = 0; j < a->n_hyper; ++j)
    if (a->hyper_idx[j] != b->hyper_idx[j]) return 0;
  for (int j = 0; j < a->n_white; ++j)
    if (a->white_idx[j] != b->white_idx[j]) return 0;
  return 1;
}

int gst_model_set_batch(void* ctx, const gst_model_desc* descs, int nd) {
  Ctx* cx = static_cast<Ctx*>(ctx);
  if (!cx || !descs || nd <= 0) return fail("gst_model_set_batch: null argument");
  HIP_OK(hipSetDevice(cx->device));
  int nmax = 0;
  for (int i = 0; i < nd; ++i) {
    if (check_desc(&descs[i])) return -1;
    if (!same_structure(&descs[0], &descs[i]))
      return fail("gst_model_set_batch: datasets differ in basis shape, parameters or MH "
                  "index sets (dataset " + std::to_string(i) + ")");
    nmax = std::max(nmax, descs[i].n);
  }
  const gst_model_desc* d = &descs[0];
  const int nf = d->nfourier, ntm = d->ntm, m = d->m, nec = d->n_ecorr;
  bool disjoint = true;   // the batch's datasets all: one hyper class per batch structure
  for (int i = 0; i < nd && nec > 0; ++i) disjoint = disjoint && ecorr_disjoint(&descs[i]);
  const bool gen = !classic(d) && general_fits(d);
  const Shape* sh = shape_for(nf + (gen ? nec : 0), ntm, gen);
  const int MT = sh ? sh->MT : 0, K0 = sh ? sh->K0 : 0;
  const int raug = sh ? sh->RA : 0;
  const int nsl = (nmax + 63) / 64;
  // TOA slots of 64 held in registers: 2, 3, 4 (J1713-sized), 6, 8 (mid-size, n <= 512),
  // 12, 16 (wide mid-size, n <= 1024: the run_sims model's shape only; these keep one chain
  // per SIMD, their two-chains-per-SIMD builds would spill kilobytes per lane)
  // (the general white-noise model: 2, 3 (MT = 10 only), 4, 8); the smallest instantiated
  // slot count that holds n
  static const int kSlots[] = {2, 3, 4, 6, 8, 12, 16};
  int NS = 16;
  for (int ns : kSlots)
    if (ns >= nsl && sh && pick(MT, ns, K0, raug, gen, false, 4, false)) { NS = ns; break; }
  const bool fits = sh && (classic(d) || gen) && round_up(nmax, 4) <= 64 * NS &&
                    pick(MT, NS, K0, raug, gen, false, 4, false);
  int path = cx->path_req;
  if (path == GST_PATH_AUTO) path = fits ? GST_PATH_PERSISTENT : GST_PATH_LARGE;
  if (path == GST_PATH_PERSISTENT && !fits) {
    char b[220];
    std::snprintf(b, sizeof b,
                  "gst_model_set: no persistent-kernel instance for MT=%d NS=%d K0=%d RA=%d "
                  "GEN=%d (n=%d m=%d nfourier=%d ntm=%d n_ecorr=%d); use the large path", MT, NS,
                  K0, raug, gen ? 1 : 0, nmax, m, nf, ntm, nec);
    return fail(b);
  }
  if (path == GST_PATH_LARGE) {
    // hyper blocks past HYPER_LDS_MAX columns: ECORR epochs around a small timing-model +
    // Fourier block are eliminated first (lg_hyper<2>), other blocks are factored in global
    // memory (lg_hyper<1>), whose LDS holds a 16-column panel of all mp rows plus three vectors
    const int ms = nf + nec + 1, mpl = round_up(round_up(ntm > 0 ? ntm : 1, 16) + nf + nec + 1, 16);
    const int hc = gst::hyper_class(nf + nec, 0, nec, ntm + nf + 1, disjoint ? 1 : 0), qx = ntm + nf + 1;
    if (hc == 1 &&
        (size_t)(mpl * (gst::TM_PW + 1) + gst::TM_PW + nf + nec + 2 * ms) * 8 > 160 * 1024)
      return fail("gst_model_set: large path: basis too large for the LDS panel of the "
                  "red-noise / ECORR block elimination");
    // lg_hyper<2> (ECORR epochs eliminated first): its LDS vectors span the basis
    if (hc == 2 && (size_t)(2 * qx * (qx + 1) + nf + 2 * nec + 4 * mpl +
                            2 * gst::EC_ECH * (round_up(qx, 16) + 1)) * 8 > 160 * 1024)
      return fail("gst_model_set: large path: too many ECORR epochs for the LDS of their "
                  "elimination");
  }
  free_model(cx);
  // large path: timing-model block padded to whole 16-column MFMA tiles, no dummies
  const int ntm_pad = path == GST_PATH_LARGE ? round_up(ntm > 0 ? ntm : 1, 16) : 8 * K0;
  const int raug_pack = path == GST_PATH_LARGE ? ntm_pad + nf + nec : raug;
  std::vector<gst::DevModel> hmd(nd);
  for (int i = 0; i < nd; ++i) {
    if (pack_dataset(cx, &descs[i], hmd[i], ntm_pad, raug_pack,
                     path == GST_PATH_PERSISTENT ? MT : 0)) {
      free_model(cx);
      return -1;
    }
    hmd[i].ec_disjoint = disjoint ? 1 : 0;
  }
  void* ptr;
  if (upload(cx, hmd.data(), hmd.size() * sizeof(gst::DevModel), &ptr)) return -1;
  cx->dmd = (gst::DevModel*)ptr;
  cx->hmd = hmd;
  cx->nd = nd;
  cx->nmax = nmax;
  cx->MT = MT;
  cx->NS = NS;
  cx->K0 = K0;
  cx->raug = raug;
  cx->m = m;
  cx->WPB = 4;
  cx->gen = path == GST_PATH_PERSISTENT && gen;
  cx->path = path;
  cx->hyper_big = cx->hyper_ec = false;
  if (path == GST_PATH_LARGE) {
    const gst::DevModel& h = hmd[0];
    cx->raug = h.raug;
    cx->lds_tm = (size_t)h.mp * (gst::TM_PW + 1) * 8;
    const int ms = h.nf + h.nec + 1;
    const int hc = gst::hyper_class_of(h, 0);
    // lg_hyper<1> runs for class 1, and for class 2 under GST_DEBUG_LARGE_HYPER (its G3
    // scratch is then allocated at the first such launch)
    cx->hyper_big = gst::hyper_class_of(h, 1) == 1;
    cx->hyper_ec = hc == 2;
    const bool lds_fits = h.nf + h.nec <= gst::HYPER_LDS_MAX;   // lg_hyper<0> (also forced)
    cx->lds_hyper = lds_fits ? (size_t)(ms * (ms + 1) + h.nf + h.nec + 2 * ms) * 8 : 0;
    cx->lds_hyper_big = (size_t)(h.mp * (gst::TM_PW + 1) + gst::TM_PW + h.nf + h.nec + 2 * ms) * 8;
    // lg_hyper<2>: X and XB [qx][qx + 1], phi^-1 [nf + nec], four vectors of mp, a_e [nec],
    // two chunks of couplings [EC_ECH][qxp] and their 1 / a_e
    const int qx = h.ntm + h.nf + 1, qxp = round_up(qx, 16);
    cx->lds_hyper_ec = (size_t)(2 * qx * (qx + 1) + h.nf + h.nec + 4 * h.mp + h.nec +
                                2 * gst::EC_ECH * qxp + 2 * gst::EC_ECH) * 8;
    cx->lds_btm = (size_t)(3 * h.ntm_pad + h.raug) * 8;
    HIP_OK(hipFuncSetAttribute((const void*)gst::lg_gram,
                               hipFuncAttributeMaxDynamicSharedMemorySize, gst::GRAM_LDS * 8));
    HIP_OK(hipFuncSetAttribute((const void*)gst::lg_tmelim,
                               hipFuncAttributeMaxDynamicSharedMemorySize, (int)cx->lds_tm));
    if (cx->hyper_big && cx->lds_hyper_big <= 160 * 1024)
      HIP_OK(hipFuncSetAttribute((const void*)gst::lg_hyper<1>,
                                 hipFuncAttributeMaxDynamicSharedMemorySize,
                                 (int)cx->lds_hyper_big));
    if (hc == 2)
      HIP_OK(hipFuncSetAttribute((const void*)gst::lg_hyper<2>,
                                 hipFuncAttributeMaxDynamicSharedMemorySize,
                                 (int)cx->lds_hyper_ec));
    if (lds_fits)
      HIP_OK(hipFuncSetAttribute((const void*)gst::lg_hyper<0>,
                                 hipFuncAttributeMaxDynamicSharedMemorySize, (int)cx->lds_hyper));
    HIP_OK(hipFuncSetAttribute((const void*)gst::lg_btm,
                               hipFuncAttributeMaxDynamicSharedMemorySize, (int)cx->lds_btm));
  }
  cx->has_model = true;
  return 0;
}

int gst_model_set(void* ctx, const gst_model_desc* d) { return gst_model_set_batch(ctx, d, 1); }

int gst_model_info(void* ctx, int* ndatasets, int* nmax, int* tape_stride) {
  Ctx* cx = static_cast<Ctx*>(ctx);
  if (!cx || !cx->has_model) return fail("gst_model_info: no model set");
  if (ndatasets) *ndatasets = cx->nd;
  if (nmax) *nmax = cx->nmax;
  if (tape_stride) *tape_stride = gst_tape_stride(cx->nmax, cx->m);
  return 0;
}

// timing events (gst_set_timing): pair i brackets one launch of kernel kind evkind[i]
static int ev_mark(Ctx* cx, int kind, hipStream_t st, bool begin) {
  if (!cx->timing) return 0;
  if (begin) {
    if (2 * cx->evused + 2 > cx->evpool.size()) {
      hipEvent_t e0, e1;
      HIP_OK(hipEventCreate(&e0));
      HIP_OK(hipEventCreate(&e1));
      cx->evpool.push_back(e0);
      cx->evpool.push_back(e1);
      cx->evkind.push_back(0);
    }
    cx->evkind[cx->evused] = kind;
    HIP_OK(hipEventRecord(cx->evpool[2 * cx->evused], st));
  } else {
    HIP_OK(hipEventRecord(cx->evpool[2 * cx->evused + 1], st));
    ++cx->evused;
  }
  return 0;
}

#define LG_LAUNCH(kind, kern, grid, block, lds)                                  \
  do {                                                                           \
    if (ev_mark(cx, kind, st, true)) return -1;                                  \
    hipLaunchKernelGGL(kern, grid, block, lds, st, cx->dmd, a);                  \
    HIP_OK(hipGetLastError());                                                   \
    if (ev_mark(cx, kind, st, false)) return -1;                                 \
  } while (0)

// per-TOA scratch row stride of the large path: the batch's largest npad
static int large_ys(const Ctx* cx) {
  int ys = 0;
  for (const gst::DevModel& h : cx->hmd) ys = std::max(ys, h.npad);
  return ys;
}

static int ensure_scratch(Ctx* cx, int C, hipStream_t st) {
  // lg_hyper<1>'s G3: class-1 models, and class-2 ones under GST_DEBUG_LARGE_HYPER
  const bool need_g3 = cx->hyper_big && (!cx->hyper_ec || (cx->debug & GST_DEBUG_LARGE_HYPER));
  if (C <= cx->scratch_C && (!need_g3 || cx->ls.G3)) return 0;
  if (C <= cx->scratch_C) {
    const size_t mp = cx->hmd[0].mp;
    HIP_OK(hipMallocAsync((void**)&cx->ls.G3, (size_t)cx->scratch_C * mp * mp * 8, st));
    HIP_OK(hipMemsetAsync(cx->ls.G3, 0, (size_t)cx->scratch_C * mp * mp * 8, st));
    return 0;
  }
  free_scratch(cx, st);
  const gst::DevModel& h = cx->hmd[0];
  const size_t mp = h.mp, npad = large_ys(cx);
  HIP_OK(hipMallocAsync((void**)&cx->ls.G, (size_t)C * mp * mp * 8, st));
  HIP_OK(hipMallocAsync((void**)&cx->ls.G2, (size_t)C * mp * mp * 8, st));
  HIP_OK(hipMallocAsync((void**)&cx->ls.y, (size_t)C * npad * 8, st));
  HIP_OK(hipMallocAsync((void**)&cx->ls.w, (size_t)C * npad * 8, st));
  HIP_OK(hipMallocAsync((void**)&cx->ls.sc, (size_t)C * 16 * 8, st));
  HIP_OK(hipMallocAsync((void**)&cx->ls.v, (size_t)C * mp * 8, st));
  HIP_OK(hipMemsetAsync(cx->ls.G, 0, (size_t)C * mp * mp * 8, st));
  HIP_OK(hipMemsetAsync(cx->ls.G2, 0, (size_t)C * mp * mp * 8, st));
  HIP_OK(hipMemsetAsync(cx->ls.sc, 0, (size_t)C * 16 * 8, st));
  HIP_OK(hipMemsetAsync(cx->ls.v, 0, (size_t)C * mp * 8, st));
  if (need_g3) {   // lg_hyper<1>'s factor of the red-noise / ECORR block
    HIP_OK(hipMallocAsync((void**)&cx->ls.G3, (size_t)C * mp * mp * 8, st));
    HIP_OK(hipMemsetAsync(cx->ls.G3, 0, (size_t)C * mp * mp * 8, st));
  }
  cx->scratch_C = C;
  return 0;
}

// The red-noise MH block's launches: one per hyper kernel class present (gst_large.hpp
// hyper_class); a chain of another class returns at once.
static int launch_hyper(Ctx* cx, gst::LArgs& a, const bool (&hcls)[7], dim3 g8, dim3 b8,
                        dim3 g16, dim3 b16, dim3 g_chain, dim3 b_chain, hipStream_t st) {
  if (hcls[0]) {
    a.kclass = 8;
    LG_LAUNCH(GST_K_HYPER, gst::lg_hyper_reg<8>, g8, b8, 0);
  }
  if (hcls[1]) {
    a.kclass = 16;
    LG_LAUNCH(GST_K_HYPER, gst::lg_hyper_reg<16>, g16, b16, 0);
  }
  if (hcls[2]) {
    a.kclass = 0;
    LG_LAUNCH(GST_K_HYPER, gst::lg_hyper<0>, g_chain, b_chain, cx->lds_hyper);
  }
  if (hcls[3]) {
    // (a class-2 model forced here by GST_DEBUG_LARGE_HYPER may have a block whose panel
    // does not fit the LDS: refuse it rather than fail at launch)
    if (cx->lds_hyper_big > 160 * 1024)
      return fail("gst: GST_DEBUG_LARGE_HYPER: this model's red-noise / ECORR block is too "
                  "large for the blocked elimination's LDS panel (lg_hyper<1>)");
    a.kclass = 1;
    LG_LAUNCH(GST_K_HYPER, gst::lg_hyper<1>, g_chain, b_chain, cx->lds_hyper_big);
  }
  if (hcls[4]) {
    a.kclass = 2;
    LG_LAUNCH(GST_K_HYPER, gst::lg_hyper<2>, g_chain, b_chain, cx->lds_hyper_ec);
  }
  // class 2 on one wave per chain (lg_hyper_ecr<MT, RA>, gst_large.hpp ec_reg_mt)
  if (hcls[5]) {
    a.kclass = 2;
    const int w = gst::HE<6, 46>::WPB;
    const auto kern = &gst::lg_hyper_ecr<6, 46>;
    LG_LAUNCH(GST_K_HYPER, kern, dim3((a.C + w - 1) / w), dim3(64 * w), 0);
  }
  if (hcls[6]) {
    a.kclass = 2;
    const int w = gst::HE<8, 62>::WPB;
    const auto kern = &gst::lg_hyper_ecr<8, 62>;
    LG_LAUNCH(GST_K_HYPER, kern, dim3((a.C + w - 1) / w), dim3(64 * w), 0);
  }
  return 0;
}

// One sweep = record, white, gram, tmelim, hyper, btm, tb, toa launches (gst_large.hpp).
static int launch_large(Ctx* cx, const gst::DevState& ds, const gst::DevRec& dr,
                        const gst::DevTape& dt, int C, int nsweeps, long long sweep0,
                        int record_every, unsigned mask, unsigned long long seed,
                        long long chain0, int eval_only, double* ow, double* oh,
                        hipStream_t st) {
  if (ensure_scratch(cx, C, st)) return -1;
  const gst::DevModel& h = cx->hmd[0];
  const int ys = large_ys(cx);
  gst::LArgs a{ds, dr, dt, cx->ls, ys, C, nsweeps, 0, record_every, mask, seed, sweep0, chain0,
               eval_only, ow, oh};
  const int nsb = (h.mp / 16 + 3) / 4;
  const int npairs = nsb * (nsb + 1) / 2;
  // kernel classes present among the batch's datasets (gst_large.hpp white_class /
  // toa_class / hyper_class): one launch per class, each chain runs in its own dataset's
  // class, so its arithmetic never depends on the other datasets of the batch.  Hyper blocks
  // of up to HR_COLS (62) / HR_COLS_WIDE (126) columns: one wave per chain, register-resident
  // elimination (lg_hyper_reg<8> / <16>); larger ones: lg_hyper (LDS)
  const int hyper_lds = (cx->debug & GST_DEBUG_LARGE_HYPER) ? 1 : 0;
  bool wcls[3] = {false, false, false}, tcls[2] = {false, false};
  bool hcls[7] = {false, false, false, false, false, false, false};
  for (const gst::DevModel& hm : cx->hmd) {
    wcls[gst::white_class(hm.npad)] = true;
    tcls[gst::toa_class(hm.npad)] = true;
    const int hc = gst::hyper_class_of(hm, hyper_lds);
    const int emt = gst::ec_reg_mt_of(hm, hyper_lds, cx->debug);
    hcls[hc == 8 ? 0 : (hc == 16 ? 1 : (hc == 0 ? 2 : (hc == 1 ? 3 : (emt > 0 ? 4 + emt : 4))))] = true;
  }
  a.hyper_lds = hyper_lds;
  const dim3 g_hr8((C + gst::HR<8>::WPB - 1) / gst::HR<8>::WPB), b_hr8(64 * gst::HR<8>::WPB);
  const dim3 g_hr16((C + gst::HR<16>::WPB - 1) / gst::HR<16>::WPB), b_hr16(64 * gst::HR<16>::WPB);
  // Grams of at most GS_NTMAX 16-column tiles: one wave per chain (lg_gram_small<NT>)
  int gram_small = h.mp / 16;
  for (const gst::DevModel& hm : cx->hmd)
    if (hm.mp != h.mp) gram_small = 0;
  if (gram_small > gst::GS_NTMAX || (cx->debug & GST_DEBUG_LARGE_GRAM)) gram_small = 0;
  // datasets on the structured ECORR Gram (one tile count per batch: same structure)
  int gram_ec_nt = 0;
  bool gram_dense = false;
  // lg_tmelim and lg_btm return at once for class-2 chains (the epochs-first kernels factor the
  // timing model and draw all of b): a batch of class-2 datasets does not launch them
  bool tm_needed = false;
  for (const gst::DevModel& hm : cx->hmd) tm_needed = tm_needed || gst::hyper_class_of(hm, hyper_lds) != 2;
  for (const gst::DevModel& hm : cx->hmd) {
    if (gst::gram_ec_of(hm, hyper_lds, cx->debug))
      gram_ec_nt = hm.gx_nt;
    else
      gram_dense = true;
  }
  const dim3 g_gs((C + gst::GS_WPB - 1) / gst::GS_WPB), b_gs(64 * gst::GS_WPB);
  const dim3 g_gec((C + gst::GEC_CPB - 1) / gst::GEC_CPB);
  const dim3 g_chain(C), b_chain(gst::LBLK);
  const dim3 g_gram(npairs * ((C + gst::GRAM_WAVES - 1) / gst::GRAM_WAVES)), b_gram(64 * gst::GRAM_WAVES);
  const dim3 g_tb(ys / 64, (C + 64 * gst::TB_CG - 1) / (64 * gst::TB_CG));
  cx->evused = 0;
  HIP_OK(hipEventRecord(cx->ev0, st));
  LG_LAUNCH(GST_K_TB, gst::lg_tb, g_tb, b_chain, 0);   // y = r - T b for the current b
  const bool rec_on = record_every > 0 && !eval_only;
  const int nit = eval_only ? 1 : nsweeps;
  for (int it = 0; it < nit; ++it) {
    a.it = it;
    if (rec_on && it % record_every == 0) LG_LAUNCH(GST_K_RECORD, gst::lg_record, g_chain, b_chain, 0);
    if (wcls[0]) {
      a.kclass = 0;
      LG_LAUNCH(GST_K_WHITE, gst::lg_white<gst::TBLK_WAVE>, g_chain, dim3(gst::TBLK_WAVE), 0);
    }
    if (wcls[1]) {
      a.kclass = 1;
      LG_LAUNCH(GST_K_WHITE, gst::lg_white<gst::TBLK_SMALL>, g_chain, dim3(gst::TBLK_SMALL), 0);
    }
    if (wcls[2]) {
      a.kclass = 2;
      LG_LAUNCH(GST_K_WHITE, gst::lg_white<gst::TBLK>, g_chain, dim3(gst::TBLK), 0);
    }
    if ((mask & (6u | GST_STAGE_GRAM)) || eval_only) {
      if (ev_mark(cx, GST_K_GRAM, st, true)) return -1;
      // the structured Gram for the datasets it takes (gram_ec_of), the dense one for the
      // rest (each skips the other's chains)
      switch (gram_ec_nt) {
        case 1: hipLaunchKernelGGL(gst::lg_gram_ec<1>, g_gec, b_gs, 0, st, cx->dmd, a); break;
        case 2: hipLaunchKernelGGL(gst::lg_gram_ec<2>, g_gec, b_gs, 0, st, cx->dmd, a); break;
        case 3: hipLaunchKernelGGL(gst::lg_gram_ec<3>, g_gec, b_gs, 0, st, cx->dmd, a); break;
        case 4: hipLaunchKernelGGL(gst::lg_gram_ec<4>, g_gec, b_gs, 0, st, cx->dmd, a); break;
        default: break;
      }
      if (gram_dense) switch (gram_small) {
        case 1: hipLaunchKernelGGL(gst::lg_gram_small<1>, g_gs, b_gs, 0, st, cx->dmd, a); break;
        case 2: hipLaunchKernelGGL(gst::lg_gram_small<2>, g_gs, b_gs, 0, st, cx->dmd, a); break;
        case 3: hipLaunchKernelGGL(gst::lg_gram_small<3>, g_gs, b_gs, 0, st, cx->dmd, a); break;
        case 4: hipLaunchKernelGGL(gst::lg_gram_small<4>, g_gs, b_gs, 0, st, cx->dmd, a); break;
        case 5: hipLaunchKernelGGL(gst::lg_gram_small<5>, g_gs, b_gs, 0, st, cx->dmd, a); break;
        case 6: hipLaunchKernelGGL(gst::lg_gram_small<6>, g_gs, b_gs, 0, st, cx->dmd, a); break;
        default:
          hipLaunchKernelGGL(gst::lg_gram, g_gram, b_gram, gst::GRAM_LDS * 8, st, cx->dmd, a, nsb,
                             npairs);
      }
      HIP_OK(hipGetLastError());
      if (ev_mark(cx, GST_K_GRAM, st, false)) return -1;
      if (!eval_only) cx->gram_large += (unsigned long long)C;
      if (tm_needed) LG_LAUNCH(GST_K_TMELIM, gst::lg_tmelim, g_chain, b_chain, cx->lds_tm);
      if (!(mask & GST_STAGE_GRAM)) {   // timing diagnostic: Gram + TM elimination only
        if (launch_hyper(cx, a, hcls, g_hr8, b_hr8, g_hr16, b_hr16, g_chain, b_chain, st))
          return -1;
        if (eval_only) break;
        if ((mask & 4u) && !(cx->debug & GST_DEBUG_EXACT_BDRAW)) {
          // the b draw's floor pass (include/gst.h gst_sweep): chains whose Sigma is beyond
          // fp64 resolution re-eliminate G with Sigma + f I and draw there; every other chain
          // returns at once (SC_FLOOR == 0)
          a.floor_pass = 1;
          if (tm_needed) LG_LAUNCH(GST_K_TMELIM, gst::lg_tmelim, g_chain, b_chain, cx->lds_tm);
          if (launch_hyper(cx, a, hcls, g_hr8, b_hr8, g_hr16, b_hr16, g_chain, b_chain, st))
            return -1;
          a.floor_pass = 0;
        }
        if (mask & 4u) {
          if (tm_needed) LG_LAUNCH(GST_K_BTM, gst::lg_btm, g_chain, b_chain, cx->lds_btm);
          LG_LAUNCH(GST_K_TB, gst::lg_tb, g_tb, b_chain, 0);
        }
      }
    }
    if (!eval_only && (mask & 0x78u)) {
      if (tcls[0]) {
        a.kclass = 0;
        LG_LAUNCH(GST_K_TOA, gst::lg_toa<gst::TBLK_SMALL>, g_chain, dim3(gst::TBLK_SMALL), 0);
      }
      if (tcls[1]) {
        a.kclass = 1;
        LG_LAUNCH(GST_K_TOA, gst::lg_toa<gst::TBLK>, g_chain, dim3(gst::TBLK), 0);
      }
    }
  }
  HIP_OK(hipEventRecord(cx->ev1, st));
  cx->timed = true;
  return 0;
}

static int launch(Ctx* cx, const gst_state* s, const gst_records* r, const gst_tape* tp,
                  int C, int nsweeps, long long sweep0, int record_every, unsigned mask,
                  unsigned long long seed, long long chain0, int eval_only, double* ow,
                  double* oh, void* stream) {
  if (!cx || !cx->has_model) return fail("gst: no model set");
  if (!s || !s->x || !s->b || !s->z || !s->alpha || !s->pout || !s->theta || !s->nu)
    return fail("gst: state pointers must all be set");
  if (C <= 0) return 0;
  HIP_OK(hipSetDevice(cx->device));
  const bool tape = tp && tp->data;
  if (!s->dataset && cx->nd > 1)
    return fail("gst: the model has several datasets: state.dataset must be set");
  gst::DevState ds{s->x,     s->b,  s->z,      s->alpha,   s->pout, s->theta,
                   s->nu,    s->status, s->dataset, cx->nmax, cx->nd, nullptr, nullptr,
                   cx->debug, eval_only ? nullptr : cx->gram_cnt};
  gst::DevRec dr{};
  if (r) dr = gst::DevRec{r->x, r->b, r->z, r->alpha, r->pout, r->theta, r->nu, r->nrec};
  else record_every = 0;
  if (tape && tp->stride != gst_tape_stride(cx->nmax, cx->m))
    return fail("gst: tape stride mismatch");
  gst::DevTape dt{tape ? tp->data : nullptr, tape ? tp->stride : 0};
  if (cx->path == GST_PATH_LARGE)
    return launch_large(cx, ds, dr, dt, C, nsweeps, sweep0, record_every, mask, seed, chain0,
                        eval_only, ow, oh, (hipStream_t)stream);
  // chains per workgroup: the fewest (1, 2, default) that still fit one workgroup per CU
  int wpb = cx->WPB;
  if (!tape) {
    if (wpb >= 1 && C <= cx->ncu) wpb = 1;
    else if (wpb >= 2 && C <= 2 * cx->ncu) wpb = 2;
  }
  // two waves per chain when every chain would otherwise leave a SIMD idle (the general
  // white-noise instances too, since round 6)
  const bool pair = !tape && !eval_only && !(mask & GST_STAGE_GRAM) &&
                    (cx->waves == GST_WAVES_TWO || (cx->waves == GST_WAVES_AUTO && C <= 2 * cx->ncu));
  kfn_t k = pick(cx->MT, cx->NS, cx->K0, cx->raug, cx->gen, tape, wpb,
                 C > 4 * cx->ncu && cx->NS <= gst::OCC2_NS_MAX, pair);
  if (!k) return fail("gst: no kernel instance");
  // timing-model factor scratch: [C][waves per chain][slots with s < K0][64] doubles
  const int ntms = cx->MT * (cx->MT + 1) / 2 - (cx->MT - cx->K0) * (cx->MT - cx->K0 + 1) / 2;
  const size_t need = (size_t)C * (pair ? 2 : 1) * ntms * 64 * sizeof(double);
  hipStream_t st = (hipStream_t)stream;
  if (need > cx->tmfac_bytes) {
    free_tmfac(cx, st);
    HIP_OK(hipMallocAsync((void**)&cx->tmfac, need, st));
    cx->tmfac_bytes = need;
  }
  ds.tmfac = cx->tmfac;
  const dim3 grid(pair ? C : (C + wpb - 1) / wpb), block(pair ? 128 : 64 * wpb);
  // two chains per SIMD: the progress rule of fair_prio (with more chains than resident
  // slots, the later workgroups count as behind and the launch's tail shortens: config 4
  // 8.24 -> 8.32 M chain-sweeps/s).  Only in launches that run the red-noise block: the
  // counter's same-address atomics serialise at ~12 ns each across the XCDs, which a full
  // sweep hides but a stage-masked launch of a few microseconds per sweep would be timing
  if (!tape && !pair && C > 4 * cx->ncu && (mask & GST_STAGE_HYPER)) {
    HIP_OK(hipMemsetAsync(cx->prog, 0, sizeof(unsigned long long), st));
    ds.prog = cx->prog;
  }
  HIP_OK(hipEventRecord(cx->ev0, st));
  hipLaunchKernelGGL(k, grid, block, 0, st, cx->dmd, ds, dr, dt, C, nsweeps, sweep0,
                     record_every, mask, seed, chain0, eval_only, ow, oh);
  HIP_OK(hipGetLastError());
  HIP_OK(hipEventRecord(cx->ev1, st));
  cx->timed = true;
  return 0;
}

int gst_sweep(void* ctx, const gst_state* state, const gst_records* rec, const gst_tape* tape,
              int nchains, int nsweeps, long long sweep0, int record_every,
              unsigned stage_mask, unsigned long long seed, long long chain0, void* stream) {
  if (nsweeps < 0) return fail("gst_sweep: nsweeps < 0");
  if (rec && record_every > 0 && rec->nrec < (nsweeps + record_every - 1) / record_every)
    return fail("gst_sweep: record buffer too small");
  return launch(static_cast<Ctx*>(ctx), state, rec, tape, nchains, nsweeps, sweep0,
                record_every, stage_mask, seed, chain0, 0, nullptr, nullptr, stream);
}

int gst_eval_lnlike(void* ctx, const gst_state* state, int nchains, double* out_white,
                    double* out_hyper, void* stream) {
  if (!out_white || !out_hyper) return fail("gst_eval_lnlike: null outputs");
  return launch(static_cast<Ctx*>(ctx), state, nullptr, nullptr, nchains, 0, 0, 0, 0u, 0ull,
                0, 1, out_white, out_hyper, stream);
}

int gst_debug_stamps(void* ctx, unsigned long long* dev_buf) {
  Ctx* cx = static_cast<Ctx*>(ctx);
  if (!cx || !cx->has_model) return fail("gst_debug_stamps: no model");
#ifdef GST_STAMPS
  for (auto& h : cx->hmd) h.stamps = dev_buf;
  HIP_OK(hipMemcpy(cx->dmd, cx->hmd.data(), cx->hmd.size() * sizeof(gst::DevModel),
                   hipMemcpyHostToDevice));
  return 0;
#else
  (void)dev_buf;
  return fail("gst_debug_stamps: library built without GST_STAMPS");
#endif
}

int gst_sync(void* ctx, void* stream) {
  Ctx* cx = static_cast<Ctx*>(ctx);
  if (cx) HIP_OK(hipSetDevice(cx->device));
  HIP_OK(hipStreamSynchronize((hipStream_t)stream));
  return 0;
}

int gst_set_path(void* ctx, int path) {
  Ctx* cx = static_cast<Ctx*>(ctx);
  if (!cx) return fail("gst_set_path: null ctx");
  if (path < GST_PATH_AUTO || path > GST_PATH_LARGE) return fail("gst_set_path: bad path");
  cx->path_req = path;
  return 0;
}

int gst_set_waves(void* ctx, int waves) {
  Ctx* cx = static_cast<Ctx*>(ctx);
  if (!cx) return fail("gst_set_waves: null ctx");
  if (waves < GST_WAVES_AUTO || waves > GST_WAVES_TWO) return fail("gst_set_waves: bad value");
  cx->waves = waves;
  return 0;
}

int gst_set_debug(void* ctx, int flags) {
  Ctx* cx = static_cast<Ctx*>(ctx);
  if (!cx) return fail("gst_set_debug: null ctx");
  if (flags & ~(GST_DEBUG_POISON | GST_DEBUG_LARGE_GRAM | GST_DEBUG_LARGE_HYPER |
                GST_DEBUG_EXACT_BDRAW | GST_DEBUG_MFMA_GRAM | GST_DEBUG_EPOCHS_LDS))
    return fail("gst_set_debug: unknown flag");
  cx->debug = flags;
  return 0;
}

int gst_get_path(void* ctx, int* path) {
  Ctx* cx = static_cast<Ctx*>(ctx);
  if (!cx || !path) return fail("gst_get_path: null argument");
  if (!cx->has_model) return fail("gst_get_path: no model set");
  *path = cx->path;
  return 0;
}

int gst_set_timing(void* ctx, int on) {
  Ctx* cx = static_cast<Ctx*>(ctx);
  if (!cx) return fail("gst_set_timing: null ctx");
  cx->timing = on != 0;
  return 0;
}

int gst_kernel_times(void* ctx, double* ms, int* launches, int nkinds) {
  Ctx* cx = static_cast<Ctx*>(ctx);
  if (!cx || !ms || !launches) return fail("gst_kernel_times: null argument");
  for (int k = 0; k < nkinds; ++k) {
    ms[k] = 0.0;
    launches[k] = 0;
  }
  for (size_t i = 0; i < cx->evused; ++i) {
    const int k = cx->evkind[i];
    if (k < 0 || k >= nkinds) continue;
    HIP_OK(hipEventSynchronize(cx->evpool[2 * i + 1]));
    float f = 0.f;
    HIP_OK(hipEventElapsedTime(&f, cx->evpool[2 * i], cx->evpool[2 * i + 1]));
    ms[k] += f;
    launches[k] += 1;
  }
  return 0;
}

int gst_simulate(const gst_sim_desc* d, void* stream) {
  if (!d) return fail("gst_simulate: null descriptor");
  if (d->n <= 0 || d->ndatasets < 0 || d->ntm < 0 || d->nfourier < 0)
    return fail("gst_simulate: bad sizes");
  if (d->ndatasets == 0) return 0;
  if (d->nfourier > gst::SIM_MAX_NF || d->ntm > gst::SIM_MAX_NF)
    return fail("gst_simulate: nfourier and ntm must be <= 512");
  if (d->residuals_clean && d->ntm > gst::SIM_MAX_TM_CLEAN)
    return fail("gst_simulate: the clean twin needs ntm <= 64");
  if (!d->red && (!d->F || !d->log_f || !d->log_df) && d->nfourier > 0)
    return fail("gst_simulate: power-law red noise needs F, log_f and log_df");
  if ((d->ntm > 0 && !d->U) || !d->theta || !d->sigma_out || !d->dof ||
      (!d->red && (!d->log10_A || !d->gamma)) || !d->residuals || !d->toaerrs_out || !d->z)
    return fail("gst_simulate: missing pointer");
  gst::SimArgs a{};
  a.n = d->n;
  a.nf = d->red ? 0 : d->nfourier;
  a.ntm = d->ntm;
  a.D = d->ndatasets;
  a.F = d->F;
  a.lf = d->log_f;
  a.ldf = d->log_df;
  a.log_fyr = d->log_fyr;
  a.log_12pi2 = std::log(12.0) + 2.0 * std::log(M_PI);
  a.U = d->U;
  a.red = d->red;
  a.err_in = d->toaerrs;
  a.theta = d->theta;
  a.sigma_out = d->sigma_out;
  a.log10_A = d->log10_A;
  a.gamma = d->gamma;
  a.dof = d->dof;
  a.k0 = (uint32_t)(d->seed & 0xffffffffull);
  a.k1 = (uint32_t)(d->seed >> 32);
  a.ds0 = d->dataset0;
  a.r = d->residuals;
  a.err = d->toaerrs_out;
  a.z = d->z;
  a.r_clean = d->residuals_clean;
  hipLaunchKernelGGL(gst::gst_simulate_kernel, dim3(d->ndatasets), dim3(gst::SIM_BLOCK), 0,
                     (hipStream_t)stream, a);
  HIP_OK(hipGetLastError());
  return 0;
}

int gst_gram_counts(void* ctx, long long* counts, int reset) {
  Ctx* cx = static_cast<Ctx*>(ctx);
  if (!cx || !counts) return fail("gst_gram_counts: null argument");
  HIP_OK(hipSetDevice(cx->device));
  HIP_OK(hipDeviceSynchronize());
  unsigned long long h[2] = {0ull, 0ull};
  HIP_OK(hipMemcpy(h, cx->gram_cnt, sizeof h, hipMemcpyDeviceToHost));
  counts[0] = (long long)h[0];
  counts[1] = (long long)h[1];
  counts[2] = (long long)cx->gram_large;
  if (reset) {
    HIP_OK(hipMemset(cx->gram_cnt, 0, sizeof h));
    cx->gram_large = 0;
  }
  return 0;
}

int gst_debug_variates(int kind, double a, double b, long long n, unsigned long long seed,
                       unsigned call, double* out, void* stream) {
  if (!out || n < 0) return fail("gst_debug_variates: bad argument");
  if (kind < 0 || kind > 2) return fail("gst_debug_variates: kind must be 0, 1 or 2");
  if (!(a > 0.0) || (kind == 1 && !(b > 0.0))) return fail("gst_debug_variates: shapes must be > 0");
  if ((kind == 2 && n % 256) || n > (1ll << 31))
    return fail("gst_debug_variates: n must be <= 2^31 (kind 2: a multiple of 256)");
  if (n == 0) return 0;
  const long long threads = kind == 2 ? n / 4 : n;
  hipLaunchKernelGGL(debug_variates_kernel, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, kind, a, b, n, seed, call, out);
  HIP_OK(hipGetLastError());
  return 0;
}

int gst_last_sweep_ms(void* ctx, double* ms) {
  Ctx* cx = static_cast<Ctx*>(ctx);
  if (!cx || !ms) return fail("gst_last_sweep_ms: null argument");
  if (!cx->timed) return fail("gst_last_sweep_ms: nothing launched");
  HIP_OK(hipEventSynchronize(cx->ev1));
  float f = 0.f;
  HIP_OK(hipEventElapsedTime(&f, cx->ev0, cx->ev1));
  *ms = f;
  return 0;
}

}  // extern "C"
