// Register-resident shapes of the persistent sweep kernel and the per-shape instance
// pickers.  Each shape's instances (tape / Philox, chains per workgroup, one or two chains
// per SIMD, two waves per chain) are compiled in a translation unit of their own
// (gst_inst.hip built once per shape with -DGST_SHAPE=..., in parallel; build.py), and
// gst.hip dispatches to them through pick_<shape>().
//
// Shape (MT, NS, K0, RA, GEN): MT = padded matrix dim / 8, NS = TOA slots of 64, K0 =
// timing-model panels of 8, RA = augmented-row index = 8*K0 + nfourier (+ n_ecorr) (elimination
// length), GEN = general white-noise model.
#pragma once
#include "gst_kernel.hpp"

namespace gst {

typedef void (*kfn_t)(const DevModel*, const DevState, const DevRec, const DevTape, int, int,
                      long long, int, unsigned, unsigned long long, long long, int, double*,
                      double*);

// X(MT, NS, K0, RA, GEN) for every instantiated shape (build.py reads this list); GEN = 1:
// the general white-noise model (per-backend efac / equad, ECORR columns; one chain per SIMD)
#define GST_SHAPES(X)                                                              \
  X(10, 2, 2, 76, 0) /* J1713-like, n <= 128 (no_outlier datasets) */                 \
  X(10, 3, 2, 76, 0) /* J1713+0747: n = 130, 30 red-noise components, 14 TM columns */ \
  X(10, 4, 2, 76, 0) /* n <= 256 */                                                   \
  X(10, 6, 2, 76, 0) /* mid-size pulsars: n <= 384 */                                 \
  X(10, 8, 2, 76, 0) /* n <= 512 */                                                   \
  X(10, 12, 2, 76, 0) /* wide mid-size (round 3): n <= 768, one chain per SIMD only */ \
  X(10, 16, 2, 76, 0) /* n <= 1024 */                                                 \
  X(8, 2, 2, 56, 0)  /* <= 20 red-noise components, <= 16 TM columns */               \
  X(8, 3, 2, 56, 0)                                                                   \
  X(8, 4, 2, 56, 0)                                                                   \
  X(8, 6, 2, 56, 0)                                                                   \
  X(8, 8, 2, 56, 0)                                                                   \
  X(10, 2, 3, 76, 0) /* <= 26 components with 17..24 TM columns */                    \
  X(10, 3, 3, 76, 0)                                                                  \
  X(10, 4, 3, 76, 0)                                                                  \
  X(10, 6, 3, 76, 0)                                                                  \
  X(10, 8, 3, 76, 0)                                                               \
  X(8, 2, 2, 62, 1) /* general white noise: <= 46 Fourier + ECORR columns, n <= 128 */ \
  X(8, 4, 2, 62, 1)                                                                \
  X(10, 2, 2, 76, 1) /* <= 60 Fourier + ECORR columns */                           \
  X(10, 3, 2, 76, 1) /* J1713+0747 with per-backend efac / equad: n = 130 */          \
  X(10, 4, 2, 76, 1)                                                               \
  X(10, 8, 2, 76, 1)

// tape: parity mode (4 chains per workgroup); wpb: chains per workgroup (4, or 2 / 1 for
// sampling launches with fewer chains than fill every SIMD); occ2: the two-chains-per-SIMD
// build (256 registers per lane); pair: two waves per chain (one chain per workgroup)
#define GST_PICK_NAME(mt, ns, k0, ra, gen) pick_##mt##_##ns##_##k0##_##ra##_##gen
#define GST_DECLARE_PICK(mt, ns, k0, ra, gen) \
  kfn_t GST_PICK_NAME(mt, ns, k0, ra, gen)(bool tape, int wpb, bool occ2, bool pair);
GST_SHAPES(GST_DECLARE_PICK)
#undef GST_DECLARE_PICK

}  // namespace gst
