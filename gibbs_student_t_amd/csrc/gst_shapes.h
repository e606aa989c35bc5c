// Register-resident shapes of the persistent sweep kernel and the per-shape instance
// pickers.  Each shape's instances (tape / Philox, chains per workgroup, one or two chains
// per SIMD, two waves per chain) are compiled in a translation unit of their own
// (gst_inst.hip built once per shape with -DGST_SHAPE=..., in parallel; build.py), and
// gst.hip dispatches to them through pick_<shape>().
//
// Shape (MT, NS, K0, RA): MT = padded matrix dim / 8, NS = TOA slots of 64, K0 =
// timing-model panels of 8, RA = augmented-row index = 8*K0 + nfourier (elimination length).
#pragma once
#include "gst_kernel.hpp"

namespace gst {

typedef void (*kfn_t)(const DevModel*, const DevState, const DevRec, const DevTape, int, int,
                      long long, int, unsigned, unsigned long long, long long, int, double*,
                      double*);

// X(MT, NS, K0, RA) for every instantiated shape (build.py reads this list)
#define GST_SHAPES(X)                                                              \
  X(10, 2, 2, 76) /* J1713-like, n <= 128 (no_outlier datasets) */                 \
  X(10, 3, 2, 76) /* J1713+0747: n = 130, 30 red-noise components, 14 TM columns */ \
  X(10, 4, 2, 76) /* n <= 256 */                                                   \
  X(10, 6, 2, 76) /* mid-size pulsars: n <= 384 */                                 \
  X(10, 8, 2, 76) /* n <= 512 */                                                   \
  X(10, 12, 2, 76) /* wide mid-size (round 3): n <= 768, one chain per SIMD only */ \
  X(10, 16, 2, 76) /* n <= 1024 */                                                 \
  X(8, 2, 2, 56)  /* <= 20 red-noise components, <= 16 TM columns */               \
  X(8, 3, 2, 56)                                                                   \
  X(8, 4, 2, 56)                                                                   \
  X(8, 6, 2, 56)                                                                   \
  X(8, 8, 2, 56)                                                                   \
  X(10, 2, 3, 76) /* <= 26 components with 17..24 TM columns */                    \
  X(10, 3, 3, 76)                                                                  \
  X(10, 4, 3, 76)                                                                  \
  X(10, 6, 3, 76)                                                                  \
  X(10, 8, 3, 76)

// tape: parity mode (4 chains per workgroup); wpb: chains per workgroup (4, or 2 / 1 for
// sampling launches with fewer chains than fill every SIMD); occ2: the two-chains-per-SIMD
// build (256 registers per lane); pair: two waves per chain (one chain per workgroup)
#define GST_PICK_NAME(mt, ns, k0, ra) pick_##mt##_##ns##_##k0##_##ra
#define GST_DECLARE_PICK(mt, ns, k0, ra) \
  kfn_t GST_PICK_NAME(mt, ns, k0, ra)(bool tape, int wpb, bool occ2, bool pair);
GST_SHAPES(GST_DECLARE_PICK)
#undef GST_DECLARE_PICK

}  // namespace gst
