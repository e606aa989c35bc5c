// The persistent sweep kernel's instances for ONE shape, selected with
// -DGST_SHAPE=MT,NS,K0,RA,GEN (build.py compiles this file once per entry of GST_SHAPES, in
// parallel, and links the objects into libgst.so).
#include <hip/hip_runtime.h>

#include "gst_shapes.h"

#ifndef GST_SHAPE
#error "compile with -DGST_SHAPE=MT,NS,K0,RA,GEN"
#endif

namespace gst {
namespace {
template <int MT, int NS, int K0, int RA, bool TAPE, int WPB = 4, int OCC = 1, bool PAIR = false,
          bool GEN = false>
kfn_t kfn() {
  return &gst_sweep_kernel<MT, NS, K0, RA, TAPE, WPB, OCC, PAIR, GEN>;
}

// GEN shapes: the general white-noise model (pair mode since round 6)
template <int MT, int NS, int K0, int RA, int GEN>
kfn_t pick_shape(bool tape, int wpb, bool occ2, bool pair) {
  if constexpr (GEN != 0) {
    if (pair && !tape) return kfn<MT, NS, K0, RA, false, 2, 1, true, true>();
    if (tape) return kfn<MT, NS, K0, RA, true, 4, 1, false, true>();
    if (wpb == 1) return kfn<MT, NS, K0, RA, false, 1, 1, false, true>();
    if (wpb == 2) return kfn<MT, NS, K0, RA, false, 2, 1, false, true>();
    if (occ2 && occ_for(MT, K0) == 2) return kfn<MT, NS, K0, RA, false, 4, 2, false, true>();
    return kfn<MT, NS, K0, RA, false, 4, 1, false, true>();
  } else {
    if (tape) return kfn<MT, NS, K0, RA, true>();
    if (pair) return kfn<MT, NS, K0, RA, false, 2, 1, true>();
    if (wpb == 1) return kfn<MT, NS, K0, RA, false, 1>();
    if (wpb == 2) return kfn<MT, NS, K0, RA, false, 2>();
    if (occ2 && occ_for(MT, K0) == 2) return kfn<MT, NS, K0, RA, false, 4, 2>();
    return kfn<MT, NS, K0, RA, false>();
  }
}
}  // namespace

#define GST_DEFINE_PICK(mt, ns, k0, ra, gen)                                          \
  kfn_t GST_PICK_NAME(mt, ns, k0, ra, gen)(bool tape, int wpb, bool occ2, bool pair) { \
    return pick_shape<mt, ns, k0, ra, gen>(tape, wpb, occ2, pair);                    \
  }
#define GST_EXPAND(m, args) m args
GST_EXPAND(GST_DEFINE_PICK, (GST_SHAPE))

}  // namespace gst
