// The persistent sweep kernel's instances for ONE shape, selected with
// -DGST_SHAPE=MT,NS,K0,RA (build.py compiles this file once per entry of GST_SHAPES, in
// parallel, and links the objects into libgst.so).
#include <hip/hip_runtime.h>

#include "gst_shapes.h"

#ifndef GST_SHAPE
#error "compile with -DGST_SHAPE=MT,NS,K0,RA"
#endif

namespace gst {
namespace {
template <int MT, int NS, int K0, int RA, bool TAPE, int WPB = 4, int OCC = 1, bool PAIR = false>
kfn_t kfn() {
  return &gst_sweep_kernel<MT, NS, K0, RA, TAPE, WPB, OCC, PAIR>;
}
}  // namespace

#define GST_DEFINE_PICK(mt, ns, k0, ra)                                             \
  kfn_t GST_PICK_NAME(mt, ns, k0, ra)(bool tape, int wpb, bool occ2, bool pair) {    \
    if (tape) return kfn<mt, ns, k0, ra, true>();                                   \
    if (pair) return kfn<mt, ns, k0, ra, false, 2, 1, true>();                      \
    if (wpb == 1) return kfn<mt, ns, k0, ra, false, 1>();                           \
    if (wpb == 2) return kfn<mt, ns, k0, ra, false, 2>();                           \
    if (occ2 && occ_for(mt, k0) == 2) return kfn<mt, ns, k0, ra, false, 4, 2>();    \
    return kfn<mt, ns, k0, ra, false>();                                            \
  }
#define GST_EXPAND(m, args) m args
GST_EXPAND(GST_DEFINE_PICK, (GST_SHAPE))

}  // namespace gst
