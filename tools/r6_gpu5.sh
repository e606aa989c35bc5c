#!/bin/bash
# A/B: two chains per SIMD for the 12- / 16-slot shapes (libgst_occ2w.so) on the wide
# mid-size pulsars; the same-start mb test and the ecq exact-draw posterior test
source tools/gpu_step.sh
O=gpurun_out/r6e; mkdir -p $O
export MS_SIZES=5,7 MS_PATHS=persistent
for r in 1 2; do
  step 300 $O/mid_base_$r.log python tools/mid_size.py 2048 200
  GST_LIB=gibbs_student_t_amd/libgst_occ2w.so step 300 $O/mid_occ2w_$r.log python tools/mid_size.py 2048 200
done
step 600 $O/tests.txt $PYT tests/test_gpu_ks.py -k "same_start or exact_draw"
echo R6E_DONE
