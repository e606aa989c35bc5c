#!/bin/bash
# round 3, first GPU pass: launch-boundary invariants + waves on the product library,
# then the reverted round-2 variant (tools/diag/variant_r2x.patch) localised by waves_diff
source tools/r3/run_guarded.sh
O=gpurun_out/r3a; mkdir -p $O
step 900 $O/inv_main.txt $PYT tests/test_gpu_invariants.py tests/test_gpu_waves.py
GST_LIB=gibbs_student_t_amd/libgst_r2x.so step 300 $O/waves_r2x.txt $PYT tests/test_gpu_waves.py -k two_waves_match
GST_LIB=gibbs_student_t_amd/libgst_r2x.so WD_S=40 step 300 $O/wd_r2x.txt python -u tools/diag/waves_diff.py beta_efac_fixed
step 300 $O/bench_default.txt python -u bench.py
