#!/bin/bash
# round 3: the round-2 divergence on its own sources (f953150 + the reverted variant) vs a
# control build of f953150, and the current library's invariants
source tools/r3/run_guarded.sh
O=gpurun_out/r3b; mkdir -p $O
step 600 $O/inv_main.txt $PYT tests/test_gpu_invariants.py tests/test_gpu_waves.py
GST_LIB=gibbs_student_t_amd/libgst_f95.so step 300 $O/waves_f95.txt $PYT tests/test_gpu_waves.py -k "two_waves_match and beta_efac"
GST_LIB=gibbs_student_t_amd/libgst_f95x.so step 300 $O/waves_f95x.txt $PYT tests/test_gpu_waves.py -k "two_waves_match and beta_efac"
GST_LIB=gibbs_student_t_amd/libgst_f95x.so WD_S=40 step 300 $O/wd_f95x.txt python -u tools/diag/waves_diff.py beta_efac_fixed
GST_LIB=gibbs_student_t_amd/libgst_f95x.so step 600 $O/inv_f95x.txt $PYT tests/test_gpu_invariants.py
step 600 $O/cfg4_full.txt $PYT tests/test_gpu_config4_full.py
step 600 $O/vvh17_protocol.txt python -u tools/vvh17_protocol.py 1024 $O/vvh17_protocol.json
step 600 $O/cfg4_rhat.txt python -u tools/config4_rhat.py $O/config4_rhat.json $O/config4_worst.npz
