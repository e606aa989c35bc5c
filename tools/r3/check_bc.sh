#!/bin/bash
# round 3: paired tail vs baseline (bitwise, A/B), the round-2 divergence on its own sources,
# the GPU suite on the paired build, config-4 full size, vvh17 protocol, config-4 R-hat
source tools/r3/run_guarded.sh
O=gpurun_out/r3b; mkdir -p $O
step 600 $O/bitwise.txt python -u tools/ab_bitwise.py gibbs_student_t_amd/libgst_base.so gibbs_student_t_amd/libgst.so 2048 60
AB_QUICK=1 step 600 $O/ab.txt bash tools/ab_bench.sh gibbs_student_t_amd/libgst_base.so gibbs_student_t_amd/libgst.so
GST_LIB=gibbs_student_t_amd/libgst_f95.so step 300 $O/waves_f95.txt $PYT tests/test_gpu_waves.py -k "two_waves_match and beta_efac"
GST_LIB=gibbs_student_t_amd/libgst_f95x.so step 300 $O/waves_f95x.txt $PYT tests/test_gpu_waves.py -k "two_waves_match and beta_efac"
GST_LIB=gibbs_student_t_amd/libgst_f95x.so WD_S=40 step 300 $O/wd_f95x.txt python -u tools/diag/waves_diff.py beta_efac_fixed
GST_LIB=gibbs_student_t_amd/libgst_f95x.so step 600 $O/inv_f95x.txt $PYT tests/test_gpu_invariants.py
step 900 $O/gpu_tests.txt $PYT -m gpu tests/
step 600 $O/vvh17_protocol.txt python -u tools/vvh17_protocol.py 1024 $O/vvh17_protocol.json
step 600 $O/cfg4_rhat.txt python -u tools/config4_rhat.py $O/config4_rhat.json $O/config4_worst.npz
