#!/bin/bash
# Round 4: lg_white2 (two chains per workgroup) -- bitwise against the one-chain kernel on the
# large path (TB 64 / 256 / 1024 datasets), then timings
source tools/gpu_step.sh
O=gpurun_out/r4w2; mkdir -p $O
AB_PATH=large AB_CASES=j1713,c20,syn13k,syn40k step 400 $O/bitwise.log python tools/ab_bitwise.py gibbs_student_t_amd/libgst.so gibbs_student_t_amd/libgst_ab_w2.so 64 12
cat $O/bitwise.log | grep -E "identical|DIFFER"
bash tools/r4/ab_large.sh gibbs_student_t_amd/libgst.so gibbs_student_t_amd/libgst_ab_w2.so
