#!/bin/bash
source tools/r3/run_guarded.sh
O=gpurun_out/r3t; mkdir -p $O
export TD_POISON_B=1
step 300 $O/tp_newtb.txt python -u tools/diag/tape_diff.py gibbs_student_t_amd/libgst_newtb.so gibbs_student_t_amd/libgst_newtb.so mid_beta_fixed 1
step 300 $O/tp_oldtb.txt python -u tools/diag/tape_diff.py gibbs_student_t_amd/libgst_oldtb.so gibbs_student_t_amd/libgst_oldtb.so mid_beta_fixed 1
step 300 $O/tp_oldtb_j.txt python -u tools/diag/tape_diff.py gibbs_student_t_amd/libgst_oldtb.so gibbs_student_t_amd/libgst_oldtb.so beta_fixed 1
for f in $O/tp_*.txt; do echo "== $f"; grep -v amdgpu $f | grep -v identical; done
echo CHECK_T_DONE
