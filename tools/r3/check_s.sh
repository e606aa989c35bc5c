#!/bin/bash
source tools/r3/run_guarded.sh
O=gpurun_out/r3s; mkdir -p $O
export AB_CASES=mid,j1713
step 300 $O/bw_old_new.txt python -u tools/ab_bitwise.py gibbs_student_t_amd/libgst_oldtb.so gibbs_student_t_amd/libgst_newtb.so 64 20
step 300 $O/bw_base_old.txt python -u tools/ab_bitwise.py gibbs_student_t_amd/libgst_base.so gibbs_student_t_amd/libgst_oldtb.so 64 20
grep -h -E "bitwise|DIFFER" $O/bw_*.txt
echo CHECK_S_DONE
