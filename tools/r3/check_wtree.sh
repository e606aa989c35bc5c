#!/bin/bash
# round 3: white speculative tree with register-held step data
source tools/r3/run_guarded.sh
O=gpurun_out/r3wt; mkdir -p $O
step 600 $O/bitwise.txt python -u tools/ab_bitwise.py gibbs_student_t_amd/libgst_base.so gibbs_student_t_amd/libgst_wtree.so 2048 40
grep -h -E "bitwise|DIFFER" $O/bitwise.txt
step 600 $O/ab.txt bash tools/ab_bench.sh gibbs_student_t_amd/libgst_base.so gibbs_student_t_amd/libgst_wtree.so gibbs_student_t_amd/libgst_base.so gibbs_student_t_amd/libgst_wtree.so
cat $O/ab.txt
echo CHECK_AA_DONE
