#!/bin/bash
source tools/r3/run_guarded.sh
O=gpurun_out/r3f; mkdir -p $O
step 600 $O/bitwise2048.txt python -u tools/ab_bitwise.py gibbs_student_t_amd/libgst_base.so gibbs_student_t_amd/libgst.so 2048 60
step 600 $O/bitwise1024.txt python -u tools/ab_bitwise.py gibbs_student_t_amd/libgst_base.so gibbs_student_t_amd/libgst.so 1024 60
step 600 $O/ab.txt bash tools/ab_bench.sh gibbs_student_t_amd/libgst_base.so gibbs_student_t_amd/libgst.so
cat $O/ab.txt
bash tools/profile_r3.sh
