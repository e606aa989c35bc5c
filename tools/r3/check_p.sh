#!/bin/bash
# round 3 (session 2): S0 loads before phi, pipelined T b: bitwise vs the previous build,
# A/B timing, full GPU suite
source tools/r3/run_guarded.sh
O=gpurun_out/r3p; mkdir -p $O
step 600 $O/bitwise2048.txt python -u tools/ab_bitwise.py gibbs_student_t_amd/libgst_base.so gibbs_student_t_amd/libgst.so 2048 60
step 600 $O/bitwise1024.txt python -u tools/ab_bitwise.py gibbs_student_t_amd/libgst_base.so gibbs_student_t_amd/libgst.so 1024 60
grep -h bitwise $O/bitwise*.txt
step 600 $O/ab.txt bash tools/ab_bench.sh gibbs_student_t_amd/libgst_base.so gibbs_student_t_amd/libgst.so gibbs_student_t_amd/libgst_base.so gibbs_student_t_amd/libgst.so
cat $O/ab.txt
step 900 $O/gpu_tests.txt $PYT -m gpu tests/
echo CHECK_P_DONE
