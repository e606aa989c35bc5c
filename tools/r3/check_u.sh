#!/bin/bash
# round 3 (session 2): S0 loads before phi (T b unchanged): bitwise incl. the mid fixture,
# A/B timing, full GPU suite
source tools/r3/run_guarded.sh
O=gpurun_out/r3u; mkdir -p $O
export AB_CASES=j1713,c3,c20,tm22,mid
step 600 $O/bitwise2048.txt python -u tools/ab_bitwise.py gibbs_student_t_amd/libgst_base.so gibbs_student_t_amd/libgst.so 2048 60
step 300 $O/tape_mid.txt python -u tools/diag/tape_diff.py gibbs_student_t_amd/libgst_base.so gibbs_student_t_amd/libgst.so mid_beta_fixed 1
grep -h -E "bitwise|DIFFER" $O/bitwise*.txt; grep -v amdgpu $O/tape_mid.txt | grep -v identical
step 600 $O/ab.txt bash tools/ab_bench.sh gibbs_student_t_amd/libgst_base.so gibbs_student_t_amd/libgst.so gibbs_student_t_amd/libgst_base.so gibbs_student_t_amd/libgst.so
cat $O/ab.txt
step 900 $O/gpu_tests.txt $PYT -m gpu tests/
echo CHECK_U_DONE
