#!/bin/bash
# round 3: paired elimination tail -- bitwise vs the baseline build, GPU suite, A/B timing
source tools/r3/run_guarded.sh
O=gpurun_out/r3c; mkdir -p $O
step 600 $O/bitwise.txt python -u tools/ab_bitwise.py gibbs_student_t_amd/libgst_base.so gibbs_student_t_amd/libgst.so 2048 60
step 900 $O/gpu_tests.txt $PYT -m gpu tests/ -x
AB_QUICK=1 step 600 $O/ab.txt bash tools/ab_bench.sh gibbs_student_t_amd/libgst_base.so gibbs_student_t_amd/libgst.so
cat $O/ab.txt
