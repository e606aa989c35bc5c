#!/bin/bash
# Round 4, SVD-floor b draw: GPU parity + vvh17 tests, then A/B of the round-3 library.
source tools/gpu_step.sh
mkdir -p gpurun_out/r4
step 600 gpurun_out/r4/tests_floor.log $PYT tests/test_gpu_parity.py tests/test_gpu_ks.py tests/test_gpu_batch.py tests/test_gpu_midsize.py tests/test_gpu_invariants.py tests/test_gpu_waves.py
AB_QUICK=1 step 600 gpurun_out/r4/ab_floor.log bash tools/ab_bench.sh gibbs_student_t_amd/libgst_r3.so gibbs_student_t_amd/libgst.so gibbs_student_t_amd/libgst_tp3.so gibbs_student_t_amd/libgst_r3.so gibbs_student_t_amd/libgst.so gibbs_student_t_amd/libgst_tp3.so
cat gpurun_out/r4/ab_floor.log
# config 4 from the reference start: per-dataset R-hat, window draws of the studied datasets
step 300 gpurun_out/r4/c4_rhat.log python -u tools/config4_rhat.py gpurun_out/r4/c4_rhat.json gpurun_out/r4/c4 --save 220,162,160,235,115,175,241
tail -12 gpurun_out/r4/c4_rhat.log
