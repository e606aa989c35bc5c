#!/bin/bash
# round 3: one-wave vs two-wave over 150 sweeps (the length at which round 2 saw the main
# kernel diverge) on the f953150 library and the current one; A/B of the paired tail at
# one chain per SIMD
source tools/r3/run_guarded.sh
O=gpurun_out/r3d; mkdir -p $O
GST_LIB=gibbs_student_t_amd/libgst_f95.so WD_S=150 step 300 $O/wd150_f95.txt python -u tools/diag/waves_diff.py beta_efac_fixed
WD_S=150 step 300 $O/wd150_cur.txt python -u tools/diag/waves_diff.py beta_efac_fixed
GST_LIB=gibbs_student_t_amd/libgst_base.so WD_S=150 step 300 $O/wd150_base.txt python -u tools/diag/waves_diff.py beta_efac_fixed
step 600 $O/ab.txt bash tools/ab_bench.sh gibbs_student_t_amd/libgst_base.so gibbs_student_t_amd/libgst.so
cat $O/ab.txt
