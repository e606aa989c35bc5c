#!/bin/bash
# round 3 (session 2): per-stage cycles (stamps build) at 512 chains (two waves per chain /
# one wave) and 2048 chains
source tools/r3/run_guarded.sh
O=gpurun_out/r3k; mkdir -p $O
export GST_LIB=gibbs_student_t_amd/libgst_stamps.so
step 200 $O/stages_512_auto.txt python -u tools/stage_profile.py 512 100
step 200 $O/stages_512_one.txt python -u tools/stage_profile.py 512 100 1
step 200 $O/stages_2048.txt python -u tools/stage_profile.py 2048 100
cat $O/stages_*.txt
echo CHECK_K_DONE
