#!/bin/bash
# round 3: per-stage stamps incl. record / white sub-stages (diagnostic libgst_stamps.so)
source tools/r3/run_guarded.sh
O=gpurun_out/r3stamps; mkdir -p $O
export GST_LIB=gibbs_student_t_amd/libgst_stamps.so
step 300 $O/c2048.txt python -u tools/stage_profile.py 2048 100
step 300 $O/c512.txt python -u tools/stage_profile.py 512 100
cat $O/c2048.txt $O/c512.txt
echo CHECK_STAMPS_DONE
