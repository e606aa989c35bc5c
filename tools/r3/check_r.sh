#!/bin/bash
source tools/r3/run_guarded.sh
O=gpurun_out/r3r; mkdir -p $O
GST_LIB=gibbs_student_t_amd/libgst_oldtb.so step 300 $O/mid_oldtb.txt $PYT -m gpu tests/test_gpu_parity.py -k "mid and persistent"
grep -h -E "passed|failed" $O/mid_*.txt
echo CHECK_R_DONE
