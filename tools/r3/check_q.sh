#!/bin/bash
# round 3 (session 2): which build breaks the mid-size (n = 390, 8 TOA slots) fixtures
source tools/r3/run_guarded.sh
O=gpurun_out/r3q; mkdir -p $O
GST_LIB=gibbs_student_t_amd/libgst_base.so step 300 $O/mid_base.txt $PYT -m gpu tests/test_gpu_parity.py -k "mid and persistent"
GST_LIB=gibbs_student_t_amd/libgst.so step 300 $O/mid_new.txt $PYT -m gpu tests/test_gpu_parity.py -k "mid and persistent"
grep -h -E "passed|failed" $O/mid_*.txt
echo CHECK_Q_DONE
