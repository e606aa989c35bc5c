#!/bin/bash
# Round 4: lg_tb (64 chains per wave) and lg_tmelim (4 trailing tiles per wave round) --
# large-path parity with the candidate library, then timings
source tools/gpu_step.sh
O=gpurun_out/r4t; mkdir -p $O
GST_LIB=${CAND:-gibbs_student_t_amd/libgst.so} step 300 $O/tests.log $PYT tests/test_gpu_parity.py tests/test_gpu_midsize.py tests/test_gpu_fullsize.py tests/test_gpu_batch.py tests/test_gpu_configs.py -k "large or midsize or fullsize or batch"
grep -E "passed|failed|FAILED" $O/tests.log | tail -5
