#!/bin/bash
source tools/r3/run_guarded.sh
O=gpurun_out/r3w; mkdir -p $O
step 300 $O/midsize.txt $PYT -m gpu tests/test_gpu_midsize.py
grep -h -E "passed|failed|Error|assert" $O/midsize.txt | head -20
step 900 $O/gpu_tests.txt $PYT -m gpu tests/
grep -h -E "passed|failed" $O/gpu_tests.txt
echo CHECK_W_DONE
