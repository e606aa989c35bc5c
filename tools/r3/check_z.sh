#!/bin/bash
source tools/r3/run_guarded.sh
O=gpurun_out/r3z; mkdir -p $O
step 300 $O/midsize.txt $PYT -m gpu tests/test_gpu_midsize.py
grep -h -E "passed|failed" $O/midsize.txt | tail -1
echo CHECK_Z_DONE
