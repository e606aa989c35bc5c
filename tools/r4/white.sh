#!/bin/bash
# Round 4: large-path white MH in speculative rounds -- parity (large path) and config-5 timing
source tools/gpu_step.sh
O=gpurun_out/r4w; mkdir -p $O
step 400 $O/tests.log $PYT tests/test_gpu_parity.py tests/test_gpu_midsize.py tests/test_gpu_fullsize.py tests/test_gpu_batch.py -k "large or midsize or fullsize or batch"
grep -E "passed|failed|FAILED" $O/tests.log | tail -5
step 200 $O/k5.log python tools/run_large.py 3 512
cat $O/k5.log
step 200 $O/mid.log python tools/run_large.py 10 1024 13000 30 14 10
cat $O/mid.log
