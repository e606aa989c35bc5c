#!/bin/bash
source tools/gpu_step.sh
O=gpurun_out/r6d; mkdir -p $O
step 600 $O/tests.txt $PYT tests/test_gpu_midsize.py -k "epochs"
export GR_PATHS=large
step 300 $O/rates.jsonl python tools/gen_rate.py 100 ebig,mb
echo R6D_DONE
