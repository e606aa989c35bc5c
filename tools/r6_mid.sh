#!/bin/bash
# Round 6: mid-size pulsars on both paths with the current build (stage breakdown of the large
# path).
source tools/gpu_step.sh
O=gpurun_out/r6mid; mkdir -p $O
MS_SIZES=5,7 step 400 $O/mid_size.jsonl python tools/mid_size.py 2048 200
echo R6MID_DONE
