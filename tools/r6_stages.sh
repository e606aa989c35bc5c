#!/bin/bash
# Round 6: per-stage large-path times of the ECORR fixtures (ebig, mb) at 512 / 2048 chains.
source tools/gpu_step.sh
O=gpurun_out/r6st; mkdir -p $O
GR_PATHS=large GR_STAGES=1 step 300 $O/ec_stages.jsonl python tools/gen_rate.py 100 ebig,mb
echo R6ST_DONE
