#!/bin/bash
# Round 6 final profile of the final build: full GPU suite, smoke, bench lines (configs 2-5),
# rocprof kernel stats, PMC passes (tools/profile.sh), then the ECORR stage rates and the
# J1643-sized run.
export ROUND=r6
bash tools/final_check.sh || exit $?
source tools/gpu_step.sh
O=gpurun_out/r6final2; mkdir -p $O
GR_PATHS=large GR_STAGES=1 step 300 $O/ec_stages.jsonl python tools/gen_rate.py 100 ebig,mb,jb
step 300 $O/j1643.jsonl python tools/j1643_rate.py 2048 10
echo R6FINAL2_DONE
