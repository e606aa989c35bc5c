#!/bin/bash
# Round 6: two waves per chain for the general white-noise instances -- the two-wave bitwise
# tests first, then the full GPU suite and the GEN rates at 512 / 2048 chains.
source tools/gpu_step.sh
O=gpurun_out/r6gp; mkdir -p $O
step 600 $O/tests_w.txt $PYT -x tests/test_gpu_waves.py tests/test_gpu_invariants.py
step 900 $O/tests.txt $PYT -x -m gpu tests/
GR_PATHS=persistent step 300 $O/gen_rates.jsonl python tools/gen_rate.py 200 ecb,ecq,jb
echo R6GP_DONE
