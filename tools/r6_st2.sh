#!/bin/bash
source tools/gpu_step.sh
O=gpurun_out/r6st2; mkdir -p $O
GR_PATHS=large GR_STAGES=1 step 300 $O/ec_stages.jsonl python tools/gen_rate.py 100 ebig,mb
step 300 $O/bench_c5.json python bench.py --config 5 --steps 3 --warmup 1 --no-cpu-baseline
echo R6ST2_DONE
