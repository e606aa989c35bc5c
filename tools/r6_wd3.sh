#!/bin/bash
# Round 6: lg_white three MH steps per pass on one-wave chains; no-op launches skipped for
# class-2 batches -- full GPU suite, ECORR stage rates, config-5 line.
source tools/gpu_step.sh
O=gpurun_out/r6wd3; mkdir -p $O
step 900 $O/tests.txt $PYT -x -m gpu tests/
GR_PATHS=large GR_STAGES=1 step 300 $O/ec_stages.jsonl python tools/gen_rate.py 100 ebig,mb,jb
step 300 $O/bench_c5.json python bench.py --config 5 --steps 3 --warmup 1 --no-cpu-baseline
step 300 $O/j1643.jsonl python tools/j1643_rate.py 2048 10
echo R6WD3_DONE
