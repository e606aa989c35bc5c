#!/bin/bash
# Round 6: lg_white two MH steps per pass, fused first pass, candidates in LDS -- full GPU
# suite, config 5 bench line and its kernel stats, ECORR / general white-noise rates.
source tools/gpu_step.sh
O=gpurun_out/r6w2; mkdir -p $O
step 900 $O/tests.txt $PYT -x -m gpu tests/
step 300 $O/bench_c5.json python bench.py --config 5 --steps 3 --warmup 1 --no-cpu-baseline
step 300 $O/c5_ks.log rocprofv3 --kernel-trace --stats -d $O/c5_ks -o c5 --output-format csv -- \
  python bench.py --config 5 --steps 3 --warmup 1 --no-cpu-baseline --ess-window 0
export GR_PATHS=large
step 300 $O/ec_rates.jsonl python tools/gen_rate.py 100 ebig,mb,jb
echo R6W_DONE
