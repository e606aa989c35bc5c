#!/bin/bash
# Round 5: config-4 same-start draws (256 chains per dataset; datasets 160, 220), the config-4
# bench line with a 20000-sweep ESS window, and the config 3 / 5 bench lines.
source tools/gpu_step.sh
O=gpurun_out/${TAG:-r5c4}; mkdir -p $O
step 600 $O/c4rhat.log python -u tools/config4_rhat.py $O/c4rhat_256.json $O/c4w256.npz --save 160,220 --chains 256
B="python bench.py --no-cpu-baseline"
step 400 $O/bench_c4.json $B --config 4 --steps 200 --warmup 50 --ess-window 20000
step 300 $O/bench_c5.json $B --config 5 --steps 3 --warmup 1
step 300 $O/bench_c3.json $B --config 3 --steps 500 --warmup 100
