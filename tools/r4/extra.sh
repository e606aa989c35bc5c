#!/bin/bash
# Round 4 extras: GPU draws of config-4 dataset 160 at 256 chains per dataset (against the
# oracle's 256-chain runs), lg_white / lg_toa scaling with the chain count (config 5 shape)
source tools/gpu_step.sh
O=gpurun_out/r4x; mkdir -p $O
step 400 $O/c4_256.log python tools/config4_rhat.py $O/c4_rhat_256.json $O/c4x.npz --save 160 --chains 256
for c in 256 1024; do step 200 $O/k5_$c.log python tools/run_large.py 3 $c; grep -E "path|white|toa" $O/k5_$c.log; done
