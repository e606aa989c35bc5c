#!/bin/bash
# rocprof kernel stats of the GEN pair build (jb / ecb, 512 and 2048 chains, persistent path).
source tools/gpu_step.sh
O=gpurun_out/r6jb; mkdir -p $O
GR_PATHS=persistent step 300 $O/jb_ks.log rocprofv3 --kernel-trace --stats -d $O/ks -o jb --output-format csv -- python tools/gen_rate.py 200 jb,ecb
echo R6JB_DONE
