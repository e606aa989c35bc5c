#!/bin/bash
# lg_hyper_ecr iteration: correctness against lg_hyper<2> and the fixtures, rates, profile
source tools/gpu_step.sh
O=gpurun_out/r6c; mkdir -p $O
step 600 $O/tests.txt $PYT tests/test_gpu_midsize.py -k "epochs or overlapping"
step 600 $O/tests_b.txt $PYT tests/test_gpu_parity.py -k "ebig or mb"
export GR_PATHS=large
step 300 $O/rates.jsonl python tools/gen_rate.py 100 ebig,mb
step 200 $O/ebig_ks.log rocprofv3 --kernel-trace --stats -d $O/ebig_ks -o ebig --output-format csv -- \
  python tools/gen_rate.py 100 ebig
echo R6C_DONE
