#!/bin/bash
# lg_hyper_ecr with per-epoch data in LDS: correctness, same-start tests, rates, profile
source tools/gpu_step.sh
O=gpurun_out/r6h; mkdir -p $O
step 600 $O/tests.txt $PYT tests/test_gpu_midsize.py -k "epochs or overlapping"
step 600 $O/tests_b.txt $PYT tests/test_gpu_parity.py -k "ebig or mb"
step 600 $O/tests_c.txt $PYT tests/test_gpu_ks.py -k "same_start"
export GR_PATHS=large
step 300 $O/rates.jsonl python tools/gen_rate.py 100 ebig,mb
step 200 $O/ebig_ks.log rocprofv3 --kernel-trace --stats -d $O/ebig_ks -o ebig --output-format csv -- \
  python tools/gen_rate.py 100 ebig
echo R6H_DONE
