#!/bin/bash
# Round 6: structured ECORR Gram (lg_gram_ec) -- ECORR parity tests first, then the full GPU
# suite, ECORR rates and the J1643-sized run.
source tools/gpu_step.sh
O=${OUT:-gpurun_out/r6gec}; mkdir -p $O
step 600 $O/tests_ec.txt $PYT -x tests/test_gpu_parity.py tests/test_gpu_midsize.py -k "mb or ebig or ecr or overlap or epochs"
step 900 $O/tests.txt $PYT -x -m gpu tests/
export GR_PATHS=large
step 300 $O/ec_rates.jsonl python tools/gen_rate.py 100 ebig,mb
step 300 $O/j1643.jsonl python tools/j1643_rate.py 2048 10
echo R6GEC_DONE
