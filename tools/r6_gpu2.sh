#!/bin/bash
# Round 6, second GPU pass: the one-wave epochs-first kernel (lg_hyper_ecr) against
# lg_hyper<2> and the reference fixtures, the sampler tests, ebig / mb rates and profile.
source tools/gpu_step.sh
O=gpurun_out/r6b; mkdir -p $O
step 900 $O/tests_a.txt $PYT tests/test_gpu_samplers.py tests/test_gpu_midsize.py \
  "tests/test_gpu_invariants.py::test_low_rank_gram_alpha_gate_and_path_counts"
step 900 $O/tests_b.txt $PYT tests/test_gpu_parity.py -k "ebig or mb"
export GR_PATHS=large
step 300 $O/rates.jsonl python tools/gen_rate.py 100 ebig,mb
step 200 $O/ebig_ks.log rocprofv3 --kernel-trace --stats -d $O/ebig_ks -o ebig --output-format csv -- \
  python tools/gen_rate.py 100 ebig
echo R6B_DONE
