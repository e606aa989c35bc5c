#!/bin/bash
# Round 6, first GPU pass: the new sampler / gate / ECORR-overlap tests, a driver-command
# bench line with the Gram path counts, and the epochs-first kernel's profile on ebig.
source tools/gpu_step.sh
O=gpurun_out/r6a; mkdir -p $O
step 900 $O/tests.txt $PYT -x tests/test_gpu_samplers.py \
  "tests/test_gpu_invariants.py::test_low_rank_gram_alpha_gate_and_path_counts" \
  "tests/test_gpu_invariants.py::test_low_rank_gram_matches_mfma_gram" \
  "tests/test_gpu_midsize.py::test_overlapping_ecorr_epochs_take_the_general_elimination" \
  "tests/test_gpu_midsize.py::test_epochs_first_hyper_matches_blocked_hyper"
step 300 $O/bench_driver.json python bench.py --steps 20 --warmup 5 --no-cpu-baseline
export GR_PATHS=large
step 200 $O/ebig_ks.log rocprofv3 --kernel-trace --stats -d $O/ebig_ks -o ebig --output-format csv -- \
  python tools/gen_rate.py 100 ebig
echo R6A_DONE
