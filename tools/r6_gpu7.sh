#!/bin/bash
# lg_hyper_ecr: batched b-draw epoch rows, RA-trimmed instance; per-backend split A/B
source tools/gpu_step.sh
O=gpurun_out/r6g; mkdir -p $O
step 600 $O/tests.txt $PYT tests/test_gpu_midsize.py -k "epochs or overlapping"
step 600 $O/tests_b.txt $PYT tests/test_gpu_parity.py -k "ebig or mb"
export GR_PATHS=large
for r in 1 2; do
  step 300 $O/rates_split_$r.jsonl python tools/gen_rate.py 100 ebig,mb
  GST_LIB=gibbs_student_t_amd/libgst_nosplit.so step 300 $O/rates_nosplit_$r.jsonl python tools/gen_rate.py 100 ebig,mb
done
step 200 $O/ebig_ks.log rocprofv3 --kernel-trace --stats -d $O/ebig_ks -o ebig --output-format csv -- \
  python tools/gen_rate.py 100 ebig
echo R6G_DONE
