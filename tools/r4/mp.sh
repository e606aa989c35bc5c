#!/bin/bash
# Round 4 experiment: owner-only publication stores (GST_MASKED_PUBLISH) -- parity, A/B, LDS PMC
source tools/gpu_step.sh
O=gpurun_out/r4mp; mkdir -p $O
export GST_ALLOW_ABI_MISMATCH=1
GST_LIB=gibbs_student_t_amd/libgst_mp.so step 400 $O/tests.log $PYT tests/test_gpu_parity.py tests/test_gpu_invariants.py tests/test_gpu_waves.py -k "not large"
grep -E "passed|failed" $O/tests.log | tail -2
AB_QUICK=1 step 900 $O/ab.log bash tools/ab_bench.sh gibbs_student_t_amd/libgst.so gibbs_student_t_amd/libgst_mp.so gibbs_student_t_amd/libgst.so gibbs_student_t_amd/libgst_mp.so
cat $O/ab.log
P="python bench.py --no-cpu-baseline --no-stage-costs --steps 200 --warmup 20 --ess-window 0"
for v in libgst libgst_mp; do
  GST_LIB=gibbs_student_t_amd/$v.so step 90 $O/pmc_$v.log rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VALU -d $O/pmc_$v -o p --output-format csv -- $P
done
echo MP_DONE
