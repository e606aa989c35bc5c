#!/bin/bash
# Round 6 profile, second part: the ECORR kernels (rates, kernel stats, a PMC pass of
# lg_hyper_ecr and of lg_hyper<2>), the general white-noise rates and mid-size pulsars
source tools/gpu_step.sh
# (run after: gpurun -- 'ROUND=r6 bash tools/final_check.sh')
O=gpurun_out/r6final; mkdir -p $O
export GR_PATHS=large
step 300 $O/ec_rates.jsonl python tools/gen_rate.py 100 ebig,mb
GR_DEBUG=epochs_lds step 300 $O/ec_rates_lds.jsonl python tools/gen_rate.py 100 ebig,mb
step 200 $O/ebig_ks.log rocprofv3 --kernel-trace --stats -d $O/ebig_ks -o ebig --output-format csv -- \
  python tools/gen_rate.py 100 ebig
step 90 $O/ebig_pmc.log rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAIT_ANY -d $O/ebig_pmc -o pmc --output-format csv -- python tools/gen_rate.py 100 ebig
GR_DEBUG=epochs_lds step 90 $O/ebig_pmc_lds.log rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAIT_ANY -d $O/ebig_pmc_lds -o pmc --output-format csv -- python tools/gen_rate.py 100 ebig
export GR_PATHS=persistent,large
step 300 $O/gen_rates.jsonl python tools/gen_rate.py 200 ecb,ecq,jb
step 300 $O/mid_size.jsonl python tools/mid_size.py 2048 200
echo R6_FINAL_DONE
