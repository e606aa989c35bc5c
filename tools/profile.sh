#!/bin/bash
# Profile of the current build:   gpurun -- 'ROUND=r4 bash tools/profile.sh'
# bench lines (driver command, default, configs 3/4/5), rocprofv3 kernel stats of the
# 500-sweep headline run, PMC passes of config 2 and of config 5 (one counter group per run);
# then: python tools/pmc_json.py gpurun_out/prof_$ROUND 200 2048 > profiles/${ROUND}_pmc_config2.json
source tools/gpu_step.sh
O=gpurun_out/prof_${ROUND:-r5}; mkdir -p $O
step 300 $O/bench_driver.json python bench.py --steps 20 --warmup 5
B="python bench.py --no-cpu-baseline"
step 300 $O/bench_s500.json $B --steps 500 --warmup 100
step 300 $O/bench_c1024.json $B --steps 500 --warmup 100 --chains 1024
step 200 $O/bench_c3.json $B --config 3 --steps 500 --warmup 100
step 400 $O/bench_c4.json $B --config 4 --steps 200 --warmup 50 --ess-window 20000
step 300 $O/bench_c5.json $B --config 5 --steps 3 --warmup 1
step 150 $O/ks.log rocprofv3 --kernel-trace --stats -d $O/ks -o ks --output-format csv -- \
  python bench.py --no-cpu-baseline --no-stage-costs --steps 500 --warmup 100 --ess-window 0
P="python bench.py --no-cpu-baseline --no-stage-costs --steps 200 --warmup 20 --ess-window 0"
pass() {  # name, counters...
  local n=$1; shift
  step 90 $O/$n.log rocprofv3 --pmc "$@" -d $O/$n -o $n --output-format csv -- $P
}
pass pf FETCH_SIZE
pass pw WRITE_SIZE
pass pa SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS
pass pb SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_VALU_MFMA_BUSY_CYCLES
pass pc SQ_WAIT_ANY SQ_INST_CYCLES_VMEM SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 GRBM_GUI_ACTIVE
L="python tools/run_large.py 3 512"
step 200 $O/k5.log rocprofv3 --kernel-trace --stats -d $O/k5 -o k5 --output-format csv -- $L
pass5() {
  local n=$1; shift
  step 200 $O/$n.log rocprofv3 --pmc "$@" -d $O/$n -o $n --output-format csv -- $L
}
pass5 pf5 FETCH_SIZE
pass5 pw5 WRITE_SIZE
pass5 pm5 SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE
echo PROFILE_DONE
