#!/bin/bash
# Round profile of the headline path (BASELINE config 2) plus configs 3/4, run on the GPU box:
#   gpurun -- 'bash tools/profile_config2.sh'
# Writes under gpurun_out/prof2/: bench lines, rocprofv3 kernel-trace stats, separate PMC
# passes (one counter group per run, MI355X_MICROARCH.md HBM recipe).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/prof2
mkdir -p $O
B="python bench.py --no-cpu-baseline"
timeout -k 10 300 python bench.py > $O/bench_default.log 2>&1 || exit 1
timeout -k 10 200 $B --config 3 --steps 500 --warmup 100 > $O/bench_c3.log 2>&1 || exit 1
timeout -k 10 200 $B --config 4 --steps 500 --warmup 100 > $O/bench_c4.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $O/ks -o ks --output-format csv -- \
  $B --steps 500 --warmup 100 > $O/ks.log 2>&1 || exit 1
P="$B --steps 200 --warmup 20"
pass() {  # name, counters...
  local n=$1; shift
  timeout -s KILL 90 rocprofv3 --pmc "$@" -d $O/$n -o $n --output-format csv -- $P > $O/$n.log 2>&1
}
pass pf FETCH_SIZE || exit 1
pass pw WRITE_SIZE || exit 1
pass pm SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS GRBM_GUI_ACTIVE || exit 1
pass pi SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_WAIT_ANY SQ_IFETCH SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE || exit 1
pass pc SQC_ICACHE_HITS SQC_ICACHE_MISSES || exit 1
echo PROFILE_DONE
