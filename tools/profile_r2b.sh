#!/bin/bash
# Round-2 (session 3) profile of the headline path after the spill / wave-priority work:
#   gpurun -- 'bash tools/profile_r2b.sh'
# bench lines (driver command, 500 sweeps, configs 3/4/5), rocprofv3 kernel stats of the
# 500-sweep headline run, and PMC passes (one counter group per run).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/prof_r2b
mkdir -p $O
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_driver.json 2> $O/bench_driver.err || exit 1
echo bench_driver done
B="python bench.py --no-cpu-baseline"
timeout -k 10 300 $B --steps 500 --warmup 100 > $O/bench_s500.json 2> $O/bench_s500.err || exit 1
timeout -k 10 200 $B --config 3 --steps 500 --warmup 100 > $O/bench_c3.json 2>&1 || exit 1
timeout -k 10 300 $B --config 4 --steps 200 --warmup 50 > $O/bench_c4.json 2>&1 || exit 1
timeout -k 10 200 $B --config 5 --steps 3 --warmup 1 > $O/bench_c5.json 2>&1 || exit 1
echo configs done
timeout -s KILL 150 rocprofv3 --kernel-trace --stats -d $O/ks -o ks --output-format csv -- \
  python bench.py --no-cpu-baseline --steps 500 --warmup 100 --ess-window 0 > $O/ks.log 2>&1 || exit 1
echo kernel stats done
P="python bench.py --no-cpu-baseline --steps 200 --warmup 20 --ess-window 0"
pass() {  # name, counters...
  local n=$1; shift
  timeout -s KILL 90 rocprofv3 --pmc "$@" -d $O/$n -o $n --output-format csv -- $P > $O/$n.log 2>&1
}
pass pf FETCH_SIZE || exit 1
pass pw WRITE_SIZE || exit 1
pass pa SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS || exit 1
pass pb SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_VALU_MFMA_BUSY_CYCLES || exit 1
pass pc SQ_WAIT_ANY SQ_INST_CYCLES_VMEM SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 GRBM_GUI_ACTIVE || exit 1
echo PROFILE_DONE
