#!/bin/bash
# PMC passes of the persistent kernel at a given chain count (one counter group per run).
#   gpurun -- 'bash tools/pmc_occ.sh 2048 r2occ'
set -o pipefail
export TMPDIR=/tmp
C=${1:-2048}; N=${2:-pmc}
O=gpurun_out/$N
mkdir -p $O
P="python bench.py --no-cpu-baseline --ess-window 0 --steps 100 --warmup 10 --chains $C"
pass() {  # name, counters...
  local n=$1; shift
  timeout -s KILL 90 rocprofv3 --pmc "$@" -d $O/$n -o $n --output-format csv -- $P > $O/$n.log 2>&1
}
pass pa SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS || exit 1
pass pb SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_VALU_MFMA_BUSY_CYCLES || exit 1
pass pc SQ_WAIT_ANY SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 GRBM_GUI_ACTIVE || exit 1
echo PMC_DONE
