#!/bin/bash
# Round 4: instruction / wait counters of the large-path kernels (config 5, 3 sweeps)
source tools/gpu_step.sh
O=gpurun_out/r4p; mkdir -p $O
L="python tools/run_large.py 3 512"
p5() { local n=$1; shift; step 200 $O/$n.log rocprofv3 --pmc "$@" -d $O/$n -o $n --output-format csv -- $L; }
p5 pa5 SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS
p5 pc5 SQ_WAIT_ANY SQ_INST_CYCLES_VMEM SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VMEM_RD SQ_INSTS_SALU GRBM_GUI_ACTIVE
echo PMC5_DONE
