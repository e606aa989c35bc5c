#!/bin/bash
# Round 6: config-5 kernel A/B (lg_tmelim TM_TILES 8, lg_tb TB_DEPTH 3) -- large-path tests,
# config-5 bench line and kernel stats.
source tools/gpu_step.sh
O=gpurun_out/r6c5; mkdir -p $O
step 600 $O/tests.txt $PYT -x tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_midsize.py -k "large or full or small or ecr or overlap"
step 300 $O/bench_c5.json python bench.py --config 5 --steps 3 --warmup 1 --no-cpu-baseline
step 300 $O/c5_ks.log rocprofv3 --kernel-trace --stats -d $O/c5_ks -o c5 --output-format csv -- \
  python bench.py --config 5 --steps 3 --warmup 1 --no-cpu-baseline --ess-window 0
echo R6C5_DONE
