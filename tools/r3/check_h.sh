#!/bin/bash
# round 3: large-path white-noise fix, stage-mask costs, progress counter off in stage launches
source tools/r3/run_guarded.sh
O=gpurun_out/r3h; mkdir -p $O
step 900 $O/gpu_tests.txt $PYT -m gpu tests/
step 200 $O/stages_c1024.txt python -u tools/stage_mask_timing.py 1024 100
step 200 $O/stages_c2048.txt python -u tools/stage_mask_timing.py 2048 100
step 200 $O/stages_c3.txt python -u tools/stage_mask_timing.py 512 100 c3
step 300 $O/bench_s500.json python bench.py --no-cpu-baseline --steps 500 --warmup 100
echo CHECK_H_DONE
