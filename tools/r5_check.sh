#!/bin/bash
# Round-5 GPU check: the GPU suite, then the driver's bench line.
source tools/gpu_step.sh
O=gpurun_out/${TAG:-r5a}; mkdir -p $O
step 900 $O/gpu_tests.txt $PYT -m gpu tests/ ${TESTS:-}
grep -h -E "passed|failed" $O/gpu_tests.txt
step 300 $O/bench_driver.json python bench.py --steps 20 --warmup 5
