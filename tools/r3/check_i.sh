#!/bin/bash
# round 3 (session 2): regression suite on the restored tree + headline bench lines
source tools/r3/run_guarded.sh
O=gpurun_out/r3i; mkdir -p $O
step 900 $O/gpu_tests.txt $PYT -m gpu tests/
step 300 $O/bench_driver.json python bench.py --steps 20 --warmup 5
step 200 $O/bench_s500.json python bench.py --no-cpu-baseline --steps 500 --warmup 100
echo CHECK_I_DONE
