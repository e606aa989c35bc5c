#!/bin/bash
# round 3 re-entry check of the current build: full GPU suite, smoke, the driver's bench command
source tools/gpu_step.sh
O=gpurun_out/r3v; mkdir -p $O
step 900 $O/gpu_tests.txt $PYT -m gpu tests/
grep -h -E "passed|failed" $O/gpu_tests.txt
step 300 $O/smoke.txt python -c "import __graft_entry__ as g; g.smoke()"
tail -1 $O/smoke.txt
step 300 $O/bench_driver.json python bench.py --steps 20 --warmup 5
step 300 $O/bench_s500.json python bench.py --no-cpu-baseline --steps 500 --warmup 100
echo VALIDATE_DONE
