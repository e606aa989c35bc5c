#!/bin/bash
# round 3 final: full GPU suite, smoke, then the profile run (bench lines, rocprof, PMC)
source tools/gpu_step.sh
O=gpurun_out/r3final; mkdir -p $O
step 900 $O/gpu_tests.txt $PYT -m gpu tests/
grep -h -E "passed|failed" $O/gpu_tests.txt
step 300 $O/smoke.txt python -c "import __graft_entry__ as g; g.smoke()"
tail -1 $O/smoke.txt
bash tools/profile_r3.sh
