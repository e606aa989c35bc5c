#!/bin/bash
# Round-end check: full GPU suite, smoke, then the profile run (bench lines, rocprof, PMC):
#   gpurun -- 'ROUND=r4 bash tools/final_check.sh'
source tools/gpu_step.sh
O=gpurun_out/${ROUND:-r5}final; mkdir -p $O
step 900 $O/gpu_tests.txt $PYT -m gpu tests/
grep -h -E "passed|failed" $O/gpu_tests.txt
step 300 $O/smoke.txt python -c "import __graft_entry__ as g; g.smoke()"
tail -1 $O/smoke.txt
bash tools/profile.sh
