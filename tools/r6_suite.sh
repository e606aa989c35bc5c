#!/bin/bash
# Full GPU suite + smoke of the current build.
source tools/gpu_step.sh
O=gpurun_out/${OUT:-r6suite}; mkdir -p $O
step 900 $O/tests.txt $PYT -m gpu tests/
grep -h -E "passed|failed" $O/tests.txt | tail -1
step 300 $O/smoke.txt python -c "import __graft_entry__ as g; g.smoke()"
tail -1 $O/smoke.txt
echo SUITE_DONE
