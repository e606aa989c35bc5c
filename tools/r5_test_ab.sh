#!/bin/bash
# GPU suite on the in-tree library, then an interleaved A/B of library builds.
source tools/gpu_step.sh
O=gpurun_out/${TAG:-r5t}; mkdir -p $O
step 900 $O/gpu_tests.txt $PYT -m gpu ${TESTS:-tests/}
grep -h -E "passed|failed" $O/gpu_tests.txt
if [ -n "$AB" ]; then timeout -k 10 900 bash tools/ab_r5.sh ${ABR:-2} $AB; fi
