#!/bin/bash
# round 3: 12- and 16-slot persistent shapes (n <= 1024): parity on the wide fixtures, the
# whole suite, and the mid-size survey against the large path
source tools/r3/run_guarded.sh
O=gpurun_out/r3y; mkdir -p $O
step 600 $O/wide_tests.txt $PYT -m gpu tests/test_gpu_parity.py tests/test_gpu_batch.py -k "wide or batch"
grep -h -E "passed|failed" $O/wide_tests.txt | tail -1
grep -h -E "^FAILED" $O/wide_tests.txt | head
step 900 $O/gpu_tests.txt $PYT -m gpu tests/
grep -h -E "passed|failed" $O/gpu_tests.txt | tail -1
step 400 $O/mid_size.txt python -u tools/mid_size.py 2048 100 $O/mid_size.json
cat $O/mid_size.txt | grep -v amdgpu
echo CHECK_Y_DONE
