#!/bin/bash
# round 3 (session 2): large-path white-noise loop (hoisted pointers, 4 TOAs per round);
# large-path parity + config-5 timing; mid-size survey of both paths
source tools/r3/run_guarded.sh
O=gpurun_out/r3j; mkdir -p $O
step 600 $O/large_tests.txt $PYT -m gpu tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_batch.py -k "large or fullsize or mb or batch"
step 200 $O/run_large.txt python tools/run_large.py 3 512
step 300 $O/mid_size.txt python -u tools/mid_size.py 2048 100 $O/mid_size.json
for n in 1000 4000 13000; do
  step 200 $O/large_n$n.txt python tools/run_large.py 4 1024 $n 30 14
done
echo CHECK_J_DONE
