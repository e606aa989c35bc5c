#!/bin/bash
# round 3 (session 2): per-TOA passes of the large path with 4-wave chains for datasets of
# up to 32k TOAs; large-path parity; mid-size survey; config 5 unchanged
source tools/r3/run_guarded.sh
O=gpurun_out/r3l; mkdir -p $O
step 600 $O/large_tests.txt $PYT -m gpu tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_batch.py tests/test_gpu_sampler.py tests/test_gpu_study.py -k "large or fullsize or mb or batch or study"
for n in 1000 4000 13000; do
  step 200 $O/large_n$n.txt python tools/run_large.py 4 1024 $n 30 14
done
step 200 $O/run_large.txt python tools/run_large.py 3 512
cat $O/large_n*.txt
echo CHECK_L_DONE
