#!/bin/bash
# round 3 (session 2): one-wave-per-chain Gram for small models on the large path
source tools/r3/run_guarded.sh
O=gpurun_out/r3n; mkdir -p $O
step 600 $O/large_tests.txt $PYT -m gpu tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_batch.py tests/test_gpu_sampler.py tests/test_gpu_study.py -k "large or fullsize or mb or batch or study"
for n in 1000 4000 13000; do
  step 200 $O/large_n$n.txt python tools/run_large.py 10 1024 $n 30 14 10
done
step 200 $O/large_n13000_c2048.txt python tools/run_large.py 10 2048 13000 30 14 10
step 200 $O/run_large.txt python tools/run_large.py 3 512 100000 60 300 2
cat $O/large_n*.txt $O/run_large.txt
echo CHECK_N_DONE
