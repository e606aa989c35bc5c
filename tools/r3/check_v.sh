#!/bin/bash
# round 3 (session 2): one-wave white passes for datasets up to 8k TOAs
source tools/r3/run_guarded.sh
O=gpurun_out/r3v; mkdir -p $O
step 600 $O/large_tests.txt $PYT -m gpu tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_batch.py tests/test_gpu_sampler.py tests/test_gpu_study.py tests/test_gpu_configs.py -k "large or fullsize or mb or batch or study"
grep -h -E "passed|failed" $O/large_tests.txt
for n in 1000 4000 13000; do
  step 200 $O/large_n$n.txt python tools/run_large.py 10 1024 $n 30 14 10
done
grep -h -E "path=|gram |white |hyper |toa " $O/large_n*.txt
echo CHECK_V_DONE
