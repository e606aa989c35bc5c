#!/bin/bash
# round 3 (session 2): Gram k-loops without conditional loads (persistent kernel + large-path
# small Gram): bitwise vs the previous build, A/B timing, large-path tests, mid-size survey
source tools/r3/run_guarded.sh
O=gpurun_out/r3o; mkdir -p $O
step 600 $O/bitwise2048.txt python -u tools/ab_bitwise.py gibbs_student_t_amd/libgst_base.so gibbs_student_t_amd/libgst.so 2048 60
step 600 $O/bitwise1024.txt python -u tools/ab_bitwise.py gibbs_student_t_amd/libgst_base.so gibbs_student_t_amd/libgst.so 1024 60
step 600 $O/ab.txt bash tools/ab_bench.sh gibbs_student_t_amd/libgst_base.so gibbs_student_t_amd/libgst.so gibbs_student_t_amd/libgst_base.so gibbs_student_t_amd/libgst.so
cat $O/ab.txt
step 600 $O/large_tests.txt $PYT -m gpu tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_batch.py tests/test_gpu_sampler.py tests/test_gpu_study.py -k "large or fullsize or mb or batch or study"
for n in 1000 4000 13000; do
  step 200 $O/large_n$n.txt python tools/run_large.py 10 1024 $n 30 14 10
done
grep -h -E "path=|gram |white |hyper " $O/large_n*.txt
echo CHECK_O_DONE
