#!/bin/bash
# round 3: general white-noise models (large path) + regression suite + A/B + profile
source tools/r3/run_guarded.sh
export GST_ALLOW_ABI_MISMATCH=1   # A/B against the pre-ABI-3 baseline build
O=gpurun_out/r3g; mkdir -p $O
step 600 $O/general.txt $PYT tests/test_gpu_parity.py -k "mb"
step 900 $O/gpu_tests.txt $PYT -m gpu tests/
step 600 $O/bitwise2048.txt python -u tools/ab_bitwise.py gibbs_student_t_amd/libgst_base.so gibbs_student_t_amd/libgst.so 2048 60
step 600 $O/ab.txt bash tools/ab_bench.sh gibbs_student_t_amd/libgst_base.so gibbs_student_t_amd/libgst.so
cat $O/ab.txt
step 300 $O/mid_size.txt python -u tools/mid_size.py 2048 100 $O/mid_size.json
bash tools/profile_r3.sh
