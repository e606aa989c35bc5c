#!/bin/bash
# round 3: gamma samplers with attempt 0 straight-line (gam), + branch-free z / alpha slots (gamz)
source tools/r3/run_guarded.sh
O=gpurun_out/r3gam; mkdir -p $O
L=gibbs_student_t_amd
step 600 $O/bitwise_gam.txt python -u tools/ab_bitwise.py $L/libgst_base.so $L/libgst_gam.so 2048 40
grep -h -E "bitwise|DIFFER" $O/bitwise_gam.txt
step 600 $O/bitwise_gamz.txt python -u tools/ab_bitwise.py $L/libgst_base.so $L/libgst_gamz.so 2048 40
grep -h -E "bitwise|DIFFER" $O/bitwise_gamz.txt
step 900 $O/ab.txt bash tools/ab_bench.sh $L/libgst_base.so $L/libgst_gam.so $L/libgst_gamz.so $L/libgst_base.so $L/libgst_gam.so $L/libgst_gamz.so
cat $O/ab.txt
echo CHECK_GAM_DONE
