#!/bin/bash
# round 3: localise the tape-kernel value difference of the pipelined T b (8-slot shape)
source tools/r3/run_guarded.sh
O=gpurun_out/r3x; mkdir -p $O
for v in newtb nosb plainptr ieeersq; do
  GST_LIB=gibbs_student_t_amd/libgst_$v.so step 300 $O/mid_$v.txt $PYT -m gpu tests/test_gpu_parity.py -k "mid and persistent"
  echo "$v: $(grep -h -E '(passed|failed) in' $O/mid_$v.txt)"
  step 300 $O/td_$v.txt python -u tools/diag/tape_diff.py gibbs_student_t_amd/libgst.so gibbs_student_t_amd/libgst_$v.so mid_beta_fixed 1
  grep -v amdgpu $O/td_$v.txt | grep -E "rec_b|rec_alpha" | head -2
done
echo CHECK_X_DONE
