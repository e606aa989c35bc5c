#!/bin/bash
# Round 4: vvh17 escape vs the reference for floor constants 0.25 / 0.5 / 0.75 / 1, the
# statistical vvh17 tests, lg_hyper_reg<16>, an interleaved A/B of the round-3 library
# against this one, config 5, and config-4 mode fractions at 256 chains per dataset.
source tools/gpu_step.sh
mkdir -p gpurun_out/r4
step 400 gpurun_out/r4/tests_ks.log $PYT -s tests/test_gpu_ks.py tests/test_gpu_batch.py tests/test_gpu_midsize.py
grep -E "vvh17 escape|passed|failed|FAILED" gpurun_out/r4/tests_ks.log
step 400 gpurun_out/r4/tests_parity_large.log $PYT tests/test_gpu_parity.py -k large
grep -E "passed|failed|FAILED" gpurun_out/r4/tests_parity_large.log
for v in fc025 fc075 fc1; do
  GST_ALLOW_ABI_MISMATCH=1 GST_LIB=gibbs_student_t_amd/libgst_$v.so step 200 gpurun_out/r4/esc_$v.log $PYT -s tests/test_gpu_ks.py -k escapes
  grep "vvh17 escape" gpurun_out/r4/esc_$v.log
done
step 300 gpurun_out/r4/c5.json python -u bench.py --config 5 --steps 3 --warmup 1 --no-cpu-baseline
python -c "import json;d=json.load(open('gpurun_out/r4/c5.json'));print('config5', d['ms_per_step'], json.dumps(d.get('kernels', d.get('roofline',{}).get('kernels')))[:900])"
AB_QUICK=1 step 900 gpurun_out/r4/ab2.log bash tools/ab_bench.sh gibbs_student_t_amd/libgst_r3.so gibbs_student_t_amd/libgst.so gibbs_student_t_amd/libgst_r3.so gibbs_student_t_amd/libgst.so gibbs_student_t_amd/libgst_r3.so gibbs_student_t_amd/libgst.so
cat gpurun_out/r4/ab2.log
# config-4 mode fractions with 256 chains per dataset (65536 chains)
step 300 gpurun_out/r4/c4_256.log python -u tools/config4_rhat.py gpurun_out/r4/c4_rhat_256.json gpurun_out/r4/c4_256 --chains 256 --save 220,162
tail -3 gpurun_out/r4/c4_256.log
