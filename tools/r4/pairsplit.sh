#!/bin/bash
# Round 4: pair mode draws z / alpha per half of the TOA slots -- bitwise tests (one-wave ==
# two-wave), configs, then config-3 A/B against the previous build
source tools/gpu_step.sh
O=gpurun_out/r4ps; mkdir -p $O
step 400 $O/tests.log $PYT tests/test_gpu_waves.py tests/test_gpu_configs.py tests/test_gpu_invariants.py tests/test_gpu_parity.py
grep -E "passed|failed|FAILED" $O/tests.log | tail -5
AB_CASES=j1713,c3 step 300 $O/bitwise.log python tools/ab_bitwise.py gibbs_student_t_amd/libgst_ab_head.so gibbs_student_t_amd/libgst.so 512 40
grep -E "identical|DIFFER" $O/bitwise.log
AB_CASES=c3,c20 step 300 $O/bitwise1024.log python tools/ab_bitwise.py gibbs_student_t_amd/libgst_ab_head.so gibbs_student_t_amd/libgst.so 1024 40
grep -E "identical|DIFFER" $O/bitwise1024.log
for r in 1 2 3; do
  for lib in gibbs_student_t_amd/libgst_ab_head.so gibbs_student_t_amd/libgst.so; do
    n=$(basename $lib .so)
    for a in "--config 3" "--chains 512" "--chains 1024"; do
      tag=$(echo "$a" | tr -d ' -')
      GST_LIB=$lib timeout -k 10 120 python -u bench.py --no-cpu-baseline --ess-window 0 --no-stage-costs $a --steps 500 --warmup 50 > $O/$n.$tag.$r.json 2> $O/$n.$tag.$r.err || { echo FAIL; tail -3 $O/$n.$tag.$r.err; exit 1; }
      python -c "import json;d=json.load(open('$O/$n.$tag.$r.json'));print('$n $tag r$r %10.0f kernel %.4f ms/sweep'%(d['value'],d['kernel_ms']/d['steps']))"
    done
  done
done
