#!/bin/bash
# round 3 (session 2): driver-command line at 2048 / 4096 / 8192 chains per GPU
source tools/r3/run_guarded.sh
O=gpurun_out/r3m; mkdir -p $O
for c in 2048 4096 8192; do
  step 300 $O/driver_c$c.json python bench.py --steps 20 --warmup 5 --chains $c
  grep '^{' $O/driver_c$c.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print($c, d['value'], d['ms_per_step'], d['ess_per_sec'], d['roofline']['frac'])"
done
echo CHECK_M_DONE
