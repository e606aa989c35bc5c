#!/bin/bash
# Round 4: the driver's short window (20 sweeps after 5 warmup) -- clock ramp or launch tail?
set -o pipefail
O=gpurun_out/r4s; mkdir -p $O
for a in "--steps 20 --warmup 5" "--steps 20 --warmup 3000" "--steps 500 --warmup 50" "--steps 20 --warmup 5" "--steps 20 --warmup 3000" "--steps 100 --warmup 3000"; do
  tag=$(echo "$a" | tr -d ' -')
  timeout -k 10 120 python -u bench.py --no-cpu-baseline --ess-window 0 --no-stage-costs $a > $O/$tag.json 2> $O/$tag.err || { echo "FAIL $a"; tail -3 $O/$tag.err; exit 1; }
  python -c "import json;d=json.load(open('$O/$tag.json'));print('%-28s %10.0f  kernel %.4f ms/sweep  wall %.4f ms/sweep'%('$a',d['value'],d['kernel_ms']/d['steps'],d['ms_per_step']))"
done
