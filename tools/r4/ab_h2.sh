#!/bin/bash
# Round 4: headline-build A/B (interleaved), 500-sweep and driver-command lines
set -o pipefail
O=gpurun_out/r4h2; mkdir -p $O
for r in 1 2 3; do
  for lib in "$@"; do
    n=$(basename $lib .so)
    for a in "--steps 500 --warmup 50" "--steps 20 --warmup 5"; do
      tag=$(echo "$a" | tr -d ' -')
      GST_LIB=$lib timeout -k 10 120 python -u bench.py --no-cpu-baseline --ess-window 0 --no-stage-costs $a > $O/$n.$tag.$r.json 2> $O/$n.$tag.$r.err || { echo FAIL; tail -3 $O/$n.$tag.$r.err; exit 1; }
      python -c "import json;d=json.load(open('$O/$n.$tag.$r.json'));print('$n $tag r$r %10.0f kernel %.4f ms/sweep'%(d['value'],d['kernel_ms']/d['steps']))"
    done
  done
done
