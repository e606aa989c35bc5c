#!/bin/bash
# Interleaved A/B of library builds on one box: tools/ab_r5.sh ROUNDS lib1.so lib2.so ...
# config 2 (500 sweeps and the driver's 20), config 3 and config 5 bench lines per library.
set -o pipefail
R=$1; shift
O=gpurun_out/ab5; mkdir -p $O
for r in $(seq 1 $R); do
for lib in "$@"; do
  n=$(basename $lib .so)
  for a in "--steps 500 --warmup 50" "--steps 20 --warmup 5" "--config 3 --steps 500 --warmup 50" ${AB_C5:+"--config 5 --steps 3 --warmup 1"}; do
    tag=$(echo "$a" | tr -d ' -')
    GST_LIB=$lib timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-stage-costs --ess-window 0 $a \
      > $O/$n.$tag.$r.json 2> $O/$n.$tag.$r.err || { echo "FAIL $n $a"; tail -3 $O/$n.$tag.$r.err; exit 1; }
    python -c "import json;d=json.load(open('$O/$n.$tag.$r.json'));print('%-16s %-38s %12.1f  kernel %.4f ms/sweep'%('$n','$a',d['value'],d['kernel_ms']/d['steps']))"
  done
done
done
