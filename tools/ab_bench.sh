#!/bin/bash
# A/B timing of libgst variants on the GPU box: tools/ab_bench.sh lib1.so lib2.so ...
# (bench.py headline config at 2048 and 1024 chains, config 3; no CPU leg, no ESS window)
set -o pipefail
mkdir -p gpurun_out/ab
for lib in "$@"; do
  n=$(basename $lib .so)
  CFGS=("--steps 500 --warmup 50" "--steps 20 --warmup 5" "--steps 500 --warmup 50 --chains 1024" "--config 3 --steps 500 --warmup 50")
  [ -n "$AB_QUICK" ] && CFGS=("--steps 500 --warmup 50" "--steps 20 --warmup 5")
  for a in "${CFGS[@]}"; do
    tag=$(echo "$a" | tr -d ' -')
    GST_ALLOW_ABI_MISMATCH=1 GST_LIB=$lib timeout -k 10 120 python -u bench.py --no-cpu-baseline --ess-window 0 $a \
      > gpurun_out/ab/$n.$tag.json 2> gpurun_out/ab/$n.$tag.err || { echo "FAIL $n $a"; tail -3 gpurun_out/ab/$n.$tag.err; exit 1; }
    python -c "import json,sys;d=json.load(open('gpurun_out/ab/$n.$tag.json'));print('%-14s %-40s %10.0f  kernel %.3f ms/sweep  frac %.3f'%('$n','$a',d['value'],d['kernel_ms']/d['steps'],d['roofline']['frac']))"
  done
done
