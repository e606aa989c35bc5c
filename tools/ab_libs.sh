#!/bin/bash
# Interleaved A/B of library builds / settings on one GPU box, NAME:ENV[,ENV...] per variant:
#   tools/ab_libs.sh 3 base:GST_LIB=gibbs_student_t_amd/libgst.so tb16:GST_LIB=gibbs_student_t_amd/libgst_tb16.so
# (variants: GST_BUILD_VARIANT=name GST_EXTRA_CFLAGS=-D... python gibbs_student_t_amd/build.py)
# config 2 at 500 and 20 sweeps, config 3 at 500 sweeps per variant and round; AB_C4=1 adds
# config 4 (100 sweeps), AB_C5=1 config 5 (3 sweeps).
set -o pipefail
R=$1; shift
O=gpurun_out/ab52; mkdir -p $O
for r in $(seq 1 $R); do
for v in "$@"; do
  n=${v%%:*}; envs=${v#*:}
  for a in "--steps 500 --warmup 50" "--steps 20 --warmup 5" "--config 3 --steps 500 --warmup 50" ${AB_C4:+"--config 4 --steps 100 --warmup 20"} ${AB_C5:+"--config 5 --steps 3 --warmup 1"}; do
    tag=$(echo "$a" | tr -d ' -')
    env ${envs//,/ } timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-stage-costs --ess-window 0 $a \
      > $O/$n.$tag.$r.json 2> $O/$n.$tag.$r.err || { echo "FAIL $n $a"; tail -3 $O/$n.$tag.$r.err; exit 1; }
    python -c "import json;d=json.load(open('$O/$n.$tag.$r.json'));print('%-10s %-38s %12.1f  kernel %.4f ms/sweep'%('$n','$a',d['value'],d['kernel_ms']/d['steps']))"
  done
done
done
