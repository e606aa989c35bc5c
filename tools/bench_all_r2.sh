#!/bin/bash
# Round-2 bench lines (one JSON line each) for BASELINE configs 2-5, into gpurun_out/.
set -o pipefail
mkdir -p gpurun_out
run() {  # name, timeout, args...
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" python -u bench.py "$@" > "gpurun_out/$name.json" 2> "gpurun_out/$name.err" || {
    echo "FAILED $name"; tail -5 "gpurun_out/$name.err"; exit 1; }
  echo "done $name"
}
run r2_bench_driver 240 --steps 20 --warmup 5
run r2_bench_s500 240 --steps 500 --warmup 100
run r2_bench_c3 240 --config 3 --steps 500 --warmup 100
run r2_bench_c4 420 --config 4 --steps 200 --warmup 50
run r2_bench_c5 420 --config 5 --steps 3 --warmup 1
