#!/bin/bash
# Round 4: per-TOA block sizes for mid-size pulsars (2k / 13k TOAs, 1024 chains), interleaved
set -o pipefail
O=gpurun_out/r4mid; mkdir -p $O
for r in 1 2; do
  for lib in "$@"; do
    n=$(basename $lib .so)
    for shape in "10 1024 13000 30 14 10" "10 1024 2000 30 14 10"; do
      tag=$(echo $shape | cut -d' ' -f3)
      GST_ALLOW_ABI_MISMATCH=1 GST_LIB=$lib timeout -k 10 150 python -u tools/run_large.py $shape > $O/$n.$tag.$r.log 2>&1 || { echo "FAIL $n $shape"; tail -5 $O/$n.$tag.$r.log; exit 1; }
      echo "$n $tag r$r: $(grep -E 'path=' $O/$n.$tag.$r.log)  white $(grep white $O/$n.$tag.$r.log | awk '{print $2}')  toa $(grep toa $O/$n.$tag.$r.log | awk '{print $2}')"
    done
  done
done
