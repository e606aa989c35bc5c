#!/bin/bash
# Round 4: A/B of large-path library variants (run_large per-kernel times), interleaved twice
set -o pipefail
O=gpurun_out/r4ab; mkdir -p $O
for r in 1 2; do
  for lib in "$@"; do
    n=$(basename $lib .so)
    GST_ALLOW_ABI_MISMATCH=1 GST_LIB=$lib timeout -k 10 150 python -u tools/run_large.py 3 512 100000 60 300 1 > $O/$n.k5.$r.log 2>&1 || { echo "FAIL $n"; tail -5 $O/$n.k5.$r.log; exit 1; }
    GST_ALLOW_ABI_MISMATCH=1 GST_LIB=$lib timeout -k 10 150 python -u tools/run_large.py 10 1024 13000 30 14 10 > $O/$n.mid.$r.log 2>&1 || { echo "FAIL $n mid"; tail -5 $O/$n.mid.$r.log; exit 1; }
    echo "== $n round $r"; grep -E "path=|white|toa" $O/$n.k5.$r.log $O/$n.mid.$r.log | sort -u
  done
done
