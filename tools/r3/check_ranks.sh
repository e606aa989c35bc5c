#!/bin/bash
# round 3: multi-rank bench path on one GPU (gloo ranks sharing the device)
source tools/r3/run_guarded.sh
O=gpurun_out/r3ranks; mkdir -p $O
step 300 $O/test.txt python -u -m pytest tests/test_gpu_ranks.py -x -v --timeout 280 --timeout-method thread
tail -3 $O/test.txt
export GST_DIST_BACKEND=gloo
step 300 $O/bench2.txt python -u bench.py --gpus 2 --steps 20 --warmup 5
tail -c 1500 $O/bench2.txt
echo CHECK_RANKS_DONE
