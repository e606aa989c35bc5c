#!/bin/bash
# usage: tools/gpu.sh '<command run on the GPU box>'  (logs under gpurun_out/)
cd /root/repo
timeout 1500 /usr/local/graft/bin/gpurun --timeout 900 -- "export TMPDIR=/tmp && $1" 2>&1 | tail -4
