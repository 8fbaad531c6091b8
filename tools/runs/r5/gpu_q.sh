#!/bin/bash
# 8 ranks sharing one GPU over gloo: the driver's N = 8 bench path end to end (small batch,
# so 8 stashes fit one device), all schedules + the reference grid at P = 2 / 4 / 8.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r5q
export MIPIPE_DIST_BACKEND=gloo OMP_NUM_THREADS=1
timeout -k 10 600 python bench.py --gpus 8 --steps 3 --warmup 2 --mbs 4 --microbatches 16 --ref-grid l8h8 > gpurun_out/r5q/bench8.log 2>&1
rc=$?; grep '^{' gpurun_out/r5q/bench8.log | cut -c1-300; exit $rc
