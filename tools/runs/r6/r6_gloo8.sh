#!/bin/bash
# Round 6: 8 ranks sharing one GPU over gloo -- the driver's N = 8 bench path end to end with
# this round's code (schedule comparison on GPT-2 medium, reference-depth 1F1B, v2 attention).
# Throughput is time-shared here and means nothing; the record shows the flow and the fields.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r6g8
export MIPIPE_DIST_BACKEND=gloo OMP_NUM_THREADS=1
timeout -k 10 900 python bench.py --gpus 8 --steps 3 --warmup 2 --mbs 4 --microbatches 16 > gpurun_out/r6g8/bench8.log 2>&1
rc=$?; grep '^{' gpurun_out/r6g8/bench8.log | cut -c1-400; exit $rc
