#!/bin/bash
# DP ZeRO-1: multi-rank GPU tests (DP x PP over gloo on one GPU: graphs + tape), then the
# BASELINE config 5 (DP2 x PP4) rehearsal with 8 ranks.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests/test_multirank_gpu.py tests/test_learning.py -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/z_multirank.log 2>&1
rc=$?; tail -3 gpurun_out/z_multirank.log; [ $rc -ne 0 ] && exit $rc
export MIPIPE_DIST_BACKEND=gloo OMP_NUM_THREADS=1
timeout -k 10 400 python bench.py --gpus 8 --dp 2 --model llama3-1b --recompute --mbs 1 --seq 1024 --steps 1 --warmup 1 > gpurun_out/z_cfg5.log 2>&1
rc=$?; grep '^{' gpurun_out/z_cfg5.log | cut -c1-200; exit $rc
