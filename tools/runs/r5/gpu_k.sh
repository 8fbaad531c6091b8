#!/bin/bash
# 4-rank stash test (head lag capped) + headline bench + kernel stats of the headline step.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r5k
timeout -k 10 600 python -u -m pytest -x -v --timeout 400 --timeout-method thread -m gpu tests/test_multirank_gpu.py -k "stash_follows" > gpurun_out/r5k/tests.log 2>&1
rc=$?; tail -4 gpurun_out/r5k/tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r5k/bench.log 2>&1
rc=$?; grep '^{' gpurun_out/r5k/bench.log | cut -c1-300; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r5k/prof -o run -- python3 bench.py --gpus 1 --steps 10 --warmup 3 --schedules none --ref-fp32 0 --no-supervise --no-bubble > gpurun_out/r5k/prof.log 2>&1
rc=$?; find gpurun_out/r5k/prof -name "*kernel_stats.csv" | head -3; exit $rc
