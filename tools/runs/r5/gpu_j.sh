#!/bin/bash
# 4-rank stash test (gloo ranks sharing one GPU) + the bench (ZBH1 at P = 1 change).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r5j
timeout -k 10 600 python -u -m pytest -x -v --timeout 400 --timeout-method thread -m gpu tests/test_multirank_gpu.py -k "stash_follows" > gpurun_out/r5j/tests.log 2>&1
rc=$?; tail -4 gpurun_out/r5j/tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r5j/bench.log 2>&1
rc=$?; grep '^{' gpurun_out/r5j/bench.log | cut -c1-200; exit $rc
