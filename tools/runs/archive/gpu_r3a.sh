#!/bin/bash
# Round-3 first GPU session: hardware-queue probe, full GPU suite, 1-GPU bench.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 120 python -u tools/queue_probe.py --out gpurun_out/r3_queue_probe.json > gpurun_out/queue_probe.log 2>&1 && \
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench1.log 2>&1 && \
tail -1 gpurun_out/bench1.log
