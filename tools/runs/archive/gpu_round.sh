#!/bin/bash
# One GPU session: tests, smoke, 1-GPU bench, rocprof kernel stats.  Each GPU step has its
# own time limit and the chain stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && \
timeout -k 10 600 python bench.py --steps 10 --warmup 3 > gpurun_out/bench1.log 2>&1 && \
tail -1 gpurun_out/bench1.log
