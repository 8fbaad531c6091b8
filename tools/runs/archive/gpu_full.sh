#!/bin/bash
# Full GPU check: all GPU tests, smoke, GPT-2 bench, reference model bench, reference
# 9-config table; each step under its own limit, stop at the first failure.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench1.log 2>&1 && \
timeout -k 10 300 python bench.py --model reference --mbs 8 --seq 128 --microbatches 4 --steps 20 --warmup 5 > gpurun_out/bench_ref.log 2>&1 && \
timeout -k 10 500 python -u tools/ref_table_gpu.py --json gpurun_out/ref_table_lanes.json > gpurun_out/ref_table_lanes.log 2>&1
