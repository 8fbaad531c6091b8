#!/bin/bash
# GEMM tests + reference-config table + 1-GPU bench, each step under its own limit.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_native_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/chk_test.log 2>&1 && \
timeout -k 10 400 python -u tools/ref_table_gpu.py --json gpurun_out/ref_table.json > gpurun_out/ref_table.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/chk_bench.log 2>&1
