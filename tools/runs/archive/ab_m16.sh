#!/bin/bash
# A/B of the 16x16x32-MFMA GEMM engines (default) against the 32x32x16 builds
# (MIPIPE_GEMM_M16=0): numerics tests, then interleaved per-shape microbench, then bench.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "gemm" --timeout 120 --timeout-method thread > gpurun_out/m16_test.log 2>&1 && \
MIPIPE_GEMM_M16=0 timeout -k 10 300 python tools/bench_kernels.py --only _ > gpurun_out/m16_off.log 2>&1 && \
timeout -k 10 300 python tools/bench_kernels.py --only _ > gpurun_out/m16_on.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/m16_bench.log 2>&1 && tail -1 gpurun_out/m16_bench.log
