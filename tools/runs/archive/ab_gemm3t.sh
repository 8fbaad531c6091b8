#!/bin/bash
# TT (dW) ping-pong engine: numerics, then dW microbench vs the gemm2 TT engine, then bench
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "gemm" --timeout 120 --timeout-method thread > gpurun_out/g3t_test.log 2>&1 && \
MIPIPE_GEMM3T=0 timeout -k 10 300 python tools/bench_kernels.py --only dw > gpurun_out/g3t_off.log 2>&1 && \
timeout -k 10 300 python tools/bench_kernels.py --only dw > gpurun_out/g3t_on.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/g3t_bench.log 2>&1
