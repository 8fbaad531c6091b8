#!/bin/bash
# Prefetching GEMM epilogue: numerics + epilogue probe + headline bench.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r5o
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_kernels_gpu.py -k "gemm" > gpurun_out/r5o/tests.log 2>&1
rc=$?; tail -3 gpurun_out/r5o/tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python tools/gemm_epi_probe.py --graph > gpurun_out/r5o/epi_graph.txt 2>&1
rc=$?; grep -v "^{" gpurun_out/r5o/epi_graph.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --schedules none --ref-fp32 0 > gpurun_out/r5o/bench.log 2>&1
rc=$?; grep '^{' gpurun_out/r5o/bench.log | cut -c1-260; exit $rc
