#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 200 python -u -m pytest tests/test_f32_gpu.py -x -q --timeout 120 --timeout-method thread -k gemm > gpurun_out/f32_gemm_tests.log 2>&1 || { tail -5 gpurun_out/f32_gemm_tests.log; exit 1; }
MIPIPE_GEMM_F32_WAVES=4 timeout -k 10 200 python -u -m pytest tests/test_f32_gpu.py -x -q --timeout 120 --timeout-method thread -k gemm > gpurun_out/f32_gemm_tests4.log 2>&1 || { tail -5 gpurun_out/f32_gemm_tests4.log; exit 1; }
MIPIPE_GEMM_F32_WAVES=4 timeout -k 10 300 python -u tools/f32_gemm_sweep.py > gpurun_out/f32_sweep_w4.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/f32_gemm_sweep.py > gpurun_out/f32_sweep_w8.log 2>&1 || exit 1
tail -2 gpurun_out/f32_gemm_tests4.log
paste -d'\n' gpurun_out/f32_sweep_w8.log gpurun_out/f32_sweep_w4.log | grep shape | cut -c1-200
