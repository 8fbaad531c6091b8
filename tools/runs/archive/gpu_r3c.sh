#!/bin/bash
# f32 kernels: numerics tests, GEMM split sweep, f32 microbench (GEMM + attention).
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_f32_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/f32_tests.log 2>&1
rc1=$?
tail -3 gpurun_out/f32_tests.log
if [ $rc1 -ne 0 ] && [ $rc1 -ne 1 ]; then exit $rc1; fi
timeout -k 10 300 python -u tools/f32_gemm_sweep.py --json gpurun_out/r3_f32_sweep.json > gpurun_out/f32_sweep.log 2>&1 && \
timeout -k 10 300 python -u tools/f32_bench.py --json gpurun_out/r3_f32_bench.json > gpurun_out/f32_bench.log 2>&1
rc=$?
cat gpurun_out/f32_sweep.log | tail -15
grep attn gpurun_out/f32_bench.log
exit $rc
