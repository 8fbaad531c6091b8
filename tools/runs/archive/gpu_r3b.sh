#!/bin/bash
# f32 path: kernel tests, f32 microbench, then the kernel test file (bf16 path unchanged).
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest tests/test_f32_gpu.py -v --timeout 120 --timeout-method thread > gpurun_out/f32_tests.log 2>&1
rc1=$?
echo "f32 tests rc=$rc1"
if [ $rc1 -ne 0 ] && [ $rc1 -ne 1 ]; then exit $rc1; fi
timeout -k 10 300 python -u tools/f32_bench.py --json gpurun_out/r3_f32_bench.json > gpurun_out/f32_bench.log 2>&1 && \
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/kernels_gpu.log 2>&1
rc=$?
tail -3 gpurun_out/f32_tests.log; tail -2 gpurun_out/kernels_gpu.log
exit $rc
