#!/bin/bash
# stash ring + everything graph-related (native runner, multi-rank parity with graphs and
# lanes), gemm7 (forced), then the bench.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r5i
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_native_runner_gpu.py tests/test_multirank_gpu.py tests/test_kernels_gpu.py::test_gemm7_stream_k > gpurun_out/r5i/tests.log 2>&1
rc=$?; tail -6 gpurun_out/r5i/tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r5i/bench.log 2>&1
rc=$?; grep '^{' gpurun_out/r5i/bench.log | cut -c1-200; exit $rc
