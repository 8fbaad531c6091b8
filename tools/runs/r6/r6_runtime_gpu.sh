#!/bin/bash
# Round 6: the native runtime after the ASan fixes (RCCL group peer check, runner event
# destructor, atomic open flag): engine, tape runner and multi-rank tests on the GPU.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_kernels_gpu.py -k "rccl or queue" > gpurun_out/r6_runtime_gpu_engine.log 2>&1 &&
timeout -k 10 900 python -u -m pytest -x -v --timeout 240 --timeout-method thread \
  tests/test_native_runner_gpu.py tests/test_multirank_gpu.py > gpurun_out/r6_runtime_gpu.log 2>&1
rc=$?
tail -3 gpurun_out/r6_runtime_gpu_engine.log gpurun_out/r6_runtime_gpu.log
exit $rc
