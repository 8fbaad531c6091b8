#!/bin/bash
# Round-5 fixes on the GPU: capture failure, two-thread RCCL engines, replayed-step
# reductions, f32 class-swap linears; then the driver's bench command.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r5b
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu \
  "tests/test_native_runner_gpu.py::test_capture_failure_reraises_the_original_error_and_capture_recovers" \
  "tests/test_kernels_gpu.py::test_native_rccl_engines_interleaved_from_two_threads" \
  "tests/test_kernels_gpu.py::test_native_rccl_engine_self_transfer" \
  "tests/test_reference_parity.py::test_f32_kernel_stage_matches_aten" \
  tests/test_multirank_gpu.py::test_multirank_gpu_replayed_steps_reduce_once > gpurun_out/r5b/tests.log 2>&1
rc=$?; tail -12 gpurun_out/r5b/tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r5b/bench.log 2>&1
rc=$?; grep '^{' gpurun_out/r5b/bench.log | cut -c1-300; exit $rc
