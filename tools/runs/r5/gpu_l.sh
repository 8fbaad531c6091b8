#!/bin/bash
# Engine progress report test + engine tests.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r5l
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_kernels_gpu.py -k "rccl" > gpurun_out/r5l/tests.log 2>&1
rc=$?; tail -6 gpurun_out/r5l/tests.log; exit $rc
