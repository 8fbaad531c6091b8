#!/bin/bash
# Round 6: the whole GPU test suite (as the driver runs it).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1150 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/r6_gpu_suite.log 2>&1
rc=$?
tail -15 gpurun_out/r6_gpu_suite.log
exit $rc
