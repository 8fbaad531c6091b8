#!/bin/bash
# Round 6: forward v2 dropout normaliser fix (sum P before the mask) -- attention tests incl.
# the new causal / large-grid dropout cases, then the whole GPU suite.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py \
  -k "attention" > gpurun_out/r6_dropfix_tests.log 2>&1 || { tail -40 gpurun_out/r6_dropfix_tests.log; exit 1; }
grep -c PASSED gpurun_out/r6_dropfix_tests.log; tail -2 gpurun_out/r6_dropfix_tests.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/r6_dropfix_suite.log 2>&1 || { tail -30 gpurun_out/r6_dropfix_suite.log; exit 1; }
tail -2 gpurun_out/r6_dropfix_suite.log
