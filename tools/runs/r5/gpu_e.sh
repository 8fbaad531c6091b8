#!/bin/bash
# gemm7 diagnosis: kernel trace of the split-tail engine at M=8192 N=768 K=768 with S = 2
# (planner) and S = 1 (no hand-off: a persistent data-parallel grid), vs gemm3; then the
# native-runner tests (stash ring) that the last call's -k filter left out.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r5e
for S in 2 1; do
  MIPIPE_GEMM7_S=$S timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5e/s$S -o run -- python3 tools/gemm_tail_probe.py --ms 8192 --cfgs=14,5 > gpurun_out/r5e/probe_s$S.txt 2>&1 || exit 1
  cat gpurun_out/r5e/probe_s$S.txt | grep "M=8192 N=768 K=768"
  find gpurun_out/r5e/s$S -name "*kernel_stats.csv" -exec cp {} gpurun_out/r5e/stats_s$S.csv \;
  rm -rf gpurun_out/r5e/s$S
done
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_native_runner_gpu.py > gpurun_out/r5e/tests.log 2>&1
rc=$?; tail -12 gpurun_out/r5e/tests.log; exit $rc
