#!/bin/bash
# gemm7 kernel time by chunk count (kernel trace): M=8192 (all-tail grids) with S = 1 / 2 / 3
# vs gemm3; then the stash-ring test.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r5g
for S in 1 2; do
  MIPIPE_GEMM7_S=$S timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5g/s$S -o run -- python3 tools/gemm_tail_probe.py --ms 8192 --cfgs=14 > gpurun_out/r5g/probe_s$S.txt 2>&1 || exit 1
  find gpurun_out/r5g/s$S -name "*kernel_trace.csv" -exec cp {} gpurun_out/r5g/trace_s$S.csv \;
  rm -rf gpurun_out/r5g/s$S
done
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5g/g3 -o run -- python3 tools/gemm_tail_probe.py --ms 8192 --cfgs=5 > gpurun_out/r5g/probe_g3.txt 2>&1 || exit 1
find gpurun_out/r5g/g3 -name "*kernel_trace.csv" -exec cp {} gpurun_out/r5g/trace_g3.csv \;
rm -rf gpurun_out/r5g/g3
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_native_runner_gpu.py -k stash > gpurun_out/r5g/tests_nr.log 2>&1
rc=$?; tail -5 gpurun_out/r5g/tests_nr.log; exit $rc
