#!/bin/bash
# gemm7 hand-off by plain stores + release fence (default) vs the sc1 build (variant): all-tail
# grids at M=8192, S = 2, kernel trace; then the stash-ring test.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r5h
MIPIPE_GEMM7_S=2 timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r5h/p -o run -- python3 tools/gemm_tail_probe.py --ms 8192 --cfgs=14,5 > gpurun_out/r5h/probe.txt 2>&1 || exit 1
find gpurun_out/r5h/p -name "*kernel_trace.csv" -exec cp {} gpurun_out/r5h/trace.csv \;
rm -rf gpurun_out/r5h/p; grep M= gpurun_out/r5h/probe.txt
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_native_runner_gpu.py -k stash tests/test_kernels_gpu.py::test_gemm7_stream_k > gpurun_out/r5h/tests.log 2>&1
rc=$?; tail -5 gpurun_out/r5h/tests.log; exit $rc
