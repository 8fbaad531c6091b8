#!/bin/bash
# gemm7 (stream-K) correctness, then the tail probe (planner = gemm7 where it applies, vs
# the forced ping-pong engine and hipBLASLt), then the bench.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r5c
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_kernels_gpu.py -k "gemm7 or gemm2_configs" > gpurun_out/r5c/tests.log 2>&1
rc=$?; tail -5 gpurun_out/r5c/tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python tools/gemm_tail_probe.py --ms 8192,16384,32768 --cfgs=-1,5 > gpurun_out/r5c/tail.txt 2>&1
rc=$?; cat gpurun_out/r5c/tail.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python tools/gemm_tail_probe.py --ms 8192,32768 --cfgs=-1,5 --graph > gpurun_out/r5c/tail_graph.txt 2>&1
rc=$?; cat gpurun_out/r5c/tail_graph.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r5c/bench.log 2>&1
rc=$?; grep '^{' gpurun_out/r5c/bench.log | cut -c1-200; exit $rc
