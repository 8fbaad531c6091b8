#!/bin/bash
# gemm7 v3 (gemm3 lead rounds + LDS-staged split tail, self-clearing tags): numerics, probe
# (eager + graph), then the stash-ring / native-runner tests, then the bench.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r5f
timeout -k 10 300 python -u -m pytest -x -v --timeout 150 --timeout-method thread -m gpu tests/test_kernels_gpu.py -k "gemm7 or gemm2_configs or fused_colsum or dropout_epilogues" > gpurun_out/r5f/tests.log 2>&1
rc=$?; tail -4 gpurun_out/r5f/tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python tools/gemm_tail_probe.py --ms 8192,32768 --cfgs=-1,5 > gpurun_out/r5f/tail.txt 2>&1
rc=$?; cat gpurun_out/r5f/tail.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python tools/gemm_tail_probe.py --ms 8192,32768 --cfgs=-1,5 --graph > gpurun_out/r5f/tail_graph.txt 2>&1
rc=$?; cat gpurun_out/r5f/tail_graph.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_native_runner_gpu.py > gpurun_out/r5f/tests_nr.log 2>&1
rc=$?; tail -5 gpurun_out/r5f/tests_nr.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r5f/bench.log 2>&1
rc=$?; grep '^{' gpurun_out/r5f/bench.log | cut -c1-200; exit $rc
