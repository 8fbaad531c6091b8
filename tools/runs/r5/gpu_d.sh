#!/bin/bash
# gemm7 (split-tail) numerics + probes (eager and graph-replayed), the stash ring test,
# native runner / multirank regressions, then the bench.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r5d
timeout -k 10 400 python -u -m pytest -x -v --timeout 150 --timeout-method thread -m gpu tests/test_kernels_gpu.py -k "gemm7 or gemm2_configs or fused_colsum" tests/test_native_runner_gpu.py > gpurun_out/r5d/tests.log 2>&1
rc=$?; tail -8 gpurun_out/r5d/tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python tools/gemm_tail_probe.py --ms 8192,16384,32768 --cfgs=-1,5 > gpurun_out/r5d/tail.txt 2>&1
rc=$?; cat gpurun_out/r5d/tail.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python tools/gemm_tail_probe.py --ms 8192,32768 --cfgs=-1,5 --graph > gpurun_out/r5d/tail_graph.txt 2>&1
rc=$?; cat gpurun_out/r5d/tail_graph.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r5d/bench.log 2>&1
rc=$?; grep '^{' gpurun_out/r5d/bench.log | cut -c1-200; exit $rc
