#!/bin/bash
# GELU derivative saved by the forward epilogue: kernels + native model tests, probe, bench.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r5v
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_kernels_gpu.py tests/test_native_gpu.py tests/test_learning.py > gpurun_out/r5v/tests.log 2>&1
rc=$?; tail -2 gpurun_out/r5v/tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python tools/gemm_epi_probe.py --graph > gpurun_out/r5v/epi_graph.txt 2>&1
rc=$?; grep -v "^{\|amdgpu" gpurun_out/r5v/epi_graph.txt; [ $rc -ne 0 ] && exit $rc
for i in 1 2; do
timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 --schedules none --ref-fp32 0 > gpurun_out/r5v/bench_$i.log 2>&1 || exit 1
grep '^{' gpurun_out/r5v/bench_$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["last_loss"])'
done
