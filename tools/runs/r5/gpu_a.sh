#!/bin/bash
# Round-5 baseline on a fresh box: the driver's bench command and the bf16 GEMM tail probe
# (planner vs hipBLASLt) at the pipeline microbatch token counts.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r5a
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r5a/bench.log 2>&1
rc=$?; grep '^{' gpurun_out/r5a/bench.log | cut -c1-400; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python tools/gemm_tail_probe.py --ms 8192,16384,32768 --cfgs -1 > gpurun_out/r5a/tail.txt 2>&1
rc=$?; cat gpurun_out/r5a/tail.txt; exit $rc
