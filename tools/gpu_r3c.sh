#!/bin/bash
# f32 GEMM split sweep + per-kernel times.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u tools/f32_gemm_sweep.py --json gpurun_out/r3_f32_sweep.json > gpurun_out/f32_sweep.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_f32 -o run -- python3 tools/f32_bench.py > gpurun_out/f32_prof.log 2>&1
rc=$?
cat gpurun_out/f32_sweep.log | tail -16
exit $rc
