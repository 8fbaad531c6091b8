#!/bin/bash
# Full GPU suite, the 1-GPU bench, the fp32 reference step under rocprof, f32 PMC passes.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_suite.log 2>&1
rc=$?
tail -3 gpurun_out/gpu_suite.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py > gpurun_out/bench_1gpu.log 2>&1 || exit 1
tail -1 gpurun_out/bench_1gpu.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_ref2 -o run -- python3 tools/ref_table_gpu.py --engine native --precision fp32 --only 8x8 --iters 5 --warmup 2 > gpurun_out/ref_prof2.log 2>&1 || exit 1
grep tokens_per_s gpurun_out/ref_prof2.log | cut -c1-160
bash tools/f32_pmc.sh || exit 1
echo done
