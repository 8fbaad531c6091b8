#!/bin/bash
# box-speed check: GPT-2 bench (N=1) next to the fp32 L8H8 reference-table row
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/y_bench.log 2>&1 && \
timeout -k 10 200 python -u tools/ref_table_gpu.py --engine native --precision fp32 --only 8x8,4x4 > gpurun_out/y_fp32.log 2>&1 && \
timeout -k 10 200 python -u tools/ref_table_gpu.py --engine trainer --fwd-bwd --precision fp32 --only 8x8,4x4 > gpurun_out/y_fp32_tr.log 2>&1
rc=$?
tail -1 gpurun_out/y_bench.log | cut -c150-260; grep -h tokens_per_s gpurun_out/y_fp32.log gpurun_out/y_fp32_tr.log | cut -c1-100
exit $rc
