#!/bin/bash
# Kernel stats + timeline of the reference model L8H8 bf16 trainer step (1 GPU, 4 lanes).
set -o pipefail
mkdir -p gpurun_out/prof_refbf16
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_refbf16 -o run -- \
  python3 bench.py --model reference --mbs 8 --seq 128 --microbatches 4 --steps 3 --warmup 2 --no-bubble > gpurun_out/prof_refbf16/bench.log 2>&1 || exit 1
find gpurun_out/prof_refbf16 -name "*kernel_stats.csv" -exec cp {} gpurun_out/prof_refbf16/kernel_stats.csv \;
find gpurun_out/prof_refbf16 -name "*kernel_trace.csv" -size -60M -exec cp {} gpurun_out/prof_refbf16/kernel_trace.csv \;
python3 tools/timeline_stats.py gpurun_out/prof_refbf16/kernel_trace.csv --steps 1 --top 15 > gpurun_out/prof_refbf16/timeline.json
