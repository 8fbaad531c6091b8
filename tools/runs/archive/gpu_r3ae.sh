#!/bin/bash
# Kernel stats + timeline of the default 1-GPU bench (2 x 64-sequence microbatches).
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash tools/prof.sh gpt2s_mbs64 && python3 tools/timeline_stats.py gpurun_out/prof_gpt2s_mbs64/kernel_trace.csv --steps 1 --top 15 > gpurun_out/prof_gpt2s_mbs64/timeline.json
