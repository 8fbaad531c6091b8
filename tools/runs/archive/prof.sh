#!/bin/bash
# rocprofv3 kernel trace + stats of a short bench run; summaries land in gpurun_out/prof_<tag>
set -o pipefail
TAG=${1:-bench}; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/prof_$TAG
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- \
  python3 bench.py --steps 3 --warmup 2 --no-bubble "$@" > gpurun_out/prof_$TAG/bench.log 2>&1
rc=$?
find gpurun_out/prof_$TAG -name "*kernel_stats.csv" -exec cp {} gpurun_out/prof_$TAG/kernel_stats.csv \; 2>/dev/null
find gpurun_out/prof_$TAG -name "*kernel_trace.csv" -size -60M -exec cp {} gpurun_out/prof_$TAG/kernel_trace.csv \; 2>/dev/null
exit $rc
