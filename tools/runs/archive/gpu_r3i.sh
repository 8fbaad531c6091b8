#!/bin/bash
# bench.py at N=1: 2 vs 4 microbatches per step (weak-scaling m = 2P vs 4P), interleaved
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
: > gpurun_out/bench_m_ab.txt
for mm in 2 4 2 4; do
  timeout -k 10 300 python -u bench.py --microbatches $mm > gpurun_out/bench_m$mm.log 2>&1 || exit 1
  echo "m=$mm $(tail -1 gpurun_out/bench_m$mm.log | cut -c1-260)" >> gpurun_out/bench_m_ab.txt
done
cat gpurun_out/bench_m_ab.txt
