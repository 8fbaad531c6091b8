#!/bin/bash
# bench.py at N=1: microbatch size 16 vs 32 sequences (interleaved pairs)
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
: > gpurun_out/bench_mbs_ab.txt
for mb in 16 32 16 32; do
  timeout -k 10 300 python -u bench.py --mbs $mb > gpurun_out/bench_mbs$mb.log 2>&1 || exit 1
  echo "mbs=$mb $(tail -1 gpurun_out/bench_mbs$mb.log | cut -c150-400)" >> gpurun_out/bench_mbs_ab.txt
done
cat gpurun_out/bench_mbs_ab.txt
