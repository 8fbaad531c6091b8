#!/bin/bash
# attention kernels timed eagerly and replayed from a HIP graph (short-sequence shapes are
# launch-bound when timed eagerly); short path on / off
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
: > gpurun_out/attn_graph.txt
for ab in 1 0; do
  MIPIPE_ATTN_BWD_SHORT=$ab timeout -k 10 200 python -u tools/bench_kernels.py --only attn > gpurun_out/attn_graph_$ab.log 2>&1 || exit 1
  sed "s/^/short=$ab /" gpurun_out/attn_graph_$ab.log | grep attn_ >> gpurun_out/attn_graph.txt
done
cat gpurun_out/attn_graph.txt
