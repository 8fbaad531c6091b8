#!/bin/bash
# Single-lane (the PP>1 execution mode: one compute stream + dW side stream) efficiency vs
# microbatch size at 128 sequences per step: mbs 16 / 32 / 64 (m = 8 / 4 / 2), MIPIPE_LANES=1.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
: > gpurun_out/lane1_mbs_ab.txt
for cfg in "16 8" "32 4" "64 2" "16 8" "32 4" "64 2"; do
  set -- $cfg
  MIPIPE_LANES=1 timeout -k 10 300 python -u bench.py --steps 8 --warmup 3 --mbs $1 --microbatches $2 > gpurun_out/l1_$1_$2.log 2>&1 || exit 1
  echo "lanes=1 mbs=$1 m=$2 $(tail -1 gpurun_out/l1_$1_$2.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["config"]["microbatch_lanes"])')" >> gpurun_out/lane1_mbs_ab.txt
done
cat gpurun_out/lane1_mbs_ab.txt
