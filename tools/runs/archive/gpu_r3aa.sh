#!/bin/bash
# bench.py N=1: microbatch size / count at 128 sequences per step: (mbs 32, m 4) default vs
# (mbs 64, m 2); interleaved.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
: > gpurun_out/mbs64_ab.txt
for cfg in "32 4" "64 2" "32 4" "64 2"; do
  set -- $cfg
  timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --mbs $1 --microbatches $2 > gpurun_out/mbs64_$1_$2.log 2>&1 || exit 1
  echo "mbs=$1 m=$2 $(tail -1 gpurun_out/mbs64_$1_$2.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["config"]["microbatch_lanes"], d["hbm_peak_gb_per_gpu"])')" >> gpurun_out/mbs64_ab.txt
done
cat gpurun_out/mbs64_ab.txt
