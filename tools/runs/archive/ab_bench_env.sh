#!/bin/bash
# bench.py A/B of one environment toggle on the same box, alternating runs:  ab_bench_env.sh VAR
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
VAR=$1
for i in 1 2; do
  for v in 0 1; do
    env $VAR=$v timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-bubble > gpurun_out/ab.log 2>&1 || exit 1
    echo "$VAR=$v $(tail -1 gpurun_out/ab.log | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
