#!/bin/bash
# Same-box A/B: this tree (GELU derivative saved) vs _ab/old (the previous commit), interleaved.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r5w
for i in 1 2 3; do
  timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 --schedules none --ref-fp32 0 > gpurun_out/r5w/new_$i.log 2>&1 || exit 1
  (cd _ab/old && timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 --schedules none --ref-fp32 0) > gpurun_out/r5w/old_$i.log 2>&1 || exit 1
  for v in new old; do echo "$v $i $(grep '^{' gpurun_out/r5w/${v}_$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["last_loss"])')"; done
done
