#!/bin/bash
# headline config alternatives on one GPU: microbatch size x count (global batch 128)
set -e
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/mbs
for rep in 1 2; do
for cfg in "" "--mbs 32 --microbatches 4" "--mbs 128 --microbatches 1"; do
  tag=$(echo "x$cfg" | tr -d ' -')
  timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-bubble --schedules none --ref-fp32 0 $cfg > gpurun_out/mbs/b_${tag}_${rep}.json 2> gpurun_out/mbs/b_${tag}_${rep}.err || echo "fail $tag" >> gpurun_out/mbs/summary.txt
  echo "cfg [$cfg] rep $rep $(python -c "import json;d=json.loads(open('gpurun_out/mbs/b_${tag}_${rep}.json').read().splitlines()[-1]);print(d['value'], d['config']['microbatch_lanes'])")" >> gpurun_out/mbs/summary.txt
done
done
