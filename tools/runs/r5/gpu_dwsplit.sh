#!/bin/bash
# A/B: cap on the dW (TT, f32-accumulate) split-K factor on the headline step (2 lanes)
set -e
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/dws
for rep in 1 2; do
for c in 32 16 8; do
  MIPIPE_DW_MAXSPLIT=$c timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-bubble --schedules none --ref-fp32 0 > gpurun_out/dws/b_${c}_${rep}.json 2> gpurun_out/dws/b_${c}_${rep}.err
  echo "cap $c rep $rep $(python -c "import json,sys;d=json.loads(open('gpurun_out/dws/b_${c}_${rep}.json').read().splitlines()[-1]);print(d['value'])")" >> gpurun_out/dws/summary.txt
done
done
