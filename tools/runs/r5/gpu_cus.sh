#!/bin/bash
# A/B: f32 split-K CU count with 4 concurrent lanes (reference fp32 workload): the runtime's
# lane-aware default (256/4 = 64) vs the old 256 and a no-split-leaning 32
set -e
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/cus2
for rep in 1 2; do
for c in default 256 32; do
  echo "cus $c" >> gpurun_out/cus2/probe.txt
  if [ $c = default ]; then LANES=4 timeout -k 10 200 python -u tools/r5/lane_probe.py >> gpurun_out/cus2/probe.txt 2>&1
  else MIPIPE_F32_CUS=$c LANES=4 timeout -k 10 200 python -u tools/r5/lane_probe.py >> gpurun_out/cus2/probe.txt 2>&1; fi
done
done
timeout -k 10 300 python -u bench.py --phase ref --ref-p 1 --no-supervise --steps 20 --warmup 5 --no-bubble > gpurun_out/cus2/ref.json 2>&1
