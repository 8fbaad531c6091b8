#!/bin/bash
# A/B: norm backward rows per workgroup on the reference fp32 workload (4 lanes)
set -e
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/rpb
for rep in 1 2; do
for k in 8 4 16; do
  echo "rpb $k" >> gpurun_out/rpb/probe.txt
  MIPIPE_NORM_BWD_RPB=$k LANES=4 timeout -k 10 200 python -u tools/r5/lane_probe.py >> gpurun_out/rpb/probe.txt 2>&1
done
done
