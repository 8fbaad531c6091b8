#!/bin/bash
# A/B of the f32 GEMM knobs on the reference fp32 workload with 4 lanes (after the lane-aware split)
set -e
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/f32k
for rep in 1 2; do
for k in default MIPIPE_F32_SK=auto MIPIPE_F32_TILE=64 MIPIPE_F32_CUS=48; do
  echo "knob $k" >> gpurun_out/f32k/probe.txt
  if [ $k = default ]; then LANES=4 timeout -k 10 200 python -u tools/r5/lane_probe.py >> gpurun_out/f32k/probe.txt 2>&1
  else env $k LANES=4 timeout -k 10 200 python -u tools/r5/lane_probe.py >> gpurun_out/f32k/probe.txt 2>&1; fi
done
done
