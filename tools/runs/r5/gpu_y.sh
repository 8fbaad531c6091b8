#!/bin/bash
# Probe: staggered first-wave start of gemm3 (epilogue HBM bursts spread in time).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r5y
for s in 0 60 120 240 0; do
  MIPIPE_G3_STAGGER=$s timeout -k 10 200 python tools/gemm_epi_probe.py --graph > gpurun_out/r5y/epi_$s.txt 2>&1 || exit 1
  echo "== stagger $s"; grep -v "^{\|amdgpu" gpurun_out/r5y/epi_$s.txt | grep -E "fc1 plain|bias\+gelu|dGELU dX \(no|dX plain|fc2 bias\+res"
done
