#!/bin/bash
# Round 6: norm backward workgroup cap (2 / 4 / 8 per CU) at 16K and 64K rows, then the step.
set -o pipefail
mkdir -p gpurun_out
for T in 16384 65536; do
  for nb in 512 1024 2048 512; do
    echo "T=$T blocks=$nb: $(NORM_PROBE_T=$T MIPIPE_NORM_BWD_BLOCKS=$nb timeout -k 10 120 python tools/norm_probe.py 2>/dev/null | grep 'norm_bwd layernorm' | tr '\n' ' ')" | tee -a gpurun_out/r6_norm_blocks.txt || exit 1
  done
done
