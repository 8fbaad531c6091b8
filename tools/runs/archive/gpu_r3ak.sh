#!/bin/bash
# norm backward rows per workgroup (MIPIPE_NORM_BWD_RPB) on the reference model L8H8 bf16
# trainer (1024-token microbatches): 8 (default) vs 16 / 32 / 4, interleaved.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
: > gpurun_out/rpb_ab.txt
for r in 8 16 32 4 8 16 32 4; do
  MIPIPE_NORM_BWD_RPB=$r timeout -k 10 200 python -u tools/ref_table_gpu.py --engine trainer --precision bf16 --only 8x8 > gpurun_out/rpb.log 2>&1 || exit 1
  echo "rpb=$r $(grep tokens_per_s gpurun_out/rpb.log | cut -c1-90)" >> gpurun_out/rpb_ab.txt
done
cat gpurun_out/rpb_ab.txt
