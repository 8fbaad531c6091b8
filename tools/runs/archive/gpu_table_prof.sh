#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u tools/ref_table_gpu.py --json gpurun_out/ref_table_lanes.json > gpurun_out/ref_table_lanes.log 2>&1 && \
bash tools/prof.sh gpt2lanes && \
bash tools/prof.sh reflanes --model reference --mbs 8 --seq 128 --microbatches 4
