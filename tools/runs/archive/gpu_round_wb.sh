#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 120 python -u tools/wbatch_probe.py > gpurun_out/wbatch_probe.txt 2>&1 && \
bash tools/gpu_round.sh
