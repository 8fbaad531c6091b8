#!/bin/bash
# Round 6: the whole GPU test suite (as the driver runs it), then the dK/dV tile-edge A/B.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/r6_gpu_suite.log 2>&1
rc=$?
tail -15 gpurun_out/r6_gpu_suite.log
[ $rc -eq 0 ] || exit $rc
bash tools/runs/r6/r6_attn_dkdv_tedge.sh
