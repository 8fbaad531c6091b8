#!/bin/bash
set -e
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/f32t
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_f32_gpu.py -k "lane_aware or layouts or reference_block" > gpurun_out/f32t/log.txt 2>&1
