#!/bin/bash
set -e
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/lanes
timeout -k 10 300 python -u tools/r5/lane_probe.py > gpurun_out/lanes/probe.txt 2>&1
