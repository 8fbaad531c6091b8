#!/bin/bash
set -e
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/bend
timeout -k 10 700 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bend/bench.json 2> gpurun_out/bend/bench.err
