#!/bin/bash
# Code-path rehearsal of the BASELINE.json multi-GPU configs on ONE GPU (8 ranks share
# the device, gloo host-staged p2p; shortened sequences/batches so it fits and finishes).
# Completion + finite loss only; timings are meaningless.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export MIPIPE_DIST_BACKEND=gloo OMP_NUM_THREADS=1
timeout -k 10 400 python bench.py --gpus 8 --model gpt2-medium --schedule Interleaved1F1B --vstages 2 --mbs 2 --seq 512 --steps 1 --warmup 1 --schedules none --ref-fp32 0 > gpurun_out/cfg3.log 2>&1 && \
timeout -k 10 400 python bench.py --gpus 8 --model llama3-8b --recompute --mbs 1 --seq 1024 --steps 1 --warmup 1 --schedules none --ref-fp32 0 > gpurun_out/cfg4.log 2>&1 && \
timeout -k 10 400 python bench.py --gpus 8 --dp 2 --model llama3-1b --recompute --mbs 1 --seq 1024 --steps 1 --warmup 1 --schedules none --ref-fp32 0 > gpurun_out/cfg5.log 2>&1
