#!/bin/bash
# Learning check with the round-3 code: GPT-2 small on the learnable pattern stream, 1 GPU,
# 2 microbatches of 64 sequences (the bench default), 200 steps.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u train.py --config configs/gpt2_small_1f1b_pp4.yaml parallel.pp=1 parallel.microbatches=2 \
  train.micro_batch=64 train.data=pattern train.steps=200 > gpurun_out/learn.log 2>&1
rc=$?; grep -E "step +(20|60|100|140|180|200) " gpurun_out/learn.log; tail -3 gpurun_out/learn.log; exit $rc
