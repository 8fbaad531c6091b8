#!/bin/bash
# train.py on one GPU with HIP graphs + native runner: 30 steps with checkpoints, then a
# resume from step 20; the resumed run must reproduce steps 21-30.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
rm -rf gpurun_out/ck
C="--config configs/gpt2_small_1f1b_pp4.yaml parallel.pp=1 parallel.microbatches=2 train.micro_batch=8 train.seq_len=512 train.log_every=5 train.steps=30"
timeout -k 10 300 python train.py $C train.ckpt_dir=gpurun_out/ck train.ckpt_every=10 > gpurun_out/train_a.log 2>&1 && \
timeout -k 10 300 python train.py $C train.resume=gpurun_out/ck/step0000020 > gpurun_out/train_b.log 2>&1
rc=$?
rm -rf gpurun_out/ck
exit $rc
