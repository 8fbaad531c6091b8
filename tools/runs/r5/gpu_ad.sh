#!/bin/bash
# train.py CLI on the GPU: 2 ranks sharing one GPU (gloo), PP=2 GPT-2 small, HIP graphs +
# stash ring + comm audit, checkpoint at step 4, resume to step 6.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r5ad
export MIPIPE_DIST_BACKEND=gloo OMP_NUM_THREADS=2
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29811 train.py --config configs/gpt2_small_1f1b_pp4.yaml parallel.pp=2 train.steps=4 train.micro_batch=4 train.seq_len=512 train.ckpt_dir=/tmp/ck train.ckpt_every=4 > gpurun_out/r5ad/run1.log 2>&1
rc=$?; tail -4 gpurun_out/r5ad/run1.log; [ $rc -ne 0 ] && exit $rc
ls /tmp/ck
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29812 train.py --config configs/gpt2_small_1f1b_pp4.yaml parallel.pp=2 train.steps=6 train.micro_batch=4 train.seq_len=512 train.resume=/tmp/ck/step0000004 > gpurun_out/r5ad/run2.log 2>&1
rc=$?; tail -4 gpurun_out/r5ad/run2.log; exit $rc
