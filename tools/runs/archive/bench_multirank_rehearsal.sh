#!/bin/bash
# bench.py's multi-rank path (torch.distributed.run self-launch, barrier + max-over-ranks
# timing, bubble reduction, rank-0 JSON) on ONE GPU: ranks share the device and gloo
# carries the p2p through host memory.  Timings are meaningless here; the point is that
# the N>1 code path the driver runs on the 8-GPU node completes and prints its line.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export MIPIPE_DIST_BACKEND=gloo OMP_NUM_THREADS=2
timeout -k 10 300 python bench.py --gpus 2 --steps 2 --warmup 1 --mbs 4 > gpurun_out/mr_bench2.log 2>&1 && \
timeout -k 10 300 python bench.py --gpus 4 --steps 2 --warmup 1 --mbs 4 --graphs 1 > gpurun_out/mr_bench4.log 2>&1 && \
timeout -k 10 300 python bench.py --gpus 4 --dp 2 --steps 2 --warmup 1 --mbs 4 > gpurun_out/mr_bench4dp.log 2>&1 && \
timeout -k 10 300 python bench.py --gpus 2 --steps 2 --warmup 1 --mbs 4 --schedule GPipe > gpurun_out/mr_bench2g.log 2>&1
