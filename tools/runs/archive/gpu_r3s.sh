#!/bin/bash
# bench.py's N>1 launch at FULL size (GPT-2 small, mbs 32, m = 4N) with the ranks sharing one
# GPU over gloo: init / HIP-graph capture / tape / distributed head complete and the HBM of
# every rank fits (timings meaningless).  N = 8 at mbs 8 (eight full-size ranks would
# need ~400 GB on one device).
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export MIPIPE_DIST_BACKEND=gloo OMP_NUM_THREADS=2
timeout -k 10 400 python bench.py --gpus 2 --steps 2 --warmup 1 > gpurun_out/fs_bench2.log 2>&1 && \
timeout -k 10 500 python bench.py --gpus 4 --steps 2 --warmup 1 > gpurun_out/fs_bench4.log 2>&1 && \
timeout -k 10 500 python bench.py --gpus 8 --steps 1 --warmup 1 --mbs 8 > gpurun_out/fs_bench8.log 2>&1
rc=$?
for f in gpurun_out/fs_bench*.log; do echo "$f: $(grep '^{' $f | cut -c1-200)"; done
exit $rc
