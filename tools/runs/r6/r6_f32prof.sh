#!/bin/bash
# Round 6: kernel-time profile of the reference-precision step (fp32 L8 H8, 32 x 128, m = 4, P = 1).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/f32prof6
timeout -k 10 400 python -u bench.py --phase ref --ref-p 1 --no-supervise --steps 20 --warmup 5 --no-bubble > gpurun_out/f32prof6/plain.log 2>&1 || { tail -20 gpurun_out/f32prof6/plain.log; exit 1; }
tail -3 gpurun_out/f32prof6/plain.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/f32prof6/trace -o run -- python3 -u bench.py --phase ref --ref-p 1 --no-supervise --steps 20 --warmup 5 --no-bubble > gpurun_out/f32prof6/prof.log 2>&1 || { tail -20 gpurun_out/f32prof6/prof.log; exit 1; }
find gpurun_out/f32prof6/trace -name "*kernel_stats.csv" -exec cp {} gpurun_out/f32prof6/kernel_stats.csv \;
rm -rf gpurun_out/f32prof6/trace
head -30 gpurun_out/f32prof6/kernel_stats.csv | cut -c1-150
