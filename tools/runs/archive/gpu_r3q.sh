#!/bin/bash
# The reference's 54-run sweep (L {4,8,12} x H {4,8,12} x P {2,4} x {GPipe, 1F1B, Interleaved1F1B},
# batch 32 x 128, m = 4, fwd+bwd, fp32) through the reference-compatible API on ONE MI355X:
# the P ranks share the GPU and gloo stages the p2p through host memory, like the
# reference's gloo runs (a lower bound for P GPUs).  One sweep per layer count.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export MIPIPE_DIST_BACKEND=gloo OMP_NUM_THREADS=2
for L in "$@"; do
  timeout -k 10 560 python -u tools/ref_sweep.py --device cuda --engine native --precision fp32 --layers $L \
    --timeout 120 --out gpurun_out/ref_sweep_fp32_1gpu_L$L > gpurun_out/ref_sweep_L$L.log 2>&1 || exit 1
  grep -c "tok/s" gpurun_out/ref_sweep_L$L.log
done
