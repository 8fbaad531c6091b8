#!/bin/bash
# Round 6: forward v3 (tile software pipeline: K Q^T of tile t+1 beside tile t's softmax / P V)
# vs forward v2; v3 at 3 waves per SIMD (default build, 5 VGPRs spilled) and at 2 (f3w2 build).
set -o pipefail
mkdir -p gpurun_out
MIPIPE_ATTN_FWD=3 timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py \
  -k "attention" > gpurun_out/r6_attn_fwd3pipe_tests.log 2>&1 || { tail -30 gpurun_out/r6_attn_fwd3pipe_tests.log; exit 1; }
tail -2 gpurun_out/r6_attn_fwd3pipe_tests.log
for shape in "16 1024 12 64" "64 1024 12 64"; do
  for v in v2 v3 v3w2 v2b v3b v3w2b; do
    case $v in
      v2|v2b) env="MIPIPE_ATTN_FWD=2" ;;
      v3|v3b) env="MIPIPE_ATTN_FWD=3" ;;
      v3w2|v3w2b) env="MIPIPE_ATTN_FWD=3 MIPIPE_EXT_VARIANT=f3w2" ;;
    esac
    echo "$v $shape: $(env $env timeout -k 10 120 python tools/attn_time.py $shape)" | tee -a gpurun_out/r6_attn_fwd3pipe_time.txt || exit 1
  done
done
