#!/bin/bash
# Round 6: backward dQ v2 (buffer-load ring, unrolled over the ring) vs v1; forward v2 at ring depth 2.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py \
  -k "attention" > gpurun_out/r6_attn_dq2_tests.log 2>&1 || { tail -30 gpurun_out/r6_attn_dq2_tests.log; exit 1; }
tail -2 gpurun_out/r6_attn_dq2_tests.log
for shape in "16 1024 12 64" "64 1024 12 64"; do
  for v in old new old2 new2; do
    case $v in
      old|old2) env="MIPIPE_ATTN_FWD=1 MIPIPE_ATTN_BWD_DQ=1 MIPIPE_ATTN_BWD_DKDV=1" ;;
      new|new2) env="" ;;
    esac
    echo "$v $shape: $(env $env timeout -k 10 120 python tools/attn_time.py $shape)" | tee -a gpurun_out/r6_attn_dq2_time.txt || exit 1
  done
done
