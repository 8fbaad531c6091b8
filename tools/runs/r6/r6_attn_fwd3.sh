#!/bin/bash
# Round 6: attention forward v2 with MFMA row sums + asm max chain; ring depth 3 (3 WG/CU)
# vs 2 (the fwdnb2 variant build, 4 WG/CU); correctness on the default build first.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py \
  -k "attention" > gpurun_out/r6_attn_fwd3_tests.log 2>&1 || { tail -30 gpurun_out/r6_attn_fwd3_tests.log; exit 1; }
tail -2 gpurun_out/r6_attn_fwd3_tests.log
MIPIPE_EXT_VARIANT=fwdnb2 timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py \
  -k "attention_fwd_bwd or cross_lengths" > gpurun_out/r6_attn_fwd3_tests_nb2.log 2>&1 || { tail -30 gpurun_out/r6_attn_fwd3_tests_nb2.log; exit 1; }
tail -2 gpurun_out/r6_attn_fwd3_tests_nb2.log
for shape in "16 1024 12 64" "64 1024 12 64"; do
  for v in v1 nb3 nb2 nb3b; do
    case $v in
      v1) env="MIPIPE_ATTN_FWD=1" ;;
      nb3|nb3b) env="" ;;
      nb2) env="MIPIPE_EXT_VARIANT=fwdnb2" ;;
    esac
    echo "$v $shape: $(env $env timeout -k 10 120 python tools/attn_time.py $shape)" | tee -a gpurun_out/r6_attn_fwd3_time.txt || exit 1
  done
done
