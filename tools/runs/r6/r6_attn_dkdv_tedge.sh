#!/bin/bash
# Round 6: dQ v2 with the two 32-key halves processed one after the other (166 VGPRs, 3 waves
# per SIMD; the _C_dqh variant build, -D MP_DQ2_HALVES=1) vs both halves at once (195, 2 waves).
set -o pipefail
mkdir -p gpurun_out
MIPIPE_EXT_VARIANT=dqh timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py \
  -k "attention" > gpurun_out/r6_attn_dqh_tests.log 2>&1 || { tail -30 gpurun_out/r6_attn_dqh_tests.log; exit 1; }
tail -2 gpurun_out/r6_attn_dqh_tests.log
for shape in "16 1024 12 64" "64 1024 12 64"; do
  for v in cur dqh cur2 dqh2; do
    case $v in
      dqh|dqh2) env="MIPIPE_EXT_VARIANT=dqh" ;;
      cur|cur2) env="MIPIPE_ATTN_FWD=2" ;;
    esac
    echo "$v $shape: $(env $env timeout -k 10 120 python tools/attn_time.py $shape)" | tee -a gpurun_out/r6_attn_dqh_time.txt || exit 1
  done
done
