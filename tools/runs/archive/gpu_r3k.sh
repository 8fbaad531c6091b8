#!/bin/bash
# bf16 key-split short-sequence attention forward (LDS-DMA staging): tests, kernel A/B,
# reference-model step A/B
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_native_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/attn_tests2.log 2>&1
rc=$?; tail -2 gpurun_out/attn_tests2.log; [ $rc -ne 0 ] && exit $rc
: > gpurun_out/attn_ks2_ab2.txt
for ab in 1 0 1 0; do
  MIPIPE_ATTN_KS2=$ab timeout -k 10 120 python -u tools/bench_kernels.py --only attn_B8S128 > gpurun_out/attn_ks2b_$ab.log 2>&1 || exit 1
  echo "ks2=$ab $(grep attn_B8S128 gpurun_out/attn_ks2b_$ab.log)" >> gpurun_out/attn_ks2_ab2.txt
done
for ab in 1 0 1 0; do
  MIPIPE_ATTN_KS2=$ab timeout -k 10 200 python -u tools/ref_table_gpu.py --engine trainer --only 8x8 > gpurun_out/l8h8_ks2_$ab.log 2>&1 || exit 1
  echo "L8H8 bf16 trainer ks2=$ab $(grep tokens_per_s gpurun_out/l8h8_ks2_$ab.log | cut -c1-90)" >> gpurun_out/attn_ks2_ab2.txt
done
cat gpurun_out/attn_ks2_ab2.txt
