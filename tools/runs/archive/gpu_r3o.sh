#!/bin/bash
# One-launch short attention backward: kernel tests, A/B at the reference shape
# (MIPIPE_ATTN_BWD_SHORT=0: the two-kernel path), L8H8 bf16 trainer A/B.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "attn or attention" > gpurun_out/attn_tests.log 2>&1
rc=$?; tail -2 gpurun_out/attn_tests.log; [ $rc -ne 0 ] && exit $rc
: > gpurun_out/attn_short_ab.txt
for ab in 1 0 1 0; do
  MIPIPE_ATTN_BWD_SHORT=$ab timeout -k 10 120 python -u tools/bench_kernels.py --only attn_B8S128 > gpurun_out/attn_short_$ab.log 2>&1 || exit 1
  echo "short=$ab $(grep attn_B8S128 gpurun_out/attn_short_$ab.log)" >> gpurun_out/attn_short_ab.txt
done
for ab in 1 0 1 0; do
  MIPIPE_ATTN_BWD_SHORT=$ab timeout -k 10 200 python -u tools/ref_table_gpu.py --engine trainer --precision bf16 --only 8x8 > gpurun_out/attn_short_tr_$ab.log 2>&1 || exit 1
  echo "L8H8 bf16 trainer short=$ab $(grep tokens_per_s gpurun_out/attn_short_tr_$ab.log | cut -c1-110)" >> gpurun_out/attn_short_ab.txt
done
cat gpurun_out/attn_short_ab.txt
