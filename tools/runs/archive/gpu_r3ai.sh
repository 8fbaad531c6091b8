#!/bin/bash
# short attention backward: delta from global rows (A/B build _C_sdr.so, -D MP_SHORT_DELTA_REGS=1)
# vs the O tile in LDS: kernel tests on the variant, microbench (interleaved), L8H8 trainer.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
MIPIPE_EXT_VARIANT=sdr timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "attn or attention" > gpurun_out/sdr_tests.log 2>&1
rc=$?; tail -2 gpurun_out/sdr_tests.log; [ $rc -ne 0 ] && exit $rc
: > gpurun_out/sdr_ab.txt
for v in "" sdr "" sdr; do
  MIPIPE_EXT_VARIANT=$v timeout -k 10 120 python -u tools/bench_kernels.py --only attn_B8S128 > gpurun_out/sdr_bk.log 2>&1 || exit 1
  echo "${v:-default} $(grep attn_B8S128 gpurun_out/sdr_bk.log)" >> gpurun_out/sdr_ab.txt
done
for v in "" sdr "" sdr; do
  MIPIPE_EXT_VARIANT=$v timeout -k 10 200 python -u tools/ref_table_gpu.py --engine trainer --precision bf16 --only 8x8 > gpurun_out/sdr_tr.log 2>&1 || exit 1
  echo "L8H8 trainer ${v:-default} $(grep tokens_per_s gpurun_out/sdr_tr.log | cut -c1-90)" >> gpurun_out/sdr_ab.txt
done
cat gpurun_out/sdr_ab.txt
