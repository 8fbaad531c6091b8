#!/bin/bash
# norm backward column partials + reduce for small grids (A/B build _C_ncp.so,
# -D MP_NORM_COLPART_MIN=32) vs per-column atomics below 256 workgroups (default):
# norm tests on the variant, reference model L8H8 bf16 trainer (1024-token rows), GPT-2 bench.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
MIPIPE_EXT_VARIANT=ncp timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_native_gpu.py -x -q --timeout 120 --timeout-method thread -k "norm or reference or block" > gpurun_out/ncp_tests.log 2>&1
rc=$?; tail -2 gpurun_out/ncp_tests.log; [ $rc -ne 0 ] && exit $rc
: > gpurun_out/ncp_ab.txt
for v in "" ncp "" ncp; do
  MIPIPE_EXT_VARIANT=$v timeout -k 10 200 python -u tools/ref_table_gpu.py --engine trainer --precision bf16 --only 8x8,4x4 > gpurun_out/ncp_tr.log 2>&1 || exit 1
  echo "${v:-default} $(grep tokens_per_s gpurun_out/ncp_tr.log | cut -c1-70 | tr '\n' ' ')" >> gpurun_out/ncp_ab.txt
done
cat gpurun_out/ncp_ab.txt
