#!/bin/bash
# Attention forward max3: numerics + same-box A/B timing (this tree vs _ab/old).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r5aa
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_kernels_gpu.py -k "attn or attention" > gpurun_out/r5aa/tests.log 2>&1
rc=$?; tail -2 gpurun_out/r5aa/tests.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2 3; do
  echo "new $(timeout -k 10 120 python tools/attn_time.py 2>/dev/null | grep '^{')" || exit 1
  echo "old $(cd _ab/old && timeout -k 10 120 python tools/attn_time.py 2>/dev/null | grep '^{')" || exit 1
done
