#!/bin/bash
# gemm3 tile raster group (MP_G3_GROUP, A/B builds) at the new default bench (2 x 64-sequence
# microbatches: M = 65536): default 2 vs 1 / 4 / 8, interleaved.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
: > gpurun_out/group_ab.txt
for v in "" g1 g4 g8 "" g1 g4 g8; do
  MIPIPE_EXT_VARIANT=$v timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > gpurun_out/grp_${v:-def}.log 2>&1 || exit 1
  echo "${v:-default(2)} $(tail -1 gpurun_out/grp_${v:-def}.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')" >> gpurun_out/group_ab.txt
done
cat gpurun_out/group_ab.txt
