#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
R="--model reference --mbs 8 --seq 128 --microbatches 4 --steps 20 --warmup 5"
for L in 3 4 2; do timeout -k 10 200 env MIPIPE_LANES=$L python bench.py $R > gpurun_out/ln2_ref_$L.log 2>&1 || exit 1; done && \
for L in 2 1 2 1; do timeout -k 10 200 env MIPIPE_LANES=$L python bench.py --steps 10 --warmup 3 > gpurun_out/ln2_gpt2_$L.log 2>&1 || exit 1; done
