#!/bin/bash
# Grouped weight-gradient launches: kernel tests, then the reference model (L8H8, batch
# 32 x 128, m = 4) and GPT-2 small benches with MIPIPE_WGRAD_GROUP=1 / 0 interleaved.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
R="--model reference --mbs 8 --seq 128 --microbatches 4 --steps 20 --warmup 5"
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_native_gpu.py tests/test_native_runner_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/wg_test.log 2>&1 && \
for i in 1 2; do
  timeout -k 10 200 env MIPIPE_WGRAD_GROUP=1 python bench.py $R > gpurun_out/wg_ref_on_$i.log 2>&1 && \
  timeout -k 10 200 env MIPIPE_WGRAD_GROUP=0 python bench.py $R > gpurun_out/wg_ref_off_$i.log 2>&1 || exit 1
done && \
timeout -k 10 200 python bench.py --steps 10 --warmup 3 > gpurun_out/wg_gpt2.log 2>&1
