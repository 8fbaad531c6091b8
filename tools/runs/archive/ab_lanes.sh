#!/bin/bash
# Microbatch lanes (PP = 1): runner / kernel tests, then the reference model (L8H8, batch
# 32 x 128, m = 4) with MIPIPE_LANES=2 / 1 interleaved, then the GPT-2 small bench.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
R="--model reference --mbs 8 --seq 128 --microbatches 4 --steps 20 --warmup 5"
timeout -k 10 300 python -u -m pytest tests/test_native_runner_gpu.py tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/ln_test.log 2>&1 && \
for i in 1 2; do
  timeout -k 10 200 env MIPIPE_LANES=2 python bench.py $R > gpurun_out/ln_ref_on_$i.log 2>&1 && \
  timeout -k 10 200 env MIPIPE_LANES=1 python bench.py $R > gpurun_out/ln_ref_off_$i.log 2>&1 || exit 1
done && \
timeout -k 10 200 python bench.py --steps 10 --warmup 3 > gpurun_out/ln_gpt2.log 2>&1
