#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_native_runner_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/lm_test.log 2>&1 && \
for i in 1 2; do
timeout -k 10 200 python bench.py --model reference --mbs 8 --seq 128 --microbatches 4 --steps 20 --warmup 5 > gpurun_out/lm_ref_$i.log 2>&1 && \
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > gpurun_out/lm_gpt2_$i.log 2>&1 || exit 1; done
