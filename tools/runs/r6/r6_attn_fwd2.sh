#!/bin/bash
# Round 6: attention forward v2 (paired causal blocks, buffer-loaded K/V, lazy rescale):
# correctness, then v1 vs v2 time at the probe shape and the headline microbatch.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py \
  -k "attention" > gpurun_out/r6_attn_fwd2_tests.log 2>&1 || { tail -30 gpurun_out/r6_attn_fwd2_tests.log; exit 1; }
tail -2 gpurun_out/r6_attn_fwd2_tests.log
for shape in "16 1024 12 64" "64 1024 12 64"; do
  for v in 1 2; do
    echo "v$v $shape: $(MIPIPE_ATTN_FWD=$v timeout -k 10 120 python tools/attn_time.py $shape)" | tee -a gpurun_out/r6_attn_fwd2_time.txt || exit 1
  done
done
