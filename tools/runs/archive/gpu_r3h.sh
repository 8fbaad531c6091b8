#!/bin/bash
# bf16 attention (key-split short-sequence forward): kernel tests, A/B at the reference
# shape; then compat-vs-trainer.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "attn or attention" > gpurun_out/attn_tests.log 2>&1
rc=$?; tail -2 gpurun_out/attn_tests.log; [ $rc -ne 0 ] && exit $rc
: > gpurun_out/attn_ks2_ab.txt
for ab in 1 0 1 0; do
  MIPIPE_ATTN_KS2=$ab timeout -k 10 120 python -u tools/bench_kernels.py --only attn_B8S128 > gpurun_out/attn_ks2_$ab.log 2>&1 || exit 1
  echo "ks2=$ab $(grep attn_B8S128 gpurun_out/attn_ks2_$ab.log)" >> gpurun_out/attn_ks2_ab.txt
done
cat gpurun_out/attn_ks2_ab.txt
bash tools/gpu_r3g.sh
