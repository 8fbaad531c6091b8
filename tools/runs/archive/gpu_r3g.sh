#!/bin/bash
# compat API (reference-compatible Schedule1F1B.step loop) vs PipelineTrainer fwd+bwd, L8H8, both precisions
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
: > gpurun_out/compat_vs_trainer.txt
for prec in bf16 fp32; do
  timeout -k 10 200 python -u tools/ref_table_gpu.py --engine native --precision $prec --only 8x8 > gpurun_out/cvt_native_$prec.log 2>&1 || exit 1
  timeout -k 10 200 python -u tools/ref_table_gpu.py --engine trainer --fwd-bwd --precision $prec --only 8x8 > gpurun_out/cvt_trainer_$prec.log 2>&1 || exit 1
  echo "$prec compat  $(grep tokens_per_s gpurun_out/cvt_native_$prec.log | cut -c1-110)" >> gpurun_out/compat_vs_trainer.txt
  echo "$prec trainer $(grep tokens_per_s gpurun_out/cvt_trainer_$prec.log | cut -c1-110)" >> gpurun_out/compat_vs_trainer.txt
done
cat gpurun_out/compat_vs_trainer.txt
