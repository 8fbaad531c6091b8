#!/bin/bash
# The reference table at the reference's precision (fp32): this framework's kernels
# (native) vs the reference's nn.Module on ATen; then a kernel-trace profile of L8H8.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 500 python -u tools/ref_table_gpu.py --engine native --precision fp32 --json gpurun_out/r3_ref_table_fp32_native.json > gpurun_out/ref_native.log 2>&1 && \
timeout -k 10 400 python -u tools/ref_table_gpu.py --engine aten --json gpurun_out/r3_ref_table_fp32_aten.json > gpurun_out/ref_aten.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_ref -o run -- python3 tools/ref_table_gpu.py --engine native --precision fp32 --only 8x8 --iters 5 --warmup 2 > gpurun_out/ref_prof.log 2>&1
rc=$?
grep tokens_per_s gpurun_out/ref_native.log | cut -c1-200
grep tokens_per_s gpurun_out/ref_aten.log | cut -c1-200
[ $rc -ne 0 ] && exit $rc
# A/B: fused lane merge + clip-norm sum of squares vs separate passes (bf16 trainer, L8H8)
for ab in 1 0 1 0; do
  MIPIPE_FUSED_MERGE_NORM=$ab timeout -k 10 200 python -u tools/ref_table_gpu.py --engine trainer --only 8x8 > gpurun_out/ab_merge_$ab.log 2>&1 || exit 1
  echo "fused=$ab $(grep tokens_per_s gpurun_out/ab_merge_$ab.log | cut -c1-120)" >> gpurun_out/ab_merge.txt
done
cat gpurun_out/ab_merge.txt
