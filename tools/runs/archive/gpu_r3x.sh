#!/bin/bash
# End-of-round reference tables on one GPU: the reference's 9 (L, H) configs through the
# reference-compatible API at its precision (fp32, fwd+bwd) and at bf16.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 500 python -u tools/ref_table_gpu.py --engine native --precision fp32 --json gpurun_out/r3_end_ref_table_fp32_native.json > gpurun_out/ref_end_fp32.log 2>&1 && \
timeout -k 10 500 python -u tools/ref_table_gpu.py --engine native --precision bf16 --json gpurun_out/r3_end_ref_table_bf16_native.json > gpurun_out/ref_end_bf16.log 2>&1
rc=$?
grep -h tokens_per_s gpurun_out/ref_end_fp32.log gpurun_out/ref_end_bf16.log | cut -c1-120
exit $rc
