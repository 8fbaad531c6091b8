#!/bin/bash
# PMC counters of the short-sequence attention kernels at the reference shape (B 8, S 128,
# H 8, d_h 96, non-causal): counters + kernel trace only, one pass per counter group
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/pmc_attn_short
mkdir -p $OUT
run() {
  local tag=$1; shift; local ctr=$1; shift
  timeout -k 10 120 rocprofv3 --pmc $ctr --kernel-trace --output-format csv -d $OUT/$tag -o run -- \
    python3 tools/attn_probe.py 8 128 8 8 96 0 > $OUT/$tag.log 2>&1
}
run cyc "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY" && \
run valu "SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_ACTIVE_INST_ANY SQ_INSTS_SALU" && \
run mfma "SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT" && \
run mem "SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INST_CYCLES_VMEM_RD SQ_INSTS_SMEM"
