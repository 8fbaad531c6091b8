#!/bin/bash
# PMC counters for the attention kernels (counters + kernel trace only)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/pmc_attn
mkdir -p $OUT
run() {
  local tag=$1; shift; local ctr=$1; shift
  timeout -k 10 120 rocprofv3 --pmc $ctr --kernel-trace --output-format csv -d $OUT/$tag -o run -- \
    python3 tools/attn_probe.py "$@" > $OUT/$tag.log 2>&1
}
run cyc "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY" 16 1024 12 12 64 1 && \
run valu "SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_ACTIVE_INST_ANY SQ_INSTS_SALU" 16 1024 12 12 64 1 && \
run mfma "SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT" 16 1024 12 12 64 1 && \
run mem "SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INST_CYCLES_VMEM_RD TCC_HIT_sum" 16 1024 12 12 64 1
ls $OUT
