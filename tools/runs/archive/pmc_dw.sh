#!/bin/bash
# PMC counters: dW GEMM (GPT-2 fc1 shape) TT (as used) vs the same problem with NT operands
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/pmc_dw
mkdir -p $OUT
run() {
  local tag=$1; shift; local ctr=$1; shift
  timeout -s KILL 90 rocprofv3 --pmc $ctr --kernel-trace --output-format csv -d $OUT/$tag -o run -- \
    python3 tools/gemm_probe.py "$@" > $OUT/$tag.log 2>&1
}
for L in tt ntacc; do
  run ${L}_cyc "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS" 3072 768 16384 -1 $L 5 && \
  run ${L}_lds "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VALU" 3072 768 16384 -1 $L 5 || exit 1
done
