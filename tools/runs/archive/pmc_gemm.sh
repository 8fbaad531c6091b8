#!/bin/bash
# PMC counters for a few GEMM configs (counters only with --kernel-trace; no sys/runtime trace)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/pmc_gemm
mkdir -p $OUT
run() {  # tag, counters, args...
  local tag=$1; shift; local ctr=$1; shift
  timeout -k 10 120 rocprofv3 --pmc $ctr --kernel-trace --output-format csv -d $OUT/$tag -o run -- \
    python3 tools/gemm_probe.py "$@" > $OUT/$tag.log 2>&1
}
for cfg in 0 4; do
  run c${cfg}_lds "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS" 16384 4096 4096 $cfg nt 3 && \
  run c${cfg}_cyc "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY" 16384 4096 4096 $cfg nt 3 && \
  run c${cfg}_mfma "SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_ACTIVE_INST_ANY" 16384 4096 4096 $cfg nt 3 || exit 1
done
run tt_lds "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS" 3072 768 16384 0 tt 3
find $OUT -name "*counter_collection.csv" | head -20
