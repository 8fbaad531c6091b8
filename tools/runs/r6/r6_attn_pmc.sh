#!/bin/bash
# Round 6: PMC counters of the attention forward, v1 vs v2 (B 16, S 1024, H 12, D 64 causal).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/apmc
for v in 1 2; do
  export MIPIPE_ATTN_FWD=$v
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM --kernel-include-regex "attn_fwd" --output-format csv -d gpurun_out/apmc/v${v}_p1 -o run -- python3 tools/attn_time.py 16 1024 12 64 > gpurun_out/apmc/v${v}_p1.log 2>&1 || exit 1
  timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU GRBM_GUI_ACTIVE GRBM_COUNT --kernel-include-regex "attn_fwd" --output-format csv -d gpurun_out/apmc/v${v}_p2 -o run -- python3 tools/attn_time.py 16 1024 12 64 > gpurun_out/apmc/v${v}_p2.log 2>&1 || exit 1
  timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_INST_LEVEL_LDS SQ_INSTS_VALU_TRANS_F32 GRBM_GUI_ACTIVE --kernel-include-regex "attn_fwd" --output-format csv -d gpurun_out/apmc/v${v}_p3 -o run -- python3 tools/attn_time.py 16 1024 12 64 > gpurun_out/apmc/v${v}_p3.log 2>&1 || echo "pass 3 failed (counter names?)"
done
for v in 1 2; do echo "== v$v"; python3 tools/pmc_summary.py gpurun_out/apmc/v${v}_p1; python3 tools/pmc_summary.py gpurun_out/apmc/v${v}_p2; python3 tools/pmc_summary.py gpurun_out/apmc/v${v}_p3 || true; done > gpurun_out/apmc/summary.txt 2>&1
cat gpurun_out/apmc/summary.txt
