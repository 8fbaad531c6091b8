#!/bin/bash
# Round 6: norm / colsum bandwidth probe, and PMC counters of attention forward v2.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/apmc2
timeout -k 10 120 python tools/norm_probe.py > gpurun_out/apmc2/norm_probe.txt 2>&1 || { tail gpurun_out/apmc2/norm_probe.txt; exit 1; }
cat gpurun_out/apmc2/norm_probe.txt
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM --kernel-include-regex "attn_fwd2" --output-format csv -d gpurun_out/apmc2/p1 -o run -- python3 tools/attn_time.py 16 1024 12 64 > gpurun_out/apmc2/p1.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE GRBM_COUNT --kernel-include-regex "attn_fwd2" --output-format csv -d gpurun_out/apmc2/p2 -o run -- python3 tools/attn_time.py 16 1024 12 64 > gpurun_out/apmc2/p2.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_INST_LDS SQ_INSTS_VALU_TRANS_F32 SQ_INST_LEVEL_LDS SQ_INSTS_BRANCH SQ_IFETCH SQ_WAVE_CYCLES GRBM_GUI_ACTIVE --kernel-include-regex "attn_fwd2" --output-format csv -d gpurun_out/apmc2/p3 -o run -- python3 tools/attn_time.py 16 1024 12 64 > gpurun_out/apmc2/p3.log 2>&1 || echo "pass 3 failed"
ls gpurun_out/apmc2
