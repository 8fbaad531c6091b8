set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/attn
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/attn/stats -o run -- python3 tools/attn_bwd_probe.py > gpurun_out/attn/stats.log 2>&1 || exit 1
find gpurun_out/attn/stats -name "*kernel_stats.csv" -exec cp {} gpurun_out/attn/kernel_stats.csv \;
find gpurun_out/attn/stats -name "*kernel_trace.csv" -exec cp {} gpurun_out/attn/kernel_trace.csv \;
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM --kernel-include-regex "attn" --output-format csv -d gpurun_out/attn/pmc1 -o run -- python3 tools/attn_bwd_probe.py > gpurun_out/attn/pmc1.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_MISC GRBM_GUI_ACTIVE GRBM_COUNT --kernel-include-regex "attn" --output-format csv -d gpurun_out/attn/pmc2 -o run -- python3 tools/attn_bwd_probe.py > gpurun_out/attn/pmc2.log 2>&1 || exit 1
find gpurun_out/attn/pmc1 -name "*counter_collection.csv" -exec cp {} gpurun_out/attn/pmc1.csv \;
find gpurun_out/attn/pmc2 -name "*counter_collection.csv" -exec cp {} gpurun_out/attn/pmc2.csv \;
