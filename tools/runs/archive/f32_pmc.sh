# PMC passes over tools/f32_pmc_probe.py (one rocprofv3 run per counter group)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/f32pmc
i=0
for grp in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM GRBM_GUI_ACTIVE GRBM_COUNT" \
           "TA_BUSY_avr TA_TA_BUSY_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $grp --kernel-include-regex "gemm_f32|af32" --output-format csv -d gpurun_out/f32pmc/p$i -o run -- python3 tools/f32_pmc_probe.py > gpurun_out/f32pmc/p$i.log 2>&1 || exit 1
  find gpurun_out/f32pmc/p$i -name "*counter_collection.csv" -exec cp {} gpurun_out/f32pmc/p$i.csv \;
done
