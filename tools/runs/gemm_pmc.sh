# PMC passes over tools/gemm_pmc_probe.py (gemm3 / gemm8 / hipBLASLt on one NT shape)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
D=gpurun_out/gpmc
mkdir -p $D
ARGS="$*"
timeout -s KILL 90 rocprofv3 --kernel-trace --stats --output-format csv -d $D/stats -o run -- python3 tools/gemm_pmc_probe.py $ARGS > $D/stats.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM --output-format csv -d $D/pmc1 -o run -- python3 tools/gemm_pmc_probe.py $ARGS > $D/pmc1.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_MISC GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $D/pmc2 -o run -- python3 tools/gemm_pmc_probe.py $ARGS > $D/pmc2.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_SALU --output-format csv -d $D/pmc3 -o run -- python3 tools/gemm_pmc_probe.py $ARGS > $D/pmc3.log 2>&1 || exit 1
for p in stats pmc1 pmc2 pmc3; do find $D/$p -name "*.csv" -exec cp {} $D/ \; ; done
ls $D
