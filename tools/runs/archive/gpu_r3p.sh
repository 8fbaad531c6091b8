#!/bin/bash
# hipBLASLt kernel names / configs for the GPT-2 GEMM shapes (kernel trace), and ours vs lib.
set -o pipefail
mkdir -p gpurun_out/blas_names
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/blas_names -o run -- \
  python3 tools/blas_names_probe.py > gpurun_out/blas_names/probe.log 2>&1 || exit 1
find gpurun_out/blas_names -name "*kernel_stats.csv" -exec cp {} gpurun_out/blas_names/kernel_stats.csv \;
timeout -k 10 200 python -u tools/bench_kernels.py --only fwd > gpurun_out/bk_fwd.log 2>&1
cat gpurun_out/blas_names/probe.log
