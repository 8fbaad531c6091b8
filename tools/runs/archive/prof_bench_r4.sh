#!/bin/bash
# rocprofv3 kernel stats of the headline step (GPT-2 small, 1 GPU, bench.py's in-process
# child path: MIPIPE_BENCH_CHILD=1 skips the supervisor, so the profiled program starts no
# other program) and of the reference fp32 config step (compat API, f32 kernels).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/prof4
export MIPIPE_BENCH_CHILD=1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof4/gpt2 -o run -- python3 bench.py --steps 10 --warmup 3 --no-bubble > gpurun_out/prof4/gpt2.log 2>&1 || exit 1
find gpurun_out/prof4/gpt2 -name "*kernel_stats.csv" -exec cp {} gpurun_out/prof4/gpt2_kernel_stats.csv \;
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof4/ref -o run -- python3 bench.py --phase ref --schedule 1F1B --steps 10 --warmup 3 > gpurun_out/prof4/ref.log 2>&1 || exit 1
find gpurun_out/prof4/ref -name "*kernel_stats.csv" -exec cp {} gpurun_out/prof4/ref_fp32_kernel_stats.csv \;
rm -rf gpurun_out/prof4/gpt2 gpurun_out/prof4/ref
