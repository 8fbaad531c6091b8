#!/bin/bash
# End-of-session check: full GPU suite, smoke, 1-GPU bench (driver's command), kernel stats
# of the default bench at m = 4, kernel microbenchmarks.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && \
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench1.log 2>&1 && \
bash tools/prof.sh gpt2s_m4 && \
timeout -k 10 300 python -u tools/bench_kernels.py --json gpurun_out/kernel_microbench.json > gpurun_out/bk_all.log 2>&1
rc=$?
tail -1 gpurun_out/pytest_gpu.log; tail -1 gpurun_out/smoke.log; tail -1 gpurun_out/bench1.log | cut -c1-300
exit $rc
