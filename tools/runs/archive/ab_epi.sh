set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "gemm" --timeout 120 --timeout-method thread > gpurun_out/epi_test.log 2>&1 && \
timeout -k 10 300 python tools/bench_kernels.py --only gelu > gpurun_out/epi_bench.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/epi_b.log 2>&1
