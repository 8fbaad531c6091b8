set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
MIPIPE_GEMM_M16T=1 timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "gemm" --timeout 120 --timeout-method thread > gpurun_out/m16t_test.log 2>&1 && \
timeout -k 10 300 python tools/bench_kernels.py --only dw > gpurun_out/m16t_off.log 2>&1 && \
MIPIPE_GEMM_M16T=1 timeout -k 10 300 python tools/bench_kernels.py --only dw > gpurun_out/m16t_on.log 2>&1 && \
true
