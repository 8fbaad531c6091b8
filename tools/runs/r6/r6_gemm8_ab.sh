# gemm8 numerics (GEMM GPU tests) + in-step A/B at 16K-token microbatches (MIPIPE_GEMM8=0 vs auto)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "gemm" --timeout 120 --timeout-method thread > gpurun_out/r6_gemm_tests.log 2>&1 || exit 1
for i in 1 2; do
  for g in 0 auto; do
    MIPIPE_GEMM8=$g timeout -k 10 200 python bench.py --mbs 16 --microbatches 8 --steps 10 --warmup 3 --schedules none \
      --ref-fp32 0 --base-configs 0 > gpurun_out/r6_ab_g8_${g}_$i.json 2> gpurun_out/r6_ab_g8_${g}_$i.err || exit 1
  done
done
