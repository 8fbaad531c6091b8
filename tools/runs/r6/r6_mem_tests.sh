# memory tests on reserved HBM + the default bench (HBM fields, perf unchanged)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests/test_native_runner_gpu.py tests/test_multirank_gpu.py -x -q --timeout 200 --timeout-method thread -k "stash or hbm or reserved" > gpurun_out/r6_mem_tests.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --schedules none --ref-fp32 0 > gpurun_out/r6_bench_mem.json 2> gpurun_out/r6_bench_mem.err || exit 1
