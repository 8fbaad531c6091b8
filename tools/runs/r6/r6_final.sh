#!/bin/bash
# Round 6 final check, the way the driver runs it: GPU suite, smoke(), default bench (N = 1).
set -o pipefail
mkdir -p gpurun_out/final
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/final/gpu_suite.log 2>&1 || { tail -30 gpurun_out/final/gpu_suite.log; exit 1; }
tail -2 gpurun_out/final/gpu_suite.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final/smoke.log 2>&1 || { tail -20 gpurun_out/final/smoke.log; exit 1; }
tail -1 gpurun_out/final/smoke.log
timeout -k 10 600 python bench.py > gpurun_out/final/bench.json 2> gpurun_out/final/bench.log || { tail -20 gpurun_out/final/bench.log; exit 1; }
tail -1 gpurun_out/final/bench.json | cut -c1-400
