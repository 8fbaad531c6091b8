#!/bin/bash
set -e
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/final
timeout -k 10 700 python -u bench.py > gpurun_out/final/bench_default.json 2> gpurun_out/final/bench_default.err
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final/smoke.log 2>&1
