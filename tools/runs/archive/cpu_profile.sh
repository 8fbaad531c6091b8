#!/bin/bash
# host-side profile of a small-microbatch bench (launch / Python overhead) + GPU kernel time
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/cpuprof
for g in 0 1; do
  timeout -k 10 300 python -m cProfile -o gpurun_out/cpuprof/g$g.prof bench.py --mbs 1 --seq 1024 --steps 20 --warmup 3 --no-bubble --graphs $g > gpurun_out/cpuprof/g$g.log 2>&1 || exit 1
  python - <<PY
import pstats
p = pstats.Stats("gpurun_out/cpuprof/g$g.prof")
p.sort_stats("tottime").print_stats(18)
PY
done > gpurun_out/cpuprof/summary.txt 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/cpuprof/roc -o run -- python3 bench.py --mbs 1 --seq 1024 --steps 20 --warmup 3 --no-bubble --graphs 1 > gpurun_out/cpuprof/roc.log 2>&1
find gpurun_out/cpuprof/roc -name "*kernel_stats.csv" -exec cp {} gpurun_out/cpuprof/kstats.csv \;
