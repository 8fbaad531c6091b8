#!/bin/bash
# Round 6: dK/dV v3 (paired causal key blocks on one XCD, MIPIPE_ATTN_BWD_DKDV=3) vs v2:
# attention tests on v3, standalone times, then the step (interleaved).
set -o pipefail
mkdir -p gpurun_out
MIPIPE_ATTN_BWD_DKDV=3 timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py \
  -k "attention" > gpurun_out/r6_dkdv3_tests.log 2>&1 || { tail -30 gpurun_out/r6_dkdv3_tests.log; exit 1; }
tail -1 gpurun_out/r6_dkdv3_tests.log
for shape in "16 1024 12 64" "64 1024 12 64"; do
  for v in 2 3 2 3; do
    echo "v$v $shape: $(MIPIPE_ATTN_BWD_DKDV=$v timeout -k 10 120 python tools/attn_time.py $shape)" | tee -a gpurun_out/r6_dkdv3_time.txt || exit 1
  done
done
for v in v2 v3 v2b v3b; do
  env="MIPIPE_ATTN_BWD_DKDV=2"; case $v in v3|v3b) env="MIPIPE_ATTN_BWD_DKDV=3";; esac
  out=$(env $env timeout -k 10 240 python bench.py --no-supervise --schedules none --ref-fp32 0 --no-bubble --steps 20 --warmup 5 2> gpurun_out/r6_dkdv3_bench_$v.log | tail -1)
  [ -n "$out" ] || { tail -5 gpurun_out/r6_dkdv3_bench_$v.log; exit 1; }
  echo "$v: $(echo "$out" | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")" | tee -a gpurun_out/r6_dkdv3_bench.txt
done
