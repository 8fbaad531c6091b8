#!/bin/bash
# Round 6: dQ v3 (paired causal query blocks on one XCD, MIPIPE_ATTN_BWD_DQ=3) vs v2, with dK/dV v3
# now the default: attention tests on both dQ kernels, the step interleaved, then the GPU suite.
set -o pipefail
mkdir -p gpurun_out
MIPIPE_ATTN_BWD_DQ=3 timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py \
  -k "attention" > gpurun_out/r6_dq3_tests.log 2>&1 || { tail -30 gpurun_out/r6_dq3_tests.log; exit 1; }
tail -1 gpurun_out/r6_dq3_tests.log
for v in v2 v3 v2b v3b; do
  env="MIPIPE_ATTN_BWD_DQ=2"; case $v in v3|v3b) env="MIPIPE_ATTN_BWD_DQ=3";; esac
  out=$(env $env timeout -k 10 240 python bench.py --no-supervise --schedules none --ref-fp32 0 --no-bubble --steps 20 --warmup 5 2> gpurun_out/r6_dq3_bench_$v.log | tail -1)
  [ -n "$out" ] || { tail -5 gpurun_out/r6_dq3_bench_$v.log; exit 1; }
  echo "$v: $(echo "$out" | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")" | tee -a gpurun_out/r6_dq3_bench.txt
done
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/r6_dq3_suite.log 2>&1 || { tail -30 gpurun_out/r6_dq3_suite.log; exit 1; }
tail -1 gpurun_out/r6_dq3_suite.log
