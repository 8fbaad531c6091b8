#!/bin/bash
# Round 6: memory-level parallelism in the column-sum (8 rows per wave in flight) and the norm
# backward (two rows ahead): numerics, bandwidth probe and the step, vs the previous build
# (the _C_pre variant).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py \
  -k "norm or colsum or act" > gpurun_out/r6_mlp_tests.log 2>&1 || { tail -30 gpurun_out/r6_mlp_tests.log; exit 1; }
tail -1 gpurun_out/r6_mlp_tests.log
for v in new pre; do
  env=""; [ $v = pre ] && env="MIPIPE_EXT_VARIANT=pre"
  echo "== $v"; env $env NORM_PROBE_T=65536 timeout -k 10 120 python tools/norm_probe.py 2>/dev/null | grep -v amdgpu.ids | tee -a gpurun_out/r6_mlp_probe_$v.txt || exit 1
done
for v in new pre new2 pre2; do
  env="MIPIPE_ATTN_FWD=2"; case $v in pre|pre2) env="MIPIPE_EXT_VARIANT=pre";; esac
  out=$(env $env timeout -k 10 240 python bench.py --no-supervise --schedules none --ref-fp32 0 --no-bubble --steps 20 --warmup 5 2> gpurun_out/r6_mlp_bench_$v.log | tail -1)
  [ -n "$out" ] || { tail -5 gpurun_out/r6_mlp_bench_$v.log; exit 1; }
  echo "$v: $(echo "$out" | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")" | tee -a gpurun_out/r6_mlp_bench.txt
done
