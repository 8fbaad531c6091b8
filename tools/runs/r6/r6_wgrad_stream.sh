#!/bin/bash
# Round 6: weight-gradient GEMMs on the side stream (default) vs inline, with the round-6 kernels.
set -o pipefail
mkdir -p gpurun_out
for v in side inline side2 inline2; do
  env="MIPIPE_WGRAD_STREAM=1"; case $v in inline|inline2) env="MIPIPE_WGRAD_STREAM=0";; esac
  out=$(env $env timeout -k 10 240 python bench.py --no-supervise --schedules none --ref-fp32 0 --no-bubble --steps 20 --warmup 5 2> gpurun_out/r6_wgs_$v.log | tail -1)
  [ -n "$out" ] || { tail -5 gpurun_out/r6_wgs_$v.log; exit 1; }
  echo "$v: $(echo "$out" | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")" | tee -a gpurun_out/r6_wgs.txt
done
