#!/bin/bash
# Round 6: QKV bias gradient summed inside the v2 attention backward (MIPIPE_FUSE_QKV_BIAS=1)
# vs the separate column-sum pass (default), headline step, interleaved.
set -o pipefail
mkdir -p gpurun_out
for v in sep fused sep2 fused2; do
  env="MIPIPE_FUSE_QKV_BIAS=0"; case $v in fused|fused2) env="MIPIPE_FUSE_QKV_BIAS=1";; esac
  out=$(env $env timeout -k 10 240 python bench.py --no-supervise --schedules none --ref-fp32 0 --no-bubble --steps 20 --warmup 5 2> gpurun_out/r6_qkvb_$v.log | tail -1)
  [ -n "$out" ] || { tail -5 gpurun_out/r6_qkvb_$v.log; exit 1; }
  echo "$v: $(echo "$out" | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['last_loss'])")" | tee -a gpurun_out/r6_qkvb.txt
done
