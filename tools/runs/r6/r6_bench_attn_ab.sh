#!/bin/bash
# Round 6: headline bench (N = 1) with the v2 attention kernels vs the round-5 ones, interleaved.
set -o pipefail
mkdir -p gpurun_out
for v in new old new2 old2; do
  case $v in
    old|old2) env="MIPIPE_ATTN_FWD=1 MIPIPE_ATTN_BWD_DQ=1 MIPIPE_ATTN_BWD_DKDV=1" ;;
    new|new2) env="MIPIPE_ATTN_FWD=2" ;;
  esac
  env $env timeout -k 10 400 python bench.py > gpurun_out/r6_bench_$v.json 2> gpurun_out/r6_bench_$v.log || { tail -20 gpurun_out/r6_bench_$v.log; exit 1; }
  echo "$v: $(python -c "import json,sys; d=json.loads(open('gpurun_out/r6_bench_$v.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'])")"
done
