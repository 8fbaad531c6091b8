#!/bin/bash
# Round 6: headline step shape with the v2 attention: sequences per microbatch x lanes (1 GPU).
set -o pipefail
mkdir -p gpurun_out
run() {  # tag, env, args
  local tag=$1 env=$2; shift 2
  out=$(env $env timeout -k 10 240 python bench.py --no-supervise --schedules none --ref-fp32 0 --no-bubble --steps 20 --warmup 5 "$@" 2> gpurun_out/r6_cfg_$tag.log | tail -1)
  [ -n "$out" ] || { tail -5 gpurun_out/r6_cfg_$tag.log; return 1; }
  echo "$tag: $(echo "$out" | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['config'].get('microbatch_lanes', ''))")" | tee -a gpurun_out/r6_cfg_sweep.txt
}
run m2x64_l2 "MIPIPE_LANES=2" --mbs 64 --microbatches 2 &&
run m4x32_l2 "MIPIPE_LANES=2" --mbs 32 --microbatches 4 &&
run m4x32_l4 "MIPIPE_LANES=4" --mbs 32 --microbatches 4 &&
run m8x16_l4 "MIPIPE_LANES=4" --mbs 16 --microbatches 8 &&
run m2x64_l2b "MIPIPE_LANES=2" --mbs 64 --microbatches 2 &&
run m4x32_l4b "MIPIPE_LANES=4" --mbs 32 --microbatches 4
