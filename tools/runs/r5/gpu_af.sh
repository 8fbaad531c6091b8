#!/bin/bash
# Model families on one GPU with the round-3 table's arguments (round-5 kernels).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r5af
for a in "--model gpt2-medium" "--model gpt2-large --mbs 32 --microbatches 2" "--model llama3-1b --mbs 16 --seq 2048 --microbatches 2" "--model reference --mbs 8 --seq 128 --microbatches 4"; do
  timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-bubble --schedules none --ref-fp32 0 $a > gpurun_out/r5af/bm.log 2>&1 || { tail -5 gpurun_out/r5af/bm.log; exit 1; }
  echo "$a :: $(grep '^{' gpurun_out/r5af/bm.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["model_tflops_per_gpu"], d.get("last_loss"), d.get("hbm_peak_gb_per_gpu"))')"
done
