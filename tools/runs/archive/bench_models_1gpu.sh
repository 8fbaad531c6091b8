#!/bin/bash
# bench.py on one GPU across model families (shape coverage for the GEMM / attention /
# norm kernels): prints value, step time and loss per model
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for a in "--model gpt2-medium --mbs 8" "--model gpt2-large --mbs 8" "--model llama3-1b --mbs 4 --seq 2048" "--model reference --mbs 8 --seq 128 --microbatches 4"; do
  timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-bubble $a > gpurun_out/bm.log 2>&1 || { tail -20 gpurun_out/bm.log; exit 1; }
  echo "$a :: $(tail -1 gpurun_out/bm.log | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["model_tflops_per_gpu"], d.get("last_loss"))')"
done
