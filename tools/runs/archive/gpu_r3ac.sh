#!/bin/bash
# Model families on one GPU with round-3 defaults (bench.py: HIP graphs, native tape, lanes,
# AdamW included), Llama-3 8B step, and plain GEMMs on hipBLASLt (MIPIPE_GEMM=auto) as an A/B.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
: > gpurun_out/families.txt
for a in "--model gpt2-medium" "--model gpt2-large --mbs 32 --microbatches 2" "--model llama3-1b --mbs 16 --seq 2048 --microbatches 2" "--model reference --mbs 8 --seq 128 --microbatches 4"; do
  for g in hip auto; do
    MIPIPE_GEMM=$g timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-bubble $a > gpurun_out/bm.log 2>&1 || { tail -20 gpurun_out/bm.log; exit 1; }
    echo "$a [MIPIPE_GEMM=$g] :: $(tail -1 gpurun_out/bm.log | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["model_tflops_per_gpu"], d.get("last_loss"), d["hbm_peak_gb_per_gpu"])')" >> gpurun_out/families.txt
  done
done
for g in hip auto; do
  MIPIPE_GEMM=$g timeout -k 10 400 python tools/llama8b_step.py --steps 4 > gpurun_out/l8b_$g.log 2>&1 || { tail -20 gpurun_out/l8b_$g.log; exit 1; }
  echo "llama3-8b seq 8192 [MIPIPE_GEMM=$g] :: $(tail -1 gpurun_out/l8b_$g.log)" >> gpurun_out/families.txt
done
cat gpurun_out/families.txt
