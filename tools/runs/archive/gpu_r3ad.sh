#!/bin/bash
# Model families, second half: Llama-3 1B with hipBLASLt plain GEMMs (now one lane), the
# reference model, Llama-3 8B seq 8192 step.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
: > gpurun_out/families2.txt
run() {
  timeout -k 10 300 env $1 python bench.py --steps 5 --warmup 2 --no-bubble $2 > gpurun_out/bm2.log 2>&1 || { tail -20 gpurun_out/bm2.log; return 1; }
  echo "$2 [$1] :: $(tail -1 gpurun_out/bm2.log | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["model_tflops_per_gpu"], d.get("last_loss"), d["hbm_peak_gb_per_gpu"], d["config"]["microbatch_lanes"])')" >> gpurun_out/families2.txt
}
run MIPIPE_GEMM=hip "--model reference --mbs 8 --seq 128 --microbatches 4" && \
run MIPIPE_GEMM=auto "--model llama3-1b --mbs 16 --seq 2048 --microbatches 2" && \
timeout -k 10 400 python tools/llama8b_step.py --steps 4 > gpurun_out/l8b_hip.log 2>&1 && \
echo "llama3-8b seq 8192 :: $(tail -1 gpurun_out/l8b_hip.log)" >> gpurun_out/families2.txt
rc=$?
cat gpurun_out/families2.txt
exit $rc
