#!/bin/bash
# Same-box A/B of the GELU-derivative epilogue on GPT-2 large and medium: this tree vs _ab/old
# (HEAD with that change reverted).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r5ah
for m in "--model gpt2-large --mbs 32 --microbatches 2" "--model gpt2-medium"; do
for i in 1 2; do
  timeout -k 10 250 python bench.py --steps 10 --warmup 3 --no-bubble --schedules none --ref-fp32 0 $m > gpurun_out/r5ah/n.log 2>&1 || exit 1
  (cd _ab/old && timeout -k 10 250 python bench.py --steps 10 --warmup 3 --no-bubble --schedules none --ref-fp32 0 $m) > gpurun_out/r5ah/o.log 2>&1 || exit 1
  echo "$m new $(grep '^{' gpurun_out/r5ah/n.log | python3 -c 'import sys,json; print(json.loads(sys.stdin.read())["value"])') old $(grep '^{' gpurun_out/r5ah/o.log | python3 -c 'import sys,json; print(json.loads(sys.stdin.read())["value"])')"
done; done
