#!/bin/bash
# bench.py at N=1: m = 4 (new default, m = 4N) vs m = 2, and the dW split-K cap at m = 4;
# then bench.py's multi-rank path at m = 4N on one GPU (gloo host staging, N = 2/4/8).
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
: > gpurun_out/bench_m_ab.txt
run() {  # tag "VAR=x ..." [bench args...]
  local tag=$1 envs=$2; shift 2
  timeout -k 10 300 env $envs python -u bench.py --steps 10 --warmup 3 "$@" > gpurun_out/b_$tag.log 2>&1 || return 1
  echo "$tag $(tail -1 gpurun_out/b_$tag.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["config"]["microbatches"])')" >> gpurun_out/bench_m_ab.txt
}
for r in 1 2; do
  run m4_$r "MIPIPE_X=0" && run m2_$r "MIPIPE_X=0" --microbatches 2 && run m4_split8_$r "MIPIPE_DW_MAXSPLIT=8" && \
    run m4_split16_$r "MIPIPE_DW_MAXSPLIT=16" || exit 1
done
cat gpurun_out/bench_m_ab.txt
export MIPIPE_DIST_BACKEND=gloo OMP_NUM_THREADS=2
timeout -k 10 300 python bench.py --gpus 2 --steps 2 --warmup 1 --mbs 4 > gpurun_out/mr_bench2.log 2>&1 && \
timeout -k 10 300 python bench.py --gpus 4 --steps 2 --warmup 1 --mbs 4 > gpurun_out/mr_bench4.log 2>&1 && \
timeout -k 10 400 python bench.py --gpus 8 --steps 2 --warmup 1 --mbs 2 > gpurun_out/mr_bench8.log 2>&1
rc=$?
for f in gpurun_out/mr_bench*.log; do echo "$f: $(grep '^{' $f | cut -c1-300)"; done
exit $rc
