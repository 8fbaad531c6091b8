#!/bin/bash
# End-of-round evidence: headline bench (the driver's command) + kernel stats of the headline step.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r5ac
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r5ac/bench.log 2>&1
rc=$?; grep '^{' gpurun_out/r5ac/bench.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], {k: v["tok_s"] for k, v in d["schedules"].items()})'; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r5ac/prof -o run -- python3 bench.py --gpus 1 --steps 10 --warmup 3 --schedules none --ref-fp32 0 --no-supervise --no-bubble > gpurun_out/r5ac/prof.log 2>&1
rc=$?; grep '^{' gpurun_out/r5ac/prof.log | cut -c1-120; exit $rc
