#!/bin/bash
# Whole GPU suite + smoke + the driver's bench command (all schedules + reference fp32).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r5x
timeout -k 10 1000 python -u -m pytest -x -v --timeout 400 --timeout-method thread -m gpu tests > gpurun_out/r5x/suite.log 2>&1
rc=$?; tail -3 gpurun_out/r5x/suite.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5x/smoke.log 2>&1
rc=$?; tail -1 gpurun_out/r5x/smoke.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r5x/bench.log 2>&1
rc=$?; grep '^{' gpurun_out/r5x/bench.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], {k: (v["tok_s"], v.get("hbm_peak_gb_per_gpu")) for k, v in d["schedules"].items()}, [(r["schedule"], r["tok_s"]) for r in d["reference_fp32"]["rows"]])'; exit $rc
