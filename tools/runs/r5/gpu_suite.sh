#!/bin/bash
# The whole GPU suite (what the driver runs at round end) + smoke().
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r5s
timeout -k 10 1000 python -u -m pytest -x -v --timeout 400 --timeout-method thread -m gpu tests > gpurun_out/r5s/suite.log 2>&1
rc=$?; tail -6 gpurun_out/r5s/suite.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5s/smoke.log 2>&1
rc=$?; tail -3 gpurun_out/r5s/smoke.log; exit $rc
