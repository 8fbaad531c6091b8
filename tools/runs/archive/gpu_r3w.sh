#!/bin/bash
# BASELINE configs 3-5 code-path rehearsal (8 ranks on one GPU, gloo) with the round-3 code
# (m = 4N, ZeRO-1 head, native collectives), then the report.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash tools/bench_configs_rehearsal.sh
rc=$?
for f in gpurun_out/cfg3.log gpurun_out/cfg4.log gpurun_out/cfg5.log; do echo "$f: $(grep '^{' $f | cut -c1-160)"; done
exit $rc
