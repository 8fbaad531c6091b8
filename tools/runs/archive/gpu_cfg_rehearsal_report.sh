#!/bin/bash
# Runs tools/bench_configs_rehearsal.sh and summarises each config's JSON line.
bash tools/bench_configs_rehearsal.sh; rc=$?
echo "rehearsal rc=$rc"
for f in cfg3 cfg4 cfg5; do
  [ -f gpurun_out/$f.log ] || continue
  tail -1 gpurun_out/$f.log | python -c '
import sys, json
d = json.loads(sys.stdin.read()); c = d["config"]
print(sys.argv[1], d["n_gpus"], c["model"], c["parallelism"], c["schedule"], "v", c["v"], "graphs", c["hip_graphs"],
      "native", c["native_runner"], c["p2p"], "loss", d.get("last_loss"), "arena MB", c.get("recv_arena_mb"),
      "recompute", c["recompute"])' $f
done
exit $rc
