set -o pipefail
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r6_hbm_pools.jsonl
: > $out
for cfg in "1F1B 64 2" "1F1B 16 8"; do
  set -- $cfg
  timeout -k 10 150 python tools/hbm_probe.py --pools --schedule $1 --mbs $2 --microbatches $3 >> $out 2>> gpurun_out/r6_hbm_pools.err || exit 1
done
MIPIPE_LANES=1 timeout -k 10 150 python tools/hbm_probe.py --pools --schedule 1F1B --mbs 64 --microbatches 2 >> $out 2>> gpurun_out/r6_hbm_pools.err || exit 1
