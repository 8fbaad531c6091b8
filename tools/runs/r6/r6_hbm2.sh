# HBM after the empty_cache fix: reserved (steady state) vs the reconciled plan
set -o pipefail
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r6_hbm2.jsonl
: > $out
for cfg in "GPipe 64 2" "1F1B 64 2" "ZBH1 64 2" "GPipe 16 8" "1F1B 16 8" "ZBH1 16 8" "GPipe 8 2" "1F1B 8 2" "ZBH1 8 2" "GPipe 2 8" "1F1B 2 8" "ZBH1 2 8"; do
  set -- $cfg
  timeout -k 10 150 python tools/hbm_probe.py --pools --schedule $1 --mbs $2 --microbatches $3 >> $out 2>> gpurun_out/r6_hbm2.err || exit 1
done
