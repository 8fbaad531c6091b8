# Physical HBM (allocated / reserved / device used) vs the HBM plan, GPT-2 small, one GPU
set -o pipefail
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r6_hbm.jsonl
: > $out
for cfg in "GPipe 64 2" "1F1B 64 2" "ZBH1 64 2" "GPipe 16 8" "1F1B 16 8" "ZBH1 16 8"; do
  set -- $cfg
  timeout -k 10 150 python tools/hbm_probe.py --schedule $1 --mbs $2 --microbatches $3 >> $out 2>> gpurun_out/r6_hbm.err || exit 1
done
MIPIPE_STASH_RING=0 timeout -k 10 150 python tools/hbm_probe.py --schedule 1F1B --mbs 16 --microbatches 8 >> $out 2>> gpurun_out/r6_hbm.err || exit 1
